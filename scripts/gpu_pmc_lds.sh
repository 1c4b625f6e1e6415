set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/pmclds; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad --no-var"
timeout -s KILL 90 rocprofv3 --pmc LdsLatency --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc LdsUtil --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc LdsBankConflict --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $O/p4 -o run -- $B > $O/p4.log 2>&1 || exit 4
echo done
