set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/pmc; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad --no-var > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad --no-var > $O/p2.log 2>&1 || exit 2
echo done
