set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && cat gpurun_out/bench1.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_exact -o run -- python $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof1.log 2>&1 && echo PROF_OK
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc1.log 2>&1 && echo PMC1_OK
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc2.log 2>&1 && echo PMC2_OK
