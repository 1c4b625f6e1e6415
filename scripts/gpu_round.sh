# Full GPU check: parity tests, smoke, bench (with CPU baseline), rocprofv3 kernel stats,
# separate FETCH_SIZE / WRITE_SIZE PMC passes. Every GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_exact -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-variants > $R/gpurun_out/prof1.log 2>&1 && echo PROF_OK &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-variants > $R/gpurun_out/pmc1.log 2>&1 && echo PMC1_OK &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-variants > $R/gpurun_out/pmc2.log 2>&1 && echo PMC2_OK &&
cd $R && if [ -n "$GPK_AB" ]; then bash scripts/ab/gpu_ab.sh $GPK_AB; fi
