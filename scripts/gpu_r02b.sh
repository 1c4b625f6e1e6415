#!/bin/bash
# quick loop: variational GPU tests + kernel stats of bench (no CPU baseline)
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py tests/test_sampler.py > gpurun_out/pytest_var.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profq" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > "$R/gpurun_out/profq.log" 2>&1
echo "rocprof rc=$?"
