#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py > gpurun_out/pytest_var.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/var_kernels.py 5 all > gpurun_out/var_times.log 2>&1
