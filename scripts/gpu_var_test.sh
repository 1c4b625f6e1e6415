#!/bin/bash
# variational parity tests + timing
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/var_test; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_golden_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python scripts/time_var.py && timeout -k 10 120 python scripts/time_var.py 256 192 256 32 && timeout -k 10 120 python scripts/time_var.py 256 96 64 16
