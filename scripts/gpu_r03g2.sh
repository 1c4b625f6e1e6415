#!/bin/bash
# batched fin-kernel loads + 3-wave forward bound: variational / ELBO / model / graph tests, timing
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03g2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_grad_gpu.py tests/test_variational_gpu.py tests/test_elbo_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 120 python scripts/time_var.py || exit 2
timeout -k 10 120 python scripts/time_var.py 256 192 256 32 || exit 3
timeout -k 10 120 python scripts/time_var.py 256 96 256 32 || exit 4
