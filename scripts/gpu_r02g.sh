#!/bin/bash
# exact-GP posterior + golden-fixture GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/r02g
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_posterior_gpu.py tests/test_golden_gpu.py > gpurun_out/r02g/tests.log 2>&1 || { tail -60 gpurun_out/r02g/tests.log; exit 1; }
tail -25 gpurun_out/r02g/tests.log
