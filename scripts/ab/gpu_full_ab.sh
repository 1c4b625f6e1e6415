#!/bin/bash
# full GPU suite on the production library, then interleaved A/B timing: gpu_full_ab.sh "v1 v2 v1 v2"
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/full_tests.log 2>&1 || { echo "FULL TESTS FAIL"; tail -40 $O/full_tests.log; exit 1; }
tail -2 $O/full_tests.log
bash scripts/ab/gpu_abt.sh $1
