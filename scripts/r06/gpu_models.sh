#!/bin/bash
# Round-6: the model-surface GPU tests (multi-output layers, variational covariance / rsample).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06m}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_models.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_models.log | tail -30
[ $rc -eq 0 ] || { grep -B 30 -E "^E " $O/pytest_models.log | head -80; exit $rc; }
