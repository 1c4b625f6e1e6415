#!/bin/bash
# Round-6 diagonal-chain change: exact GPU tests on the new build, then A/B vs the round-5 object.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06diag}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py tests/test_golden_gpu.py tests/test_exact_grad_gpu.py tests/test_posterior_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -n 3 $O/pytest_exact.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_exact.log | head -30; exit $rc; }
LIBS="${LIBS:-base=fine_grained_gaussian_process_forcasting_amd/_lib_ab/base/libgpk.so new=fine_grained_gaussian_process_forcasting_amd/_lib/libgpk.so}" bash scripts/r06/ab_exact.sh
