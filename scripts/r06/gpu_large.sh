#!/bin/bash
# Large-N exact path (256 < N <= 800): parity tests, then the N <= 256 exact / native tests.
set -o pipefail
OUT=gpurun_out/${TAG:-large}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_exact_large_gpu.py -v -s --timeout 200 --timeout-method thread \
  > $OUT/pytest_large.log 2>&1
rc=$?
tail -40 $OUT/pytest_large.log
echo LARGE_RC=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_native_lib.py tests/test_exact_grad_gpu.py tests/test_posterior_gpu.py \
  -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_regress.log 2>&1
rc=$?
tail -5 $OUT/pytest_regress.log
echo REGRESS_RC=$rc
exit $rc
