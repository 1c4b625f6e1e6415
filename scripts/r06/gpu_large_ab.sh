#!/bin/bash
# Large-N parity tests on the product build, then forward timing of the product and A/B builds.
set -o pipefail
OUT=gpurun_out/${TAG:-largeab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_exact_large_gpu.py -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_large.log 2>&1 || { tail -30 $OUT/pytest_large.log; exit 1; }
tail -2 $OUT/pytest_large.log
timeout -k 10 120 python -u scripts/r06/time_large_ko.py | tee -a $OUT/ab.log || exit 1
for v in $AB; do
  GPK_LIB=fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so \
    timeout -k 10 120 python -u scripts/r06/time_large_ko.py | tee -a $OUT/ab.log || exit 1
done
