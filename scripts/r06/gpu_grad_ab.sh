#!/bin/bash
# Exact backward: parity tests on the product (fused) build, then alternating A/B timing.
set -o pipefail
OUT=gpurun_out/${TAG:-gradab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_exact_grad_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py \
  -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_grad.log 2>&1 || { tail -30 $OUT/pytest_grad.log; exit 1; }
tail -2 $OUT/pytest_grad.log
for rep in 1 2 3; do
  timeout -k 10 120 python -u scripts/r06/time_grad.py | tee -a $OUT/ab.log || exit 1
  GPK_LIB=fine_grained_gaussian_process_forcasting_amd/_lib_ab/nofuse/libgpk.so \
    timeout -k 10 120 python -u scripts/r06/time_grad.py | tee -a $OUT/ab.log || exit 1
done
