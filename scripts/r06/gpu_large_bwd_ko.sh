#!/bin/bash
# Knockout timing of the N > 256 backward (scripts/r06/time_large_bwd_ko.py per build).
set -o pipefail
OUT=gpurun_out/${TAG:-lgbwdko}
mkdir -p $OUT
timeout -k 10 120 python -u scripts/r06/time_large_bwd_ko.py | tee -a $OUT/ko.log || exit 1
for ko in 1 2 4; do
  GPK_LIB=fine_grained_gaussian_process_forcasting_amd/_lib_ab/gko$ko/libgpk.so \
    timeout -k 10 120 python -u scripts/r06/time_large_bwd_ko.py | tee -a $OUT/ko.log || exit 1
done
