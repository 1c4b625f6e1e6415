#!/bin/bash
# Knockout timing of the N > 256 forward (scripts/r06/time_large_ko.py per build).
set -o pipefail
OUT=gpurun_out/${TAG:-largeko}
mkdir -p $OUT
timeout -k 10 120 python -u scripts/r06/time_large_ko.py | tee -a $OUT/ko.log || exit 1
for ko in 1 2 4 8 15; do
  GPK_LIB=fine_grained_gaussian_process_forcasting_amd/_lib_ab/ko$ko/libgpk.so \
    timeout -k 10 120 python -u scripts/r06/time_large_ko.py | tee -a $OUT/ko.log || exit 1
done
