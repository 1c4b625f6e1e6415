#!/bin/bash
# K_ZZ factor phase clocks (GPK_KZZ_STAMPS build), M = 256 and 64, D = 32
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z4; mkdir -p $O
for m in 256 64; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/kzz_stamps/libgpk.so timeout -k 10 100 python scripts/kzz_stamps.py $m 32 > $O/kzz_$m.txt 2>&1 || { tail $O/kzz_$m.txt; exit 1; }
  grep -v amdgpu.ids $O/kzz_$m.txt
done
