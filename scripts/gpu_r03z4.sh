#!/bin/bash
# K_ZZ factor phase clocks: DPP sweep (kzz_stamps) vs readlane sweep (kzz_rl), M = 256 and 64
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z4; mkdir -p $O
for v in kzz_stamps kzz_rl; do
  for m in 256 64; do
    GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 100 python scripts/kzz_stamps.py $m > $O/${v}_$m.txt 2>&1 || { tail $O/${v}_$m.txt; exit 1; }
    echo "== $v M=$m"; grep -v amdgpu.ids $O/${v}_$m.txt
  done
done
