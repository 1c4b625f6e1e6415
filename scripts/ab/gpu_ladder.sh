#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  echo "== $v"
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 120 python scripts/ab/ladder_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
done
