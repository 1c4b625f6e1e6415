#!/bin/bash
# exact-backward A/B: time_grad.py against each _lib_ab/<v>/libgpk.so (knockout builds: timing only)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 120 python scripts/time_grad.py >> $O/grad_ab.txt 2>> $O/grad_err.log || { echo "$v FAILED"; tail -20 $O/grad_err.log; exit 1; }
  tail -1 $O/grad_ab.txt
done
