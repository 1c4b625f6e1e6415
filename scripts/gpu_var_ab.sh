#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/var_ab; mkdir -p $O
timeout -k 10 120 python scripts/time_var.py > $O/t.txt 2>&1 || { cat $O/t.txt; exit 1; }
for v in "$@"; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 120 python scripts/time_var.py >> $O/t.txt 2>&1 || { cat $O/t.txt; exit 2; }
done
grep ms $O/t.txt
