#!/bin/bash
# scripts/gpu_var_ab.sh <variant>...   (VAR_ARGS="B N M D" selects the shape)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/var_ab; mkdir -p $O
timeout -k 10 120 python scripts/time_var.py $VAR_ARGS > $O/t.txt 2>&1 || { cat $O/t.txt; exit 1; }
for v in "$@"; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 120 python scripts/time_var.py $VAR_ARGS >> $O/t.txt 2>&1 || { cat $O/t.txt; exit 2; }
done
grep ms $O/t.txt
