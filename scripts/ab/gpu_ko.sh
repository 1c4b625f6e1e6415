#!/bin/bash
# time every _lib_ab/<name> given on the command line (one process each)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ko; mkdir -p $O
for v in "$@"; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 150 python scripts/ab/ko_time.py >> $O/ko.jsonl 2> $O/err_$v.log || { echo "$v FAILED"; tail -20 $O/err_$v.log; exit 1; }
  tail -1 $O/ko.jsonl
done
