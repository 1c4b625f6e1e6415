#!/bin/bash
# per _lib_ab/<name>: exact-kernel parity subset, timing (ko_time), column-plan timeline
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab5; mkdir -p $O
for v in "$@"; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py -k "(parity_small and (256 or 128 or 250)) or full_size or accuracy or cfg2 or layout" -x -q --timeout 120 --timeout-method thread > $O/pt_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 $O/pt_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pt_$v.log)"
  timeout -k 10 150 python scripts/ab/ko_time.py >> $O/ab.jsonl 2> $O/err_$v.log || { echo "$v FAILED"; tail -20 $O/err_$v.log; exit 1; }
  tail -1 $O/ab.jsonl
  timeout -k 10 150 python scripts/r05/stamps_col.py 512 > $O/tl_$v.txt 2>&1 || { echo "$v STAMPS FAILED"; tail -20 $O/tl_$v.txt; exit 2; }
done
