#!/bin/bash
# like gpu_ab.sh, but first the N=256 exact parity tests against each variant
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
for spec in "$@"; do
  v=${spec%+}
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py -k "256 or full_size or two_windows" > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAIL"; tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
  timeout -k 10 150 python scripts/ab/ko_time.py >> $O/ab.jsonl 2> $O/err_$v.log || { echo "$v FAILED"; tail -20 $O/err_$v.log; exit 1; }
  tail -1 $O/ab.jsonl
  if [ "$spec" != "$v" ]; then
    timeout -k 10 150 python scripts/stamps_exact.py 512 > $O/tl_$v.txt 2>&1 || { echo "$v STAMPS FAILED"; tail -20 $O/tl_$v.txt; exit 2; }
  fi
done
