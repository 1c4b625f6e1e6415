#!/bin/bash
# exact-kernel change check: exact parity tests, the headline timing, the per-step timeline
R="$GRAFT_REPO_ROOT"; cd "$R"; export TMPDIR=/tmp; O=$R/gpurun_out/${TAG:-ho1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_golden_gpu.py tests/test_exact_grad_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; rc=$?
tail -n 2 $O/pt.log; grep -E "FAILED|Error" $O/pt.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python scripts/r05/stamps_col.py 512 > $O/stamps_col.txt 2>&1 || exit 4
P=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab
for i in 1 2 3; do for v in base new; do
  echo "$v $(GPK_LIB=$P/$v/libgpk.so timeout -k 10 60 python scripts/time_exact.py 512 256 32 100 2>/dev/null | tail -1) $(GPK_LIB=$P/$v/libgpk.so timeout -k 10 60 python scripts/time_exact.py 128 128 32 200 2>/dev/null | tail -1)" >> $O/ab.txt || exit 5
done; done; cat $O/ab.txt
