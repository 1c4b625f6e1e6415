#!/bin/bash
# exact-backward A/B with parity: tests/test_exact_grad_gpu.py, then time_grad.py, per _lib_ab/<v>
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
for v in "$@"; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_exact_grad_gpu.py > $O/gtests_$v.log 2>&1 || { echo "$v TESTS FAIL"; grep -v "^$" $O/gtests_$v.log | tail -30; exit 1; }
  grep "hip " $O/gtests_$v.log | grep "noise=\|N=256" | head -14; tail -1 $O/gtests_$v.log
  timeout -k 10 120 python scripts/time_grad.py >> $O/grad_ab.txt 2>> $O/grad_err.log || { echo "$v FAILED"; tail -20 $O/grad_err.log; exit 1; }
  tail -1 $O/grad_ab.txt
done
