#!/bin/bash
# K_ZZ sweep with the 3-level Newton step (kzz_nt) vs the shipped build: parity tests, times
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z7; mkdir -p $O
AB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab
GPK_LIB=$AB/kzz_nt/libgpk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "kzz or variational or Kzz" tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for i in 1 2; do
  timeout -k 10 100 python scripts/time_kzz.py || exit 2
  GPK_LIB=$AB/kzz_nt/libgpk.so timeout -k 10 100 python scripts/time_kzz.py || exit 3
done
