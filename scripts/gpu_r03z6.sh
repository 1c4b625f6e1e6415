#!/bin/bash
# K_ZZ look-ahead variant (the diagonal wave applies the last update of (k+1,k+1) itself):
# parity tests with it, factor + inverse times vs the shipped build, phase clocks
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z6; mkdir -p $O
AB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab
GPK_LIB=$AB/kzz_la/libgpk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "kzz or variational or Kzz" tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 100 python scripts/time_kzz.py || exit 2
GPK_LIB=$AB/kzz_la/libgpk.so timeout -k 10 100 python scripts/time_kzz.py || exit 3
GPK_LIB=$AB/kzz_stamps/libgpk.so timeout -k 10 100 python scripts/kzz_stamps.py 256 32 > $O/kzz_256.txt 2>&1 || { tail $O/kzz_256.txt; exit 4; }
grep -v amdgpu.ids $O/kzz_256.txt
