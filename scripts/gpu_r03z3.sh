#!/bin/bash
# K_ZZ inverse on 16 waves: K_ZZ / variational parity tests, then scripts/time_kzz.py
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "kzz or variational or Kzz" tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python scripts/time_kzz.py > $O/time_kzz.txt 2>&1 || { tail -20 $O/time_kzz.txt; exit 2; }
cat $O/time_kzz.txt
