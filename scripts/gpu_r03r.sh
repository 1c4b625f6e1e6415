#!/bin/bash
# K_ZZ factor A/B (waves per workgroup, stamps) + the reworked K_ZZ adjoint kernels:
# targeted parity, timings of each variant, per-step phase clocks
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03r; mkdir -p $O
export TMPDIR=/tmp
P=fine_grained_gaussian_process_forcasting_amd/_lib_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_elbo_gpu.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 2 $O/quick.log
timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_main.txt 2>&1 || { tail -20 $O/kzz_main.txt; exit 2; }
cat $O/kzz_main.txt
for v in w12 w16; do
  GPK_LIB=$P/kzz_$v/libgpk.so timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_$v.txt 2>&1 || { tail -20 $O/kzz_$v.txt; exit 3; }
  echo "== $v"; head -2 $O/kzz_$v.txt
done
GPK_LIB=$P/kzz_stamps/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 256 32 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 4; }
cat $O/stamps.txt
GPK_LIB=$P/kzz_stamps/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 64 32 > $O/stamps64.txt 2>&1 || { tail -20 $O/stamps64.txt; exit 5; }
cat $O/stamps64.txt
echo DONE
