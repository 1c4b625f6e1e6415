#!/bin/bash
# pipelined K_ZZ trailing update: K_ZZ parity + timing + stamps, then the round-3 profiles
# (scripts/gpu_r03q.sh: kernel stats + FETCH / WRITE passes of bench.py and of the cfg-3 legs)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03u; mkdir -p $O
export TMPDIR=/tmp
P=fine_grained_gaussian_process_forcasting_amd/_lib_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_graphs_gpu.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 1 $O/quick.log
timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_main.txt 2>&1 || { tail -20 $O/kzz_main.txt; exit 2; }
cat $O/kzz_main.txt
GPK_LIB=$P/kzz_stamps/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 256 32 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 3; }
tail -n 1 $O/stamps.txt
bash scripts/gpu_r03q.sh || exit 4
echo DONE
