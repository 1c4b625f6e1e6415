#!/bin/bash
# A/B of the variational kernels (cfg 5 and the cfg-3 M=256 shape, scripts/time_var.py):
#   adjpf   gpk_var_adj_r_kernel chunk prefetch + batched fin loads + unrolled partial sums
#   finonly batched fin loads only
#   fwdpf3 / fwdpf2  gpk_var_fwd_r_kernel chunk prefetch at 3 / 2 waves per SIMD (+ adjpf's)
# parity tests with each variant first
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab_adj; mkdir -p $O
for v in adjpf finonly fwdpf3 fwdpf2; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_grad_gpu.py tests/test_variational_gpu.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/tests_$v.log)"
done
for i in 1 2; do
  for v in base adjpf finonly fwdpf3 fwdpf2; do
    L=""; [ $v != base ] && L=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
    GPK_LIB=$L timeout -k 10 120 python scripts/time_var.py || exit 2
    GPK_LIB=$L timeout -k 10 120 python scripts/time_var.py 256 192 256 32 || exit 3
  done
done
