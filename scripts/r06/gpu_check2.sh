#!/bin/bash
# Round-6 check: the full GPU suite on the product build, then adjoint A/B (cfg 5 register path:
# fp64 vs fp32 dK; cfg-3 saved-state: round-5 fp64 adjs vs the product).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06c2}; mkdir -p $O
A=fine_grained_gaussian_process_forcasting_amd/_lib_ab
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -30; exit $rc; }
for rep in 1 2 3; do for nl in dk64=$A/dk64/libgpk.so prod=fine_grained_gaussian_process_forcasting_amd/_lib/libgpk.so; do
  name=${nl%%=*}; lib=${nl#*=}
  o=$(GPK_LIB=$R/$lib timeout -k 10 120 python scripts/time_var.py 1024 256 64 32 2>/dev/null | tail -n 1) || exit 3
  echo "$rep $name $o" | tee -a $O/ab_cfg5.txt
done; done
TAG=${TAG:-r06c2} NS="192 96" REPS=2 LIBS="m0=$A/adj_m0/libgpk.so prod=fine_grained_gaussian_process_forcasting_amd/_lib/libgpk.so" bash scripts/r06/ab_var.sh
