#!/bin/bash
# K_ZZ inverse A/B: gpk_kzz_inv_nt_kernel (default build) vs gpk_kzz_inv_kernel
# (_lib_ab/invold, -DGPK_KZZ_INV_NT=0), alternating child processes, then the K_ZZ parity tests
# and a rocprofv3 kernel-stats pass of scripts/time_kzz.py on the default build.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-kzzinv}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && tail -n 2 $O/pytest.log &&
for i in 1 2 3; do
  echo "== new $i" >> $O/ab.txt && timeout -k 10 120 python scripts/time_kzz.py >> $O/ab.txt 2>&1 &&
  echo "== old $i" >> $O/ab.txt && GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/invold/libgpk.so timeout -k 10 120 python scripts/time_kzz.py >> $O/ab.txt 2>&1 || exit 3
done && cat $O/ab.txt | grep -v amdgpu.ids &&
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kzz -- python3 $R/scripts/time_kzz.py > $O/prof.log 2>&1 && echo PROF_OK
