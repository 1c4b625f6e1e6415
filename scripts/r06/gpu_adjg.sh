#!/bin/bash
# Round-6 one-pass saved-state adjoint (gpk_var_adjg_l_kernel): variational gradient + e2e tests on
# the A/B build, then adjoint time A/B (base = current _lib, adjg = the new build), alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06adjg}; mkdir -p $O
NEW=${NEW:-fine_grained_gaussian_process_forcasting_amd/_lib_ab/adjg/libgpk.so}
BASE=${BASE:-fine_grained_gaussian_process_forcasting_amd/_lib/libgpk.so}
GPK_LIB=$R/$NEW timeout -k 10 400 python -u -m pytest tests/test_variational_grad_gpu.py tests/test_e2e_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -n 3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2 3; do for n in 192 96; do for nl in base=$BASE new=$NEW; do
  name=${nl%%=*}; lib=${nl#*=}
  o=$(GPK_LIB=$R/$lib timeout -k 10 120 python scripts/r06/time_var_saved.py 256 $n 256 32 2>/dev/null | tail -n 1) || { echo FAIL $name; exit 3; }
  echo "$rep $name N=$n $o" | tee -a $O/ab.txt
done; done; done
# the product exact kernel after the round-6 diagonal-wave change
timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py tests/test_golden_gpu.py tests/test_posterior_gpu.py tests/test_exact_grad_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_exact.log 2>&1; rc=$?
tail -n 2 $O/pytest_exact.log
exit $rc
