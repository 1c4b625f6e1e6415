# DIAG_ALONE small-batch layout (gpk_exact_dev.h): exact parity tests on a build with the layout
# forced for every NB (_lib_ab/alonefull), then timing A/B of the fast-compile builds.
set -o pipefail
P=fine_grained_gaussian_process_forcasting_amd/_lib_ab
mkdir -p gpurun_out/alone
GPK_LIB=$GRAFT_REPO_ROOT/$P/alonefull/libgpk.so timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py tests/test_golden_gpu.py tests/test_exact_grad_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/alone/pytest_alonefull.log 2>&1 && tail -n 3 gpurun_out/alone/pytest_alonefull.log
