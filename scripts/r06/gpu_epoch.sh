#!/bin/bash
# Round-6 item: the exact kernel's hand-over protocol under the GPK_EPOCH_CHECK build (every
# consumed panel / hand-over / R_kk^{-T} tile checked against the epoch its consumer expects):
# the full exact suite on the check build, then the sabotage build (GPK_EPOCH_CHECK=2) must
# flag every window.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06epoch}; mkdir -p $O
L=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab
GPK_LIB=$L/epoch1/libgpk.so timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_golden_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_epoch1.log 2>&1; rc=$?
tail -n 3 $O/pytest_epoch1.log
[ $rc -eq 0 ] || exit $rc
GPK_LIB=$L/epoch2/libgpk.so timeout -k 10 120 python scripts/r06/epoch_negative.py > $O/negative.log 2>&1; rc=$?
cat $O/negative.log | tail -3
exit $rc
