#!/bin/bash
# variational adjoint parity (recompute + saved paths) and the cfg-3 legs with kernel stats
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; export TMPDIR=/tmp; O=$R/gpurun_out/${TAG:-var5}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_variational_grad_gpu.py tests/test_variational_gpu.py tests/test_native_lib.py -x -q -s --timeout 120 --timeout-method thread > $O/pt_var.log 2>&1; rc=$?
tail -n 3 $O/pt_var.log; grep -E "FAILED|Error|assert" $O/pt_var.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/var3_leg.py > $O/var3.json 2> $O/var3.err && cat $O/var3.json &&
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_var3_192 -o var3 -- python3 $R/scripts/var3_leg.py 192 > $O/prof192.log 2>&1 && echo PROF_OK
