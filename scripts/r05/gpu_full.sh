#!/bin/bash
# full GPU suite + smoke + e2e step leg (eager / graph) with kernel stats of the graphed step
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; export TMPDIR=/tmp; O=$R/gpurun_out/${TAG:-full5}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 2 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python scripts/gp_step.py cfg3 20 > $O/step.json 2> $O/step.err && tail -c 1500 $O/step.json &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_graph_gp -o step -- python3 $R/scripts/gp_step.py cfg3 23 graph-gp > $O/stepprof.log 2>&1 && echo STEPPROF_OK
