#!/bin/bash
# HIP-graph step: GPU tests, then the cfg3 / cfg1 end-to-end step (eager vs graphed).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/graphs; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_graphs_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log
timeout -k 10 300 python scripts/gp_step.py cfg3 20 > $O/cfg3.json 2> $O/cfg3.err || { tail -30 $O/cfg3.err; exit 2; }
cat $O/cfg3.json
timeout -k 10 300 python scripts/gp_step.py cfg1 20 > $O/cfg1.json 2> $O/cfg1.err || { tail -30 $O/cfg1.err; exit 3; }
cat $O/cfg1.json
