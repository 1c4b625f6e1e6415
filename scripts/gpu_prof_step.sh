#!/bin/bash
# rocprofv3 kernel stats of the graphed cfg3 GP training step (scripts/gp_step.py cfg3 N graph-gp)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profstep" -o step -- python3 "$R/scripts/gp_step.py" ${1:-cfg3} 20 graph-gp > "$R/gpurun_out/profstep.log" 2>&1 || exit 1
tail -n 2 "$R/gpurun_out/profstep.log"
