#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d "$R/gpurun_out/trs" -o step -- python3 "$R/scripts/gp_step.py" cfg1 10 > "$R/gpurun_out/trs.log" 2>&1
