#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profv" -o run -- python3 "$R/scripts/var_kernels.py" 3 all > "$R/gpurun_out/profv.log" 2>&1
