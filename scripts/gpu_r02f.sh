#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/r02
bash scripts/gpu_r02d.sh || exit 1
timeout -k 10 300 python scripts/gp_step.py cfg3 20 > gpurun_out/r02/gp_step_cfg3.json 2>/dev/null || exit 2
timeout -k 10 300 python scripts/gp_step.py cfg1 20 > gpurun_out/r02/gp_step_cfg1.json 2>/dev/null || exit 3
bash scripts/gpu_prof_var.sh
