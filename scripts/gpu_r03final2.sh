#!/bin/bash
# final validation of the shipped build (gpu_r03final.sh), then the worker-priority level A/B
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash scripts/gpu_r03final.sh || exit 1
bash scripts/gpu_ab_prio.sh prio1 prio2 prio1 prio2 || exit 2
