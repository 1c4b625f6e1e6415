#!/bin/bash
# A/B of the worker count per window at N=256 (W = 8 / 4 / 6 waves, 2 windows per CU)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash scripts/gpu_ab_exact.sh w8 w4 w6 w8
