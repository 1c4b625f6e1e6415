#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash scripts/gpu_ab_exact.sh lh0 lh1 lh0 lh1
