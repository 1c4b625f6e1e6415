#!/bin/bash
# ladder debug for the given debug variants, then tests + timing for the others: gpu_combo.sh "dbg1 dbg2" "v1+ v2"
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash scripts/ab/gpu_ladder.sh $1 || exit 1
bash scripts/ab/gpu_abt.sh $2
