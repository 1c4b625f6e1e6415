#!/bin/bash
# Round 3 first call: diag-sweep microbenchmark + baseline GPU suite + bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03; mkdir -p $O
timeout -k 10 120 ./scripts/microbench/mb_diag > $O/mb_diag.txt 2>&1 || { cat $O/mb_diag.txt; exit 1; }
cat $O/mb_diag.txt
bash scripts/gpu_check.sh
