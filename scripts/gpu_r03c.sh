#!/bin/bash
# Round 3: DPP diag microbench + exact-kernel A/B: base (readlane) / dpp / pro (+fast prologue) / flow (+dataflow workers)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03; mkdir -p $O
timeout -k 10 120 ./scripts/microbench/mb_diag > $O/mb_diag2.txt 2>&1 || { cat $O/mb_diag2.txt; exit 1; }
grep "hog=none\|same-simd\|diff" $O/mb_diag2.txt
bash scripts/gpu_ab_exact.sh base dpp pro flow
