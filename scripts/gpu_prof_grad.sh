#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp; export TMPDIR=/tmp; O=$R/gpurun_out/prof_grad; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o grad -- python3 $R/scripts/time_grad.py > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/grad_kernel_stats.csv")):
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e3, 1))
PY
