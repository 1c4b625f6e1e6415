#!/bin/bash
# M > 64 variational adjoint in the register-resident layout (two kernels): parity + cfg-3 legs + trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_grad_gpu.py tests/test_variational_gpu.py tests/test_boundary_gpu.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 200 python scripts/var3_leg.py > $O/var3.json 2> $O/var3.err || { tail -20 $O/var3.err; exit 2; }
cat $O/var3.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o var3 -- python $R/scripts/var3_leg.py > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 3; }
f=$(find $R/$O/prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r, key=lambda x:-float(x['TotalDurationNs']))[:14]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1000,1),'us')"
