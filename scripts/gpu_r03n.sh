#!/bin/bash
# fixed-order parallel column means (all variational kernels): parity + cfg-3 / cfg-5 legs + trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_grad_gpu.py tests/test_variational_gpu.py tests/test_boundary_gpu.py tests/test_e2e_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
timeout -k 10 200 python scripts/var3_leg.py > $O/var3.json 2> $O/var3.err || { tail -20 $O/var3.err; exit 2; }
cat $O/var3.json
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad --no-var3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python -c "import json; d=json.load(open('$O/bench.json'))['variational']; print('cfg5', d['kernel_ms'], round(d['roofline']['frac'],3), round(d['backward_roofline']['frac'],3))"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o var3 -- python $R/scripts/var3_leg.py > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 4; }
f=$(find $R/$O/prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r, key=lambda x:-float(x['TotalDurationNs']))[:12]: print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1000,1),'us')"
