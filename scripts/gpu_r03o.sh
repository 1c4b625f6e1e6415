#!/bin/bash
# round-3 state at HEAD + K_ZZ adjoint kernel: GPU tests, smoke, bench, graphed cfg-3 step
# kernel stats with and without the GP branch (the GP share's kernel breakdown)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cat $O/bench.json
cd /tmp
for kind in graph-gp graph-nogp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/step_$kind -o step -- python3 $R/scripts/gp_step.py cfg3 20 $kind > $R/$O/step_$kind.log 2>&1 || { tail -20 $R/$O/step_$kind.log; exit 4; }
done
echo DONE
