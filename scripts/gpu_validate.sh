#!/bin/bash
# Final validation of the in-tree build: GPU tests, smoke, one bench line (outputs under gpurun_out/validate)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/validate; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && tail -n 1 $O/pytest_gpu.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && echo BENCH_OK
