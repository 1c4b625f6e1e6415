#!/bin/bash
# exact backward: parity tests + timing
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/grad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_exact_grad_gpu.py tests/test_models_gpu.py -k "grad or exact" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -15 $O/tests.log
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-var --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['roofline']['kernel_ms'], d['backward'], d.get('posterior'))"
