#!/bin/bash
# A/B of exact-kernel builds (worker issue priority, GPK_EXACT_PRIO) (_lib_ab/<name>): N=256 / N=128 parity tests, then the headline,
# cfg-2 and strong-share timings of bench.py
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab_prio; mkdir -p $O
for v in "$@"; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAIL"; tail -30 $O/tests_$v.log; exit 1; }
  tail -n 1 $O/tests_$v.log
  timeout -k 10 200 python bench.py --no-var --no-var3 --no-grad --no-cpu-baseline --no-e2e --steps 50 --warmup 10 > $O/bench_$v.json 2> $O/bench_$v.err || { tail $O/bench_$v.err; exit 2; }
  python -c "
import json; d=json.load(open('$O/bench_$v.json'))
print('$v', 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3),
      'cfg2', round(d['cfg2']['kernel_ms'], 4), round(d['cfg2']['hbm_frac'], 3),
      'strong', {k: round(v['kernel_ms'], 4) for k, v in d['strong_share'].items() if k.startswith('G')})"
done
