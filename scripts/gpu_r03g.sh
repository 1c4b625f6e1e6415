#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/e32/libgpk.so
timeout -k 10 120 python -u scripts/debug_e32.py 256 > $O/debug_e32.txt 2>&1 || { cat $O/debug_e32.txt; exit 1; }
grep -v Warn $O/debug_e32.txt
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py -k "256 or full_size" > $O/tests_e32.log 2>&1 || { tail -30 $O/tests_e32.log; exit 1; }
tail -1 $O/tests_e32.log
for v in pro2 e32; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 120 python bench.py --no-var --no-grad --no-cpu-baseline --no-e2e --no-cfg2 --steps 50 --warmup 10 > $O/bench_$v.json 2> $O/bench_$v.err || { tail $O/bench_$v.err; exit 2; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', 'value', round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3))"
done
