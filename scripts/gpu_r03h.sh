#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O
for v in e32h e32f; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py -k "256 or full_size" > $O/tests_$v.log 2>&1 || { echo "$v TESTS FAIL"; tail -30 $O/tests_$v.log; exit 1; }
  timeout -k 10 120 python bench.py --no-var --no-grad --no-cpu-baseline --no-e2e --no-cfg2 --steps 50 --warmup 10 > $O/bench_$v.json 2> $O/bench_$v.err || { tail $O/bench_$v.err; exit 2; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', 'value', round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3))"
  timeout -k 10 120 python -u scripts/stamps_e32.py 512 > $O/tl_$v.txt 2>&1 || { tail $O/tl_$v.txt; exit 3; }
done
grep -v Warn $O/tl_e32h.txt | grep -v nanmean
