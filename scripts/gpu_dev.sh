#!/bin/bash
# Dev A/B loop for the exact kernel: parity tests + bench + phase timeline of the
# dev build (scripts/ab_build_one.sh dev gpk_exact.hip -DGPK_EXACT_DEV=1).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/dev; mkdir -p $O
export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/dev/libgpk.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py -k "256 or full_size" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python bench.py --no-var --no-grad --no-cpu-baseline --no-e2e --no-cfg2 --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
python -c "import json; d=json.load(open('$O/bench.json')); print('value', round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3))"
timeout -k 10 120 python scripts/stamps_exact.py 512 > $O/tl.txt 2>&1 || { tail $O/tl.txt; exit 3; }
grep -v Warning $O/tl.txt | grep -v "nanmean\|= np.nan"
