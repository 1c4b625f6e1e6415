#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab
bash scripts/gpu_ab_exact.sh pro pro2 f16 flowf16 || exit 1
for v in pro sb; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 120 python bench.py --B 64 --no-var --no-grad --no-cpu-baseline --no-e2e --no-cfg2 --steps 50 --warmup 10 > $O/bench64_$v.json 2> $O/bench64_$v.err || { tail $O/bench64_$v.err; exit 2; }
  python -c "import json; d=json.load(open('$O/bench64_$v.json')); print('$v B=64', 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3))"
done
