#!/bin/bash
# round-3 closing numbers: the default bench line (side legs timed by graph replay), then the
# round-3 profile passes (scripts/gpu_r03q.sh: kernel stats + FETCH / WRITE PMC passes)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "\"metric\"" $O/bench.log | tail -n 1 > $O/bench.json
python -c "
import json; d=json.load(open('$O/bench.json')); v=d['variational']
print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])
print('var', v['kernel_ms'], v['eager_ms'], v['roofline']['frac'], v['backward_roofline']['frac'])
print('grad', d['backward'], 'post', d['posterior']['kernel_ms'], d['posterior']['eager_ms'], 'cfg2', d['cfg2']['kernel_ms'], d['cfg2']['eager_ms'])
print('var3', {k: x['kernel_ms'] for k, x in d['variational_cfg3'].items()})"
bash scripts/gpu_r03q.sh
