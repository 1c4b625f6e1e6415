#!/bin/bash
# the RCCL path under torchrun at world size 1: weak (default) and --strong bench lines
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03s2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --strong --steps 30 --warmup 5 --no-var --no-var3 --no-e2e --no-cpu-baseline --no-grad > $O/strong.log 2>&1 || { tail -20 $O/strong.log; exit 1; }
grep "\"metric\"" $O/strong.log | tail -n 1 > $O/strong.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 30 --warmup 5 --no-var --no-var3 --no-e2e --no-cpu-baseline --no-grad > $O/weak.log 2>&1 || { tail -20 $O/weak.log; exit 2; }
grep "\"metric\"" $O/weak.log | tail -n 1 > $O/weak.json
python -c "
import json
for n in ('strong', 'weak'):
    d = json.load(open('$O/' + n + '.json'))
    print(n, d['value'], d['scaling'], d['config']['process_group'], d['roofline']['kernel_ms'])"
