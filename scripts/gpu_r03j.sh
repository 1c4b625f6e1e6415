#!/bin/bash
# A/B of the loaded {lo,hi} trailing operand; full GPU suite; the multi-process (RCCL) bench path
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03; mkdir -p $O
bash scripts/gpu_ab_exact.sh lh1 lh0 lh1 || exit 1
unset GPK_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 2; }
tail -n 1 $O/gputests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-var --no-grad --no-cpu-baseline --no-e2e > $O/torchrun1.json 2> $O/torchrun1.err || { tail -20 $O/torchrun1.err; exit 3; }
python -c "import json; d=json.load(open('$O/torchrun1.json')); print('torchrun n=1', d['n_gpus'], round(d['value']), d['roofline']['kernel_ms'], d.get('strong_share'))"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --strong --steps 20 --warmup 5 --no-var --no-grad --no-cpu-baseline --no-e2e > $O/torchrun1s.json 2> $O/torchrun1s.err || { tail -20 $O/torchrun1s.err; exit 4; }
python -c "import json; d=json.load(open('$O/torchrun1s.json')); print('torchrun strong n=1', d['scaling'], round(d['value']))"
