#!/bin/bash
# Full GPU test suite + one bench line of the in-tree build.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/check; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -n 1 $O/gputests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
python -c "import json; d=json.load(open('$O/bench.json')); print('value', round(d['value']), 'kernel_ms', round(d['roofline']['kernel_ms'], 4), 'frac', round(d['roofline']['frac'], 3)); print(d['variational']['kernel_ms']); print(d['backward']['kernel_ms']); e=d.get('e2e_step',{}); print('e2e', {k: (v.get('gp',{}).get('ms_per_step'), v.get('gp_share_ms')) if isinstance(v, dict) else v for k, v in e.items()})"
