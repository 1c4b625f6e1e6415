#!/bin/bash
# cfg-3 step timing with untimed graph warm-up replays (eager / graph / anomaly), 20 steps
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 400 python scripts/gp_step.py cfg3 20 > $O/gp_step.json 2> $O/gp_step.err || { tail -20 $O/gp_step.err; exit 2; }
python -c "
import json; d=json.load(open('$O/gp_step.json'))
print({m:{k:(v if not isinstance(v,dict) else round(v['ms_per_step'],3)) for k,v in d[m].items()} for m in ('eager','graph','eager_anomaly')})"
echo DONE
