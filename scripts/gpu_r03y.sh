#!/bin/bash
# fused ELBO (gpk::variational_elbo): ELBO / graph / boundary / e2e / model tests, then the cfg-3 step
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_elbo_gpu.py tests/test_graphs_gpu.py tests/test_boundary_gpu.py tests/test_e2e_gpu.py tests/test_models_gpu.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 1 $O/quick.log
timeout -k 10 400 python scripts/gp_step.py cfg3 20 > $O/gp_step.json 2> $O/gp_step.err || { tail -20 $O/gp_step.err; exit 2; }
python -c "
import json; d=json.load(open('$O/gp_step.json'))
print({m:{k:(v if not isinstance(v,dict) else round(v['ms_per_step'],3)) for k,v in d[m].items()} for m in ('eager','graph','eager_anomaly')})"
timeout -k 10 400 python scripts/gp_step.py cfg1 20 > $O/gp_step_cfg1.json 2> $O/gp_step_cfg1.err || { tail -20 $O/gp_step_cfg1.err; exit 3; }
python -c "
import json; d=json.load(open('$O/gp_step_cfg1.json'))
print('cfg1', {m:{k:(v if not isinstance(v,dict) else round(v['ms_per_step'],3)) for k,v in d[m].items()} for m in ('eager','graph','eager_anomaly')})"
echo DONE
