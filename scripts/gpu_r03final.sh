#!/bin/bash
# round-3 final: full GPU suite, smoke(), default bench line, cfg-3 / cfg-1 train steps,
# round-3 profile passes (gpu_r03q.sh), then K_ZZ phase clocks (diagnostic, last)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep "\"metric\"" $O/bench.log | tail -n 1 > $O/bench.json
python -c "
import json; d=json.load(open('$O/bench.json')); v=d['variational']
print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])
print('var', v['kernel_ms'], v['roofline']['frac'], v['backward_roofline']['frac'])
print('var3', {k: x['kernel_ms'] for k, x in d['variational_cfg3'].items()})
print('e2e', {k: d['e2e_step'].get(k) for k in ('eager', 'graph')})"
timeout -k 10 300 python scripts/gp_step.py cfg3 20 > $O/gp_step_cfg3.json 2> $O/gp_step_cfg3.err || { tail -20 $O/gp_step_cfg3.err; exit 4; }
timeout -k 10 300 python scripts/gp_step.py cfg1 20 > $O/gp_step_cfg1.json 2> $O/gp_step_cfg1.err || { tail -20 $O/gp_step_cfg1.err; exit 5; }
python -c "
import json
for c in ('cfg3', 'cfg1'):
    d = json.load(open('$O/gp_step_' + c + '.json'))
    print(c, {m: {k: (v if not isinstance(v, dict) else round(v['ms_per_step'], 3)) for k, v in d[m].items()} for m in ('eager', 'graph', 'eager_anomaly')})"
bash scripts/gpu_r03q.sh || exit 6
GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/kzz_stamps/libgpk.so timeout -k 10 100 python scripts/kzz_stamps.py 256 32 > $O/kzz_stamps_256.txt 2>&1; tail -n 25 $O/kzz_stamps_256.txt
echo DONE
