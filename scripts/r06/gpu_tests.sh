#!/bin/bash
# Round-6 GPU check: the full GPU suite (new layout / ladder / prior-covariance / N=256 grad
# cases included), smoke, and a short headline bench without the CPU / e2e legs.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06a}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 4 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 300 python bench.py --no-e2e --cpu-seconds 4 > $O/bench.json 2> $O/bench.err && echo BENCH_OK && python - <<'PY'
import json,os
d=json.load(open(os.path.join(os.environ["GRAFT_REPO_ROOT"],"gpurun_out",os.environ.get("TAG","r06a"),"bench.json")))
print("value",d["value"],"frac",d["roofline"]["frac"],"kms",d["roofline"]["kernel_ms"])
print("cpu",json.dumps(d.get("cpu_baseline"))[:800])
PY
