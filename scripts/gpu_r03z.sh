#!/bin/bash
# round-3 closing check: full GPU test suite, smoke(), the default bench line, and the
# exact-kernel phase clocks (scripts/stamps_exact.py); each step under its own limit
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep "\"metric\"" $O/bench.log | tail -n 1 > $O/bench.json
python -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['cpu_baseline'])"
timeout -k 10 200 python scripts/stamps_exact.py 512 > $O/stamps_exact.txt 2>&1 || { tail -20 $O/stamps_exact.txt; exit 4; }
head -n 30 $O/stamps_exact.txt
echo DONE
