#!/bin/bash
# round-2 artifacts: full GPU tests, bench line, rocprof kernel stats, HBM counters
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r02; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o bench -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --no-e2e > "$R/$O/prof.log" 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch" -o bench -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > "$R/$O/pmc_fetch.log" 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write" -o bench -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > "$R/$O/pmc_write.log" 2>&1 || exit 6
echo ok
