#!/bin/bash
# artifacts for profiles/: GP step timings, bench line, rocprof kernel stats, HBM counters
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/r02
timeout -k 10 300 python scripts/gp_step.py cfg3 20 > gpurun_out/r02/gp_step_cfg3.json 2> gpurun_out/r02/gp_step_cfg3.err || exit 1
timeout -k 10 300 python scripts/gp_step.py cfg1 20 > gpurun_out/r02/gp_step_cfg1.json 2> gpurun_out/r02/gp_step_cfg1.err || exit 2
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err || exit 3
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r02/prof" -o bench -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --no-e2e > "$R/gpurun_out/r02/prof.log" 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r02/pmc_fetch" -o bench -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > "$R/gpurun_out/r02/pmc_fetch.log" 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/r02/pmc_write" -o bench -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > "$R/gpurun_out/r02/pmc_write.log" 2>&1 || exit 6
echo ok
