#!/bin/bash
# round-3 profiles: rocprofv3 kernel stats of bench.py, separate FETCH_SIZE / WRITE_SIZE PMC
# passes of bench.py (exact forward / backward / posterior, cfg-5 variational) and of the
# cfg-3 variational legs (scripts/var3_leg.py); each pass its own run and time limit
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=$R/gpurun_out/r03q; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
BARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-var3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py $BARGS > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep "\"metric\"" $O/prof.log | tail -n 1 > $O/bench.json
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o bench -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-var3 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o bench -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-var3 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_var3 -o var3 -- python3 $R/scripts/var3_leg.py > $O/prof_var3.log 2>&1 || { tail -20 $O/prof_var3.log; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_var3 -o var3 -- python3 $R/scripts/var3_leg.py > $O/pmc3.log 2>&1 || { tail -20 $O/pmc3.log; exit 5; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_var3 -o var3 -- python3 $R/scripts/var3_leg.py > $O/pmc4.log 2>&1 || { tail -20 $O/pmc4.log; exit 6; }
echo DONE
