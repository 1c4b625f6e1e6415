#!/bin/bash
# Round-6 end-of-round GPU evidence in one call (outputs under gpurun_out/$TAG): parity tests,
# smoke, bench line, rocprofv3 kernel stats of the bench, separate FETCH_SIZE / WRITE_SIZE
# passes, the cfg-3 variational legs (N = 192, 96) with their own PMC passes, the graphed cfg-3
# train step, the exact kernel's phase clocks and per-step timeline, and the K_ZZ factor's
# stamps. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
T=${TAG:-r06final}; O=$R/gpurun_out/$T; mkdir -p $O
P="--no-cpu-baseline --no-e2e --no-variants"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && tail -n 2 $O/pytest_gpu.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err && echo BENCH_OK &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 30 --warmup 5 $P > $O/prof.log 2>&1 && echo PROF_OK &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o bench -- python3 $R/bench.py --steps 10 --warmup 2 $P > $O/pmc1.log 2>&1 && echo PMC1_OK &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o bench -- python3 $R/bench.py --steps 10 --warmup 2 $P > $O/pmc2.log 2>&1 && echo PMC2_OK &&
for n in 192 96; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_var3_$n -o var3 -- python3 $R/scripts/var3_leg.py $n > $O/var3_$n.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_var3_$n -o var3 -- python3 $R/scripts/var3_leg.py $n > $O/pmcv1_$n.log 2>&1 &&
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_var3_$n -o var3 -- python3 $R/scripts/var3_leg.py $n > $O/pmcv2_$n.log 2>&1 || exit 3
done && echo VAR3_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step_graph-gp -o step -- python3 $R/scripts/gp_step.py cfg3 23 graph-gp > $O/step_graph-gp.log 2>&1 && echo STEP_OK &&
cd $R && timeout -k 10 150 python scripts/stamps_exact.py 512 > $O/stamps.txt 2>&1 &&
timeout -k 10 150 python scripts/r05/stamps_col.py 512 > $O/stamps_col.txt 2>&1 && echo STAMPS_OK
