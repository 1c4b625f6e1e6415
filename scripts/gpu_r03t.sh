#!/bin/bash
# diagonal-wave K_ZZ factor (A/B: waves, stamps), ring-buffered graph verdicts, fused enc/dec
# GP call: targeted parity, K_ZZ timings, then kernel stats of the variational legs and the
# graphed cfg-3 step with / without the GP branch
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03t; mkdir -p $O
export TMPDIR=/tmp
P=fine_grained_gaussian_process_forcasting_amd/_lib_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_elbo_gpu.py tests/test_graphs_gpu.py tests/test_boundary_gpu.py tests/test_models_gpu.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 2 $O/quick.log
timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_main.txt 2>&1 || { tail -20 $O/kzz_main.txt; exit 2; }
cat $O/kzz_main.txt
GPK_LIB=$P/kzz_stamps/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 256 32 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 4; }
cat $O/stamps.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cfg2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 5; }
for kind in graph-gp graph-nogp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/step_$kind -o step -- python3 $R/scripts/gp_step.py cfg3 20 $kind > $R/$O/step_$kind.log 2>&1 || { tail -20 $R/$O/step_$kind.log; exit 6; }
done
cd $R
timeout -k 10 300 python scripts/gp_step.py cfg3 10 > $O/gp_step.json 2> $O/gp_step.err || { tail -20 $O/gp_step.err; exit 7; }
cat $O/gp_step.json
echo DONE
