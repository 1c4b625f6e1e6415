#!/bin/bash
# new K_ZZ factor (16-column steps) + K_ZZ adjoint kernel + fused ELBO terms: targeted parity
# first, K_ZZ timings, then the whole GPU suite, smoke, bench and the graphed cfg-3 step
# kernel stats with / without the GP branch
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/${OUT:-r03p}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_elbo_gpu.py "tests/test_variational_gpu.py" "tests/test_variational_grad_gpu.py" > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 2 $O/quick.log
timeout -k 10 120 python scripts/time_kzz.py > $O/kzz.txt 2>&1 || { tail -20 $O/kzz.txt; exit 2; }
cat $O/kzz.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 3; }
tail -n 2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 4; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --strong --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-var3 > $O/bench_torchrun_strong.json 2> $O/bench_torchrun_strong.err || { tail -20 $O/bench_torchrun_strong.err; exit 7; }
cat $O/bench_torchrun_strong.json
cd /tmp
for kind in graph-gp graph-nogp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/step_$kind -o step -- python3 $R/scripts/gp_step.py cfg3 20 $kind > $R/$O/step_$kind.log 2>&1 || { tail -20 $R/$O/step_$kind.log; exit 6; }
done
echo DONE
