# A/B of the posterior kernel: parity tests + bench posterior leg, default lib then each
# variant lib given as an argument. Every GPU step has its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" "$@"; do
  echo "== variant ${v:-default}"
  GPK_LIB=$v timeout -k 10 200 python -u -m pytest tests/test_posterior_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/post_ab_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/post_ab_pytest.log; [ $rc -eq 0 ] || exit $rc
  for k in 1 2; do
    GPK_LIB=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --no-cfg2 --no-var --steps 20 --warmup 5 > gpurun_out/post_ab_bench.log || exit 1
    python -c "import json;l=json.loads(open('gpurun_out/post_ab_bench.log').read().strip().splitlines()[-1]);print('post_ms',l['posterior']['kernel_ms'],'exact_ms',l['ms_per_step'])" || exit 1
  done
done
