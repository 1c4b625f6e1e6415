# A/B: for the default build and each variant lib given as arguments: exact-kernel
# parity tests, bench (no CPU leg) and phase stamps. Every GPU step has its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" "$@"; do
  echo "== variant ${v:-default}"
  GPK_LIB=$v timeout -k 10 200 python -u -m pytest tests/test_exact_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
  GPK_LIB=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --steps 50 --warmup 10 | grep -o '"kernel_ms": [0-9.]*\|"frac": [0-9.]*' || exit 1
  GPK_LIB=$v timeout -k 10 120 python scripts/stamps_exact.py 512 | grep -v "^sample\|^CUs" || exit 1
done
