# Quick A/B on the GPU: exact parity tests, bench (no CPU leg), phase stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/quick_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --steps 50 --warmup 10 || exit 1
timeout -k 10 120 python scripts/stamps_exact.py 512 || exit 1
timeout -k 10 120 python scripts/stamps_exact.py 256 || exit 1
