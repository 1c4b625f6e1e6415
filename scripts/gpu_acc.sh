set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tests/accuracy_report.py || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --steps 50 --warmup 10 || exit 1
timeout -k 10 120 python scripts/stamps_exact.py 512 || exit 1
timeout -k 10 300 python -m pytest tests -m gpu -x -q 2>&1 | tail -4
