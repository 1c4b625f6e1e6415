# A/B: parity tests on the default build, then bench + phase stamps for each variant lib.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/ab_pytest.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/ab_pytest.log
for v in "" build/ab_f32/libgpk.so; do
  echo "== variant ${v:-default}"
  GPK_LIB=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 || exit 1
  GPK_LIB=$v timeout -k 10 120 python scripts/stamps_exact.py 512 || exit 1
done
