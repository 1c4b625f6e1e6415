#!/bin/bash
# A/B of the exact kernel's trailing-update precision: split-f16 (default) vs fp32 MFMA
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/split_ab; mkdir -p $O
AB="$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/fp32upd/libgpk.so"
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-var --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > $O/bench_split.json 2> $O/bench_split.err || exit 1
GPK_LIB=$AB timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-var --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > $O/bench_fp32.json 2> $O/bench_fp32.err || exit 2
timeout -k 10 300 python tests/accuracy_report.py > $O/acc_split.txt 2>&1 || exit 3
GPK_LIB=$AB timeout -k 10 300 python tests/accuracy_report.py > $O/acc_fp32.txt 2>&1 || exit 4
GPK_LIB=$AB timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_exact_gpu.py > $O/tests_fp32.log 2>&1 || { tail -30 $O/tests_fp32.log; exit 5; }
tail -3 $O/tests_fp32.log
python - <<'PY'
import json
for k in ("split", "fp32"):
    d = json.loads(open(f"gpurun_out/split_ab/bench_{k}.json").read().strip().splitlines()[-1])
    print(k, d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
