#!/bin/bash
# K_ZZ factor: 16 waves (15 round-robin workers + diagonal wave) vs 8 waves; parity, timing, stamps
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r03v; mkdir -p $O
export TMPDIR=/tmp
P=fine_grained_gaussian_process_forcasting_amd/_lib_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_variational_gpu.py tests/test_variational_grad_gpu.py tests/test_graphs_gpu.py tests/test_e2e_gpu.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -n 1 $O/quick.log
timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_main.txt 2>&1 || { tail -20 $O/kzz_main.txt; exit 2; }
cat $O/kzz_main.txt
GPK_LIB=$P/kzz_w8/libgpk.so timeout -k 10 120 python scripts/time_kzz.py > $O/kzz_w8.txt 2>&1 || { tail -20 $O/kzz_w8.txt; exit 3; }
head -2 $O/kzz_w8.txt
GPK_LIB=$P/kzz_stamps/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 256 32 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 4; }
cat $O/stamps.txt

timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-cfg2 --no-grad > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
python -c "import json; d=json.load(open('$O/bench.json')); v=d['variational']; print('cfg5', v['kernel_ms'], v['roofline']['frac'], v['backward_roofline']['frac']); [print(k, x['kernel_ms'], x['backward_roofline']['frac']) for k, x in d['variational_cfg3'].items()]"
echo DONE
