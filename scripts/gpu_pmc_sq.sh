# SQ instruction-mix / stall counters for the exact kernel (one PMC pass each).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 90 rocprofv3 -L > $R/gpurun_out/rocprof_L.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $R/gpurun_out/rocprof_L.txt | sort -u > $R/gpurun_out/sq_counters.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc_sq1 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_sq1.log 2>&1 && echo SQ1_OK
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_sq2.log 2>&1 && echo SQ2_OK
