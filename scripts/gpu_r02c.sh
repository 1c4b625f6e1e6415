#!/bin/bash
# variational kernel timings + SQ counters
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/var_kernels.py 5 all > gpurun_out/var_times.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profv" -o run -- python3 "$R/scripts/var_kernels.py" 3 all > "$R/gpurun_out/profv.log" 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$R/gpurun_out/pmcv1" -o run -- python3 "$R/scripts/var_kernels.py" 1 all > "$R/gpurun_out/pmcv1.log" 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmcv2" -o run -- python3 "$R/scripts/var_kernels.py" 1 all > "$R/gpurun_out/pmcv2.log" 2>&1 || exit 4
echo done
