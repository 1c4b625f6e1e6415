#!/bin/bash
# SQ counters of the exact backward per _lib_ab/<v> build: one --pmc pass per variant
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/gpmc; mkdir -p $O; cd /tmp; export TMPDIR=/tmp; cd "$R"
for v in "$@"; do
  GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE --output-format csv -d $O/$v -o p -- python3 scripts/time_grad.py > $O/$v.log 2>&1 || { echo "$v PMC FAILED"; tail -5 $O/$v.log; exit 1; }
  echo "$v ok"
done
