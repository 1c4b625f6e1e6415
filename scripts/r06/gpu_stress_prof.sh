#!/bin/bash
# Determinism stress of every production kernel, then rocprofv3 stats + FETCH / WRITE passes of
# the round-6 kernels (scripts/r06/prof_new.py). Each GPU step has its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-stress}; mkdir -p $O
timeout -k 10 400 python -u scripts/r06/stress_determinism.py ${REPS:-100} > $O/stress.log 2>&1; rc=$?
cat $O/stress.log | tail -25
[ $rc -eq 0 ] || exit $rc
cd /tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o new -- python3 $R/scripts/r06/prof_new.py > $O/prof_new.log 2>&1 && echo PROF_OK &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_new -o new -- python3 $R/scripts/r06/prof_new.py > $O/pmc1_new.log 2>&1 && echo PMC1_OK &&
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_new -o new -- python3 $R/scripts/r06/prof_new.py > $O/pmc2_new.log 2>&1 && echo PMC2_OK
