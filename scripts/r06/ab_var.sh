#!/bin/bash
# A/B of saved-state adjoint builds (scripts/r06/time_var_saved.py), alternating child processes.
#   LIBS="name=path ..." NS="192 96" REPS=2 bash scripts/r06/ab_var.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06abv}; mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do for n in ${NS:-192 96}; do for nl in $LIBS; do
  name=${nl%%=*}; lib=${nl#*=}
  o=$(GPK_LIB=$R/$lib timeout -k 10 120 python scripts/r06/time_var_saved.py 256 $n 256 32 2>/dev/null | tail -n 1) || { echo FAIL $name; exit 3; }
  echo "$rep $name N=$n $o" | tee -a $O/ab.txt
done; done; done
