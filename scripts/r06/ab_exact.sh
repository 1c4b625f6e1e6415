#!/bin/bash
# A/B of exact-kernel builds: alternating child processes (scripts/time_exact.py) per shape.
#   LIBS="name=path ..." SHAPES="B:N ..." REPS=3 bash scripts/r06/ab_exact.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${TAG:-r06ab}; mkdir -p $O
SHAPES=${SHAPES:-"512:256 128:128 64:256 256:256"}; REPS=${REPS:-3}
for rep in $(seq 1 $REPS); do
  for sh in $SHAPES; do
    B=${sh%%:*}; N=${sh#*:}
    for nl in $LIBS; do
      name=${nl%%=*}; lib=${nl#*=}
      out=$(GPK_LIB=$R/$lib timeout -k 10 120 python scripts/time_exact.py $B $N 32 50 2>/dev/null | tail -n 1) || { echo "FAIL $name $B $N"; exit 3; }
      echo "$rep $name B=$B N=$N $out" | tee -a $O/ab.txt
    done
  done
done
