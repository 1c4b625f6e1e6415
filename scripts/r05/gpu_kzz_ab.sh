#!/bin/bash
# K_ZZ factor + inverse A/B: timing per variant, phase stamps, kernel stats
R="$GRAFT_REPO_ROOT"; cd "$R"; export TMPDIR=/tmp; O=$R/gpurun_out/${TAG:-kzzab}; mkdir -p $O
P=$R/fine_grained_gaussian_process_forcasting_amd
for v in main ${VARIANTS:-iso inv2 both}; do
  lib=$P/_lib/libgpk.so; [ $v = main ] || lib=$P/_lib_ab/$v/libgpk.so
  echo "== $v" >> $O/time.txt
  GPK_LIB=$lib timeout -k 10 120 python scripts/time_kzz.py >> $O/time.txt 2>&1 || exit 1
done
for v in ${STAMPS:-st0 st1}; do
  echo "== $v" >> $O/stamps.txt
  GPK_LIB=$P/_lib_ab/$v/libgpk.so timeout -k 10 120 python scripts/kzz_stamps.py 256 32 >> $O/stamps.txt 2>&1 || exit 1
done
cat $O/time.txt
