#!/bin/bash
# exact-backward timing only (knockout builds give wrong results): time_grad.py + rocprof stats per _lib_ab/<v>
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/ab; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  export GPK_LIB=$R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/$v/libgpk.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gt_$v -o gp -- python3 scripts/time_grad.py > $O/gt_$v.log 2>&1 || { echo "$v FAILED"; tail -5 $O/gt_$v.log; exit 1; }
  grep "grad median" $O/gt_$v.log
  python3 -c "
import csv,glob
f=glob.glob('$O/gt_$v/**/gp_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'grad' in r['Name']: print('   ', r['Name'][:60], round(float(r['AverageNs'])/1e3,2))
"
done
