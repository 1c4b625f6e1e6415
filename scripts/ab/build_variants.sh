#!/bin/bash
# scripts/ab/build_variants.sh name:"-DFOO=1 -DBAR=2" ... -> _lib_ab/<name>/libgpk.so (gpk_exact.hip only)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  bash $R/scripts/ab_build_one.sh $name gpk_exact.hip $flags > /dev/null &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls $R/fine_grained_gaussian_process_forcasting_amd/_lib_ab/
