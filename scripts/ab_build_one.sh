#!/bin/bash
# A/B build of ONE csrc file with extra -D flags, linked against the main build's other
# objects:  scripts/ab_build_one.sh <name> <file.hip> -DFOO=1 ...  -> _lib_ab/<name>/libgpk.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd); P=$R/fine_grained_gaussian_process_forcasting_amd
name=$1; src=$2; shift 2
out=$P/_lib_ab/$name; mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics "$@" -I $R/include -c $P/csrc/$src -o $out/$src.o
objs=$(ls $P/_lib/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $out/$src.o -o $out/libgpk.so
echo $out/libgpk.so
