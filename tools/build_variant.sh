#!/bin/bash
# A/B engine builds: tools/build_variant.sh NAME SRC "FLAGS" [REV]
# recompiles csrc/SRC.hip (or, with REV, the file as of git revision REV) with
# FLAGS and links it in place of build/SRC.o with the other default objects
# into diffopt.jl_amd/diffopt_amd/variants/libdiffopt_NAME.so (select it with
# DOPT_LIB=... for bench.py).
set -e
cd "$(dirname "$0")/../diffopt.jl_amd"
name=$1; src=$2; flags=$3; rev=$4
make -s -j8 >/dev/null
mkdir -p build/var_$name diffopt_amd/variants
file=csrc/$src.hip
if [ -n "$rev" ]; then
  file=csrc/_var_${name}_$src.hip
  git show $rev:diffopt.jl_amd/csrc/$src.hip > $file
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function $flags \
  -c $file -o build/var_$name/$src.o
[ -n "$rev" ] && rm -f $file
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o diffopt_amd/variants/libdiffopt_$name.so $objs build/var_$name/$src.o
echo diffopt.jl_amd/diffopt_amd/variants/libdiffopt_$name.so
