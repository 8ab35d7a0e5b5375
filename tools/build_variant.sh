#!/bin/bash
# A/B engine builds: tools/build_variant.sh NAME SRC "FLAGS" — recompiles
# csrc/SRC.hip with FLAGS and links it with the default objects into
# diffopt.jl_amd/diffopt_amd/variants/libdiffopt_NAME.so (select it with
# DOPT_LIB=... for bench.py).
set -e
cd "$(dirname "$0")/../diffopt.jl_amd"
name=$1; src=$2; flags=$3
make -s -j8 >/dev/null
mkdir -p build/var_$name diffopt_amd/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function $flags \
  -c csrc/$src.hip -o build/var_$name/$src.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o diffopt_amd/variants/libdiffopt_$name.so $objs build/var_$name/$src.o
echo diffopt.jl_amd/diffopt_amd/variants/libdiffopt_$name.so
