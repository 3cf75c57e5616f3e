#!/bin/bash
# Link a variant of libtonk_amd.so whose compression kernel is built with extra defines, or from
# another lz.hip (LZ_SRC=path; A/B runs on the GPU box select it with TONK_AMD_LIB=<name>):
#   tools/build_lz_variant.sh libname.so -DLZ_PROBE=32
set -e
cd "$(dirname "$0")/../tonk_amd"
make -s -j8 libtonk_amd.so
name=$1; shift
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 "$@" -I csrc -x hip -c -o build/_variant_lz.o "${LZ_SRC:-csrc/lz.hip}"
objs=$(ls build/*.o | grep -v 'lz.hip.o' | grep -v _variant)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$name" $objs build/_variant_lz.o -lpthread
echo "built tonk_amd/$name"
