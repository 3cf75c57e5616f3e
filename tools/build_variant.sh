#!/bin/bash
# Link a variant of libtonk_amd.so whose kernels come from another kernels.hip (A/B runs on the
# GPU box select it with TONK_AMD_LIB=<name>):  tools/build_variant.sh path/to/kernels.hip libname.so
set -e
cd "$(dirname "$0")/../tonk_amd"
make -s -j8 libtonk_amd.so
cp "$1" csrc/_variant_kernels.hip
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -mllvm -simplifycfg-sink-common=false -c -o build/_variant_kernels.o csrc/_variant_kernels.hip
rm -f csrc/_variant_kernels.hip
objs=$(ls build/*.o | grep -v 'kernels.hip.o' | grep -v _variant_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$2" $objs build/_variant_kernels.o -lpthread
echo "built tonk_amd/$2"
