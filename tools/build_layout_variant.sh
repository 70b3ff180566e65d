#!/bin/bash
# Build the whole HIP library (kernels AND host API: both use the state layout) with extra flags into
# build/variants/lib_<name>.so, e.g. the packed state layout: bash tools/build_layout_variant.sh aos -DPMC_AOS=1
set -e
NAME=$1; shift
D=parallel-monte-carlo_amd
OUT=$D/build/variants
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -Wno-unused-function $*"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-atomic-optimizer-strategy=None -c -o $OUT/k_$NAME.o $D/csrc/pmc_kernels.hip &
/opt/rocm/bin/hipcc $F -c -o $OUT/api_$NAME.o $D/csrc/pmc_api.hip
wait
g++ -O2 -std=c++17 -fPIC -Wall -c -o $OUT/io_$NAME.o $D/csrc/pmc_io.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$NAME.so $OUT/k_$NAME.o $OUT/api_$NAME.o $OUT/io_$NAME.o
