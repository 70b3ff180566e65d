#!/bin/bash
# Build the HIP library with pmc_api.hip compiled under other flags into build/variants/lib_<name>.so
# (same-box A/B of host-side schedule switches; select with PMC_LIB_PATH).
#   bash tools/build_api_variant.sh <name> [extra hipcc flags, e.g. -DPMC_SLAB_INTERLEAVE=0]
set -e
NAME=$1; shift
D=parallel-monte-carlo_amd
OUT=$D/build/variants
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $F "$@" -c -o $OUT/api_$NAME.o $D/csrc/pmc_api.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$NAME.so $D/build/pmc_kernels.o $OUT/api_$NAME.o $D/build/pmc_io.o
