#!/bin/bash
# Build the HIP library from a given pmc_kernels.hip into build/variants/lib_<name>.so (A/B timing
# with tools/ab_variants.sh).  Usage: bash tools/build_variant.sh <name> [kernels.hip] [extra hipcc flags]
set -e
NAME=$1; SRC=${2:-parallel-monte-carlo_amd/csrc/pmc_kernels.hip}; shift 2 || shift $#
D=parallel-monte-carlo_amd
OUT=$D/build/variants
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -I$D/csrc"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -o $OUT/k_$NAME.o $SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$NAME.so $OUT/k_$NAME.o $D/build/pmc_api.o $D/build/pmc_io.o
