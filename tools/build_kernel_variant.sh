#!/bin/bash
# Build the HIP library with pmc_kernels.hip compiled under other flags into build/variants/lib_<name>.so
# (same-box A/B of kernel-side switches or timing probes; select with PMC_LIB_PATH).
#   bash tools/build_kernel_variant.sh <name> [extra hipcc flags]
set -e
NAME=$1; shift
D=parallel-monte-carlo_amd
OUT=$D/build/variants
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c -o $OUT/kern_$NAME.o $D/csrc/pmc_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$NAME.so $OUT/kern_$NAME.o $D/build/pmc_api.o $D/build/pmc_io.o
