#!/bin/bash
# A/B: time one colour phase (MOVES list) for each library variant in build/variants.
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
for v in "$@"; do
  PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so MOVES=${MOVES:-0,10} \
    timeout -k 10 200 python tools/ablate.py > $OUT/$v.log 2>&1 || exit $?
done
