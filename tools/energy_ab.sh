#!/bin/bash
# k_energy A/B over library variants (tools/build_variant.sh), alternating, 3 rounds.
# Usage (GPU box, repo root): bash tools/energy_ab.sh <variant>...
set -o pipefail
OUT=gpurun_out/energy_ab; mkdir -p $OUT
for r in 1 2 3; do
  for v in "$@"; do
    PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python tools/energy_timing.py > $OUT/${v}_$r.log 2>&1 || exit 1
    echo "$v $(tail -n 1 $OUT/${v}_$r.log)"
  done
done
