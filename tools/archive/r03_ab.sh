#!/bin/bash
# Round 3 kernel A/B: parity of each variant (a subset of the GPU parity tests through PMC_LIB_PATH)
# then the default bench alternately (tools/bench_ab.sh).  Usage: bash tools/archive/r03_ab.sh <tag> <variant>...
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for v in "$@"; do
  PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${PARITY_K:-full_sweeps or acceptance or move_count or odd_colour or graph or single_colour or all_colour}" > $O/parity_$v.log 2>&1 || { echo "parity FAILED for $v"; tail -30 $O/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.log)"
done
REPS="${REPS:-1 2 3}" bash tools/bench_ab.sh "$@" 2>&1 | tee $O/ab.txt
