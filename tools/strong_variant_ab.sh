#!/bin/bash
# Strong rehearsal (8 and 4 ranks) over library variants, alternating; slab tests of the PARITY variants.
# Usage: PARITY="a" bash tools/strong_variant_ab.sh <tag> <variant>...
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for v in $PARITY; do
  PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "slab or world or config4" > $O/parity_$v.log 2>&1 || { echo "parity FAILED for $v"; tail -30 $O/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.log)"
done
for r in 1 2 3; do
  for v in "$@"; do
    for R in 8 4; do
      PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python tools/strong_emulation.py --ranks $R > $O/se_${v}_${R}_$r.log 2>&1 || { tail -20 $O/se_${v}_${R}_$r.log; exit 1; }
      tail -1 $O/se_${v}_${R}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v ranks $R rank_sweep_ms %.4f full_box_ms %.4f proj %.3f' % (d['rank_sweep_ms'], d['full_box_sweep_ms'], d['projected_speedup']))"
    done
  done
done | tee $O/ab.txt
