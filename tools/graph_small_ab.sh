#!/bin/bash
# Eager launches vs hipGraph replay at the small
# configs where launch overhead dominates (16^3/1e4, 64^3/1e6) and at 128^3/1e7,
# alternating.  Usage: bash tools/graph_small_ab.sh [modes]
set -o pipefail
O=gpurun_out/graph_small; mkdir -p $O
for r in 1 2; do
  for cfg in "16 10000" "64 1000000" "128 10000000"; do
    set -- $cfg
    for m in ${MODES:-eager graph}; do
      F=""; [ $m = graph ] && F="--graph"
      timeout -k 10 200 python bench.py --cps $1 --atoms $2 --steps 200 --warmup 5 --no-cpu-baseline --no-events $F > $O/c$1_${m}_$r.log 2>&1 || { tail -20 $O/c$1_${m}_$r.log; exit 1; }
      grep '^{' $O/c$1_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cps $1 $m ms/sweep %.4f trial-moves/s %.4g flags %s' % (d['ms_per_step'], d['value'], d['error_flags']))"
    done
  done
done
