#!/bin/bash
# 8- and 4-rank strong rehearsals with the interior launches on the full-capacity one-launch path
# (PMC_SMALL_LAUNCH above their cell counts) against the default threshold, alternating.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for m in 8192 20000 70000; do
    for R in 8 4; do
      PMC_SMALL_LAUNCH=$m timeout -k 10 200 python tools/strong_emulation.py --ranks $R > $O/se_${R}_${m}_$r.log 2>&1 || { tail -20 $O/se_${R}_${m}_$r.log; exit 1; }
      tail -1 $O/se_${R}_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ranks', $R, 'small_launch', $m, 'rank_sweep_ms %.4f full_box_ms %.4f proj %.3f' % (d['rank_sweep_ms'], d['full_box_sweep_ms'], d['projected_speedup']))"
    done
  done
done | tee $O/ab.txt
