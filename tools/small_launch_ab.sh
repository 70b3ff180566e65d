#!/bin/bash
# Small-launch A/B: per-sweep time at several box sizes with the small-launch path (default
# threshold) and without it (PMC_SMALL_LAUNCH=0), alternating, plus the GPU parity subset.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "full_sweeps or acceptance or move_count or small_box or graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for a in "16 10000" "24 40000" "32 80000" "48 270000" "64 1000000"; do
  for r in 1 2; do
    for m in default 0; do
      if [ $m = default ]; then env=""; else env="PMC_SMALL_LAUNCH=0"; fi
      env $env timeout -k 10 120 python tools/small_launch_timing.py $a > $O/t_${a// /_}_${m}_$r.log 2>&1 || { tail -20 $O/t_${a// /_}_${m}_$r.log; exit 1; }
      tail -1 $O/t_${a// /_}_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['cps'], d['small_launch'], round(d['ms_per_sweep'],4), d['state_sha'], d['error_flags'])"
    done
  done
done | tee $O/ab.txt
