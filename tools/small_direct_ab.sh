#!/bin/bash
# Full-capacity one-launch path (k_subsweep_full) for the slab boundary launches and larger
# whole-box thresholds: GPU slab tests, then the 8- and 4-rank strong rehearsals with
# PMC_SMALL_DIRECT default vs 0, and whole-box sweeps at 48^3 / 64^3 with PMC_SMALL_LAUNCH 8192 vs 40000.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "slab or world or config4 or full_sweeps or small_box" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for r in 1 2; do
  for m in default 0; do
    if [ $m = default ]; then env=""; else env="PMC_SMALL_DIRECT=0"; fi
    for R in 8 4; do
      env $env timeout -k 10 200 python tools/strong_emulation.py --ranks $R > $O/se_${R}_${m}_$r.log 2>&1 || { tail -20 $O/se_${R}_${m}_$r.log; exit 1; }
      tail -1 $O/se_${R}_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ranks', $R, '$m', {k: d[k] for k in d if 'ms' in k or 'speedup' in k})"
    done
  done
done | tee $O/ab_strong.txt
for a in "48 270000" "64 1000000"; do
  for r in 1 2; do
    for m in 8192 40000; do
      PMC_SMALL_LAUNCH=$m timeout -k 10 120 python tools/small_launch_timing.py $a > $O/t_${a// /_}_${m}_$r.log 2>&1 || { tail -20 $O/t_${a// /_}_${m}_$r.log; exit 1; }
      tail -1 $O/t_${a// /_}_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['cps'], d['small_launch'], round(d['ms_per_sweep'],4), d['state_sha'], d['error_flags'])"
    done
  done
done | tee $O/ab_box.txt
