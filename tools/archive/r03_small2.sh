#!/bin/bash
# Small boxes after the one-launch full-capacity phases: tests of the launch variants, eager vs
# pmc_run_small (8^3, 16^3), eager vs hipGraph replay (16^3, 32^3) through bench.py.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fallback or small_box or full_sweeps or graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for a in "8 1500" "16 10000"; do
  timeout -k 10 120 python tools/small_box_timing.py $a > $O/sb_${a// /_}.log 2>&1 || { tail -20 $O/sb_${a// /_}.log; exit 1; }
  tail -1 $O/sb_${a// /_}.log
done | tee $O/small_box.txt
for r in 1 2; do
  for c in "16 10000" "32 80000"; do
    set -- $c
    for m in eager graph; do
      F=""; [ $m = graph ] && F="--graph"
      timeout -k 10 200 python bench.py --cps $1 --atoms $2 --steps 200 --warmup 5 --no-cpu-baseline --no-events $F > $O/g$1_${m}_$r.log 2>&1 || { tail -20 $O/g$1_${m}_$r.log; exit 1; }
      grep '^{' $O/g$1_${m}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cps $1 $m ms/sweep %.4f trial-moves/s %.4g flags %s parity %s' % (d['ms_per_step'], d['value'], d['error_flags'], (d.get('parity') or {}).get('state_bitwise_equal')))"
    done
  done
done | tee $O/graph.txt
