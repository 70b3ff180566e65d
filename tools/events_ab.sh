#!/bin/bash
# Bench wall time with and without per-launch HIP events, alternating.  Usage (GPU box): bash tools/events_ab.sh
set -o pipefail
OUT=gpurun_out/events_ab; mkdir -p $OUT
for r in 1 2 3; do
  for v in ev noev; do
    fl=""; [ $v = noev ] && fl="--no-events"
    timeout -k 10 200 python bench.py --no-cpu-baseline $fl > $OUT/${v}_$r.log 2>&1 || exit 1
    grep '^{' $OUT/${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['launch_ms'], r['shift_ms'])"
  done
done
