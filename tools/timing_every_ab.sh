#!/bin/bash
# Bench at the driver's step counts with events on every launch / every 4th sweep / none.
set -o pipefail
O=gpurun_out/tev; mkdir -p $O
for r in 1 2; do for v in "1" "4" "none"; do
  fl="--timing-every $v"; [ $v = none ] && fl="--no-events"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $fl > $O/t${v}_$r.log 2>&1 || exit 1
  grep '^{' $O/t${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('every $v', d['value'], d['ms_per_step'], r['launch_ms'], r['launches_timed'], r['shift_ms'])"
done; done
