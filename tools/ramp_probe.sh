#!/bin/bash
# Clock ramp after the bench's idle analysis gap: 20 timed steps without / with the GPU re-warm,
# and 200 steps, alternating.  Usage (GPU box): bash tools/ramp_probe.sh
set -o pipefail
OUT=gpurun_out/ramp; mkdir -p $OUT
for r in 1 2; do
  for v in "20 0" "20 300" "20 1000" "200 300"; do
    set -- $v
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-events --steps $1 --prewarm-ms $2 > $OUT/s$1_p$2_$r.log 2>&1 || exit 1
    grep '^{' $OUT/s$1_p$2_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps $1 prewarm $2', d['value'], d['ms_per_step'])"
  done
done
