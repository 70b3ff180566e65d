#!/bin/bash
# Sweep cost against the sweep index (the lattice start melts over the first sweeps): 100 timed
# steps after 3 / 100 / 500 warmup sweeps.  Usage (GPU box): bash tools/warmup_probe.sh
set -o pipefail
OUT=gpurun_out/warmup; mkdir -p $OUT
for w in 3 100 500; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-events --steps 100 --warmup $w > $OUT/w$w.log 2>&1 || exit 1
  grep '^{' $OUT/w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warmup $w', d['value'], d['ms_per_step'], d['acceptance'], d['energy']['per_particle_end'])"
done
