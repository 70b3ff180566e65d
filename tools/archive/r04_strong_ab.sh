#!/bin/bash
# Round 4: strong-scaling rehearsal A/B over interior chain count and injected exchange delay.
# bench.py --config 4 --emulate-ranks R (one rank's slab of the 128^3/1e7 box, product C slab driver),
# alternating variants, REPS rounds.  Usage: R=8 CHAINS="2 3" DELAYS="0 80" REPS="1 2 3" bash tools/archive/r04_strong_ab.sh <tag>
set -o pipefail
T=${1:-r04_strong}
O=gpurun_out/$T; mkdir -p $O
for r in ${REPS:-1 2 3}; do for ch in ${CHAINS:-2 3}; do for dl in ${DELAYS:-0}; do
  f=$O/c${ch}_d${dl}_R${R:-8}_$r.json
  PMC_SLAB_CHAINS=$ch timeout -k 10 240 python bench.py --config 4 --emulate-ranks ${R:-8} --steps ${STEPS:-100} \
      --warmup 5 --no-cpu-baseline --xfer-delay-us $dl ${EXTRA:-} > $f 2> $O/c${ch}_d${dl}_R${R:-8}_$r.err || { echo "FAILED chains=$ch delay=$dl"; tail -20 $O/c${ch}_d${dl}_R${R:-8}_$r.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
r=d['roofline']
print('R${R:-8} chains=$ch delay=$dl rep=$r: rank sweep %.4f ms  interior launch %.4f ms  boundary %.4f ms  shift %.4f ms  flags %s' % (d['ms_per_step'], r['launch_ms'], r['boundary_launch_ms'] or 0, r['shift_ms'] or 0, d['error_flags']))"
done; done; done
