#!/bin/bash
# Strong-scaling rehearsal A/B over named environment variants of the product library (same build):
# bench.py --config 4 --emulate-ranks R, alternating variants x injected delays, REPS rounds.
# Usage: R=8 DELAYS="0 80" REPS="1 2" bash tools/archive/r04_variants_ab.sh <tag> "name:VAR=v,VAR=v" ...
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for r in ${REPS:-1 2}; do for v in "$@"; do for dl in ${DELAYS:-0 80}; do
  name=${v%%:*}; envs=${v#*:}
  f=$O/${name}_d${dl}_R${R:-8}_$r.json
  env $(echo $envs | tr ',' ' ') timeout -k 10 240 python bench.py --config 4 --emulate-ranks ${R:-8} --steps ${STEPS:-100} \
      --warmup 5 --no-cpu-baseline --xfer-delay-us $dl > $f 2> ${f%.json}.err || { echo "FAILED $v delay=$dl"; tail -20 ${f%.json}.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('R${R:-8} %-10s delay=%3s rep=$r: rank sweep %.4f ms  interior %.4f  boundary %.4f  shift %.4f  flags %s' % ('$name', '$dl', d['ms_per_step'], r['launch_ms'], r['boundary_launch_ms'] or 0, r['shift_ms'] or 0, d['error_flags']))"
done; done; done
