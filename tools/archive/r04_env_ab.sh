#!/bin/bash
# Config-3 (or CONFIG) bench A/B over named environment variants of the same build, alternating,
# REPS rounds.  Usage: bash tools/archive/r04_env_ab.sh <tag> "name:VAR=v,VAR=v" ...
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for r in ${REPS:-1 2 3}; do for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  f=$O/${name}_$r.json
  env $(echo $envs | tr ',' ' ') timeout -k 10 240 python bench.py --config ${CONFIG:-3} --steps ${STEPS:-20} --warmup 5 \
      --no-cpu-baseline ${EXTRA:-} > $f 2> ${f%.json}.err || { echo "FAILED $v"; tail -20 ${f%.json}.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('%-10s rep=$r: %.4e moves/s  step %.4f ms  launch %.4f ms  shift %s ms  flags %s' % ('$name', d['value'], d['ms_per_step'], r['launch_ms'], ('%.4f' % r['shift_ms']) if r['shift_ms'] else '-', d['error_flags']))"
done; done
