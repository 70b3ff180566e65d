#!/bin/bash
# Round 4: the 8-rank rehearsal with its halos through a one-rank RCCL communicator (--self-rccl:
# every exchange is a real ncclSend/ncclRecv group, RCCL's kernels and launch costs included), one-
# against two-plane halos, plus the full-capacity boundary launches.  Usage: bash tools/r04r.sh <tag>
set -o pipefail
T=${1:-r04r}; O=gpurun_out/$T; mkdir -p $O
for r in 1 2 3; do for v in "h1:PMC_SLAB_HALO=1" "h2:PMC_SLAB_HALO=2" "bfull:PMC_BOUNDARY_FULL=1"; do
  name=${v%%:*}; envs=${v#*:}; f=$O/${name}_$r.json
  env $envs timeout -k 10 240 python bench.py --config 4 --emulate-ranks 8 --self-rccl --steps 100 --warmup 5 \
      --no-cpu-baseline > $f 2> ${f%.json}.err || { echo "FAILED $v"; tail -20 ${f%.json}.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']
print('R8 rccl %-6s rep=$r: rank sweep %.4f ms  interior %.4f  boundary %.4f  flags %s' % ('$name', d['ms_per_step'], r['launch_ms'], r['boundary_launch_ms'] or 0, d['error_flags']))"
done; done
