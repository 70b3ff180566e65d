#!/bin/bash
set -o pipefail
O=gpurun_out/rewarm; mkdir -p $O
for a in "5 0" "5 12" "5 2" ; do
  set -- $a
  timeout -k 10 300 python bench.py --config $1 --rewarm $2 --steps 10 --warmup 3 --no-cpu-baseline > $O/c$1_r$2.log 2>&1 || { tail -30 $O/c$1_r$2.log; exit 1; }
  grep '^{' $O/c$1_r$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('config $1 rewarm $2 ms/step %.4f bk %s acc %s' % (d['ms_per_step'], d['energy']['bookkeeping_rel_err'], d['acceptance']))"
done
timeout -k 10 300 python bench.py --slab --self-rccl --rewarm 12 --steps 10 --warmup 3 --no-cpu-baseline > $O/slab3.log 2>&1 || { tail -30 $O/slab3.log; exit 1; }
grep '^{' $O/slab3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('slab3 rewarm 12 ms/step %.4f bk %s acc %s' % (d['ms_per_step'], d['energy']['bookkeeping_rel_err'], d['acceptance']))"
