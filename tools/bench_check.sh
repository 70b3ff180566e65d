#!/bin/bash
# The driver's bench command (N=1) twice, plus the config-5 one-rank slab line and the strong
# rehearsal.  Usage (GPU box): bash tools/bench_check.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { tail -30 $O/bench_$r.log; exit 1; }
  grep '^{' $O/bench_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench value %.4g ms/step %.4f phase %s frac %s parity %s' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], (d.get('parity') or {}).get('state_bitwise_equal')))"
done
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench5.log 2>&1 || { tail -30 $O/bench5.log; exit 1; }
grep '^{' $O/bench5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('config5 value %.4g ms/step %.4f err %s bk %s' % (d['value'], d['ms_per_step'], d['error_flags'], d['energy']['bookkeeping_rel_err']))"
