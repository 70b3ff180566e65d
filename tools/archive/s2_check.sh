#!/bin/bash
# round-2 session-2 check: rewarm test, bench (driver command), strong rehearsal 8/4 ranks
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k rewarm -x -q --timeout 120 --timeout-method thread > $O/rewarm_test.log 2>&1 || { tail -30 $O/rewarm_test.log; exit 1; }
tail -1 $O/rewarm_test.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('bench value %.4g ms/step %.4f phase %s frac %s parity %s bk %s' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], (d.get('parity') or {}).get('state_bitwise_equal'), d['energy']['bookkeeping_rel_err']))"
for R in 8 4; do
  timeout -k 10 200 python tools/strong_emulation.py --ranks $R > $O/strong$R.log 2>&1 || { tail -30 $O/strong$R.log; exit 1; }
  grep '^{' $O/strong$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('strong R=%d full %.4f rank %.4f speedup %.2f host %.3f' % (d['ranks_emulated'], d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'], d['host_issue_ms_per_sweep']))"
done
