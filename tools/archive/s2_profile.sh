#!/bin/bash
# Round-2 final measurement set (GPU box): GPU tests, the driver's bench command, rocprofv3 kernel
# stats of the same command, config 5 / 5box lines, strong rehearsal 8/4, energy timing.
# Usage: bash tools/archive/s2_profile.sh <tag>
set -o pipefail
T=$1; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench value %.4g ms/step %.4f phase %.4f frac %.4f parity %s' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], d['parity']['state_bitwise_equal']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep '^{' $O/prof.log > $O/prof_bench.json
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench5.log 2>&1 || { tail -20 $O/bench5.log; exit 1; }
grep '^{' $O/bench5.log > $O/bench5.json
timeout -k 10 400 python bench.py --config 5box --steps 10 --warmup 3 > $O/bench5box.log 2>&1 || { tail -20 $O/bench5box.log; exit 1; }
grep '^{' $O/bench5box.log > $O/bench5box.json
for f in bench5 bench5box; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f value %.4g ms/step %.4f parity %s bk %s' % (d['value'], d['ms_per_step'], (d.get('parity') or {}).get('state_bitwise_equal'), d['energy']['bookkeeping_rel_err']))"; done
for R in 8 4; do
  timeout -k 10 200 python tools/strong_emulation.py --ranks $R > $O/strong$R.log 2>&1 || { tail -30 $O/strong$R.log; exit 1; }
  grep '^{' $O/strong$R.log > $O/strong$R.json
  python3 -c "import json; d=json.load(open('$O/strong$R.json')); print('strong R=%d full %.4f rank %.4f speedup %.2f host %.3f' % (d['ranks_emulated'], d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'], d['host_only_ms_per_sweep']))"
done
timeout -k 10 120 python tools/energy_timing.py > $O/energy.log 2>&1 || { tail -20 $O/energy.log; exit 1; }
tail -n 1 $O/energy.log
