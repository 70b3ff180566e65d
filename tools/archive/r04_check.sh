#!/bin/bash
# Round-4 end check on one box: the GPU suite, smoke, and the driver's default bench command.
# Usage (GPU box, repo root): bash tools/archive/r04_check.sh <tag>
set -o pipefail
T=${1:-r04_check}; O=gpurun_out/$T; mkdir -p $O
bash tools/archive/r03_tests.sh $T || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log > $O/bench_default.json
python3 -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; p=d['parity']; print('default bench', d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], p['state_bitwise_equal'], p['counters_equal'], d['vs_baseline'])"
