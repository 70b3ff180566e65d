#!/bin/bash
# Round-3 measurement set on one box: GPU suite, smoke, bench lines (configs 3/4/4x8/5), rocprofv3
# kernel stats of the driver's bench command, TCC traffic and SQ counters of k_subsweep, energy timing.
# Usage (GPU box, repo root): bash tools/archive/r03_final.sh <tag>
set -o pipefail
T=$1; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
bash tools/archive/r03_tests.sh $T || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
bash tools/archive/r03_bench.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python3 tools/rocprof_timed_mean.py $(find $O/prof -name "*kernel_trace.csv" | head -1) 20 | tee $O/rocprof_timed_mean.txt
grep '^{' $O/prof_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench under rocprof', d['value'], d['roofline']['launch_ms'])"
bash tools/tcc_traffic.sh $T > $O/tcc.log 2>&1 || { tail -20 $O/tcc.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/tcc_$T/summary.json')); print('traffic per launch', d['read_bytes_per_launch'], d['write_bytes_per_launch'], d['traffic_bytes_per_launch'])"
bash tools/sq_counters.sh $T > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
tail -3 $O/sq.log
timeout -k 10 200 python tools/energy_timing.py > $O/energy.log 2>&1 || { tail -20 $O/energy.log; exit 1; }
tail -1 $O/energy.log
