#!/bin/bash
# Round-2 measurement set on the GPU box: default bench line, eager vs hipGraph A/B, occupancy
# probes, rocprofv3 kernel-trace stats of the bench, SQ instruction counters and the k_subsweep
# traffic passes.  Usage: bash tools/archive/r02_profile.sh <tag>
set -o pipefail
T=$1; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > $O/parity_first.log 2>&1; tail -n 1 $O/parity_first.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
for r in 1 2; do
  for mode in eager graph; do
    F=""; [ $mode = graph ] && F="--graph"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-events --steps 40 $F > $O/ab_${mode}_$r.log 2>&1 || { tail -20 $O/ab_${mode}_$r.log; exit 1; }
    grep '^{' $O/ab_${mode}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['ms_per_step'])"
  done
done
for v in occ134 occ200 occ400; do
  [ -f parallel-monte-carlo_amd/build/variants/lib_$v.so ] || continue
  PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep '^{' $O/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
bash tools/sq_counters.sh $T > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
bash tools/tcc_traffic.sh $T > $O/tcc.log 2>&1 || { tail -20 $O/tcc.log; exit 1; }
timeout -k 10 120 python tools/energy_timing.py > $O/energy.log 2>&1 || { tail -20 $O/energy.log; exit 1; }
tail -n 1 $O/energy.log
echo done
