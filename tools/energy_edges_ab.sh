#!/bin/bash
# Energy A/B with rocprofv3 per-kernel stats per variant (rows / edges / queue), energy tests first.
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for v in $PARITY; do
  PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "energy_paths or full_sweeps_parity_16 or slab_driver_equals" > $O/parity_$v.log 2>&1 || { echo "parity FAILED for $v"; tail -30 $O/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.log)"
done
for r in 1 2; do
  for v in "$@"; do
    PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${v}_$r -o run -- python3 tools/energy_timing.py > $O/${v}_$r.log 2>&1 || { tail -20 $O/${v}_$r.log; exit 1; }
    f=$(find $O/p_${v}_$r -name "*kernel_stats.csv" | head -1)
    echo "$v $r $(tail -1 $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["equal"], round(d["ms_per_call_incl_sync"],4))') $(python3 -c "
import csv,sys
out=[]
for r in csv.DictReader(open('$f')):
    if 'energy' in r['Name']:
        out.append(r['Name'].split('(')[0].split('::')[-1] + ' %.1f' % (float(r['AverageNs'])/1e3))
print('; '.join(out))")"
  done
done | tee $O/ab.txt
