#!/bin/bash
# Energy-kernel A/B over library variants (tools/build_variant.sh): the energy path tests of each
# NEW variant (PARITY list), then tools/energy_timing.py (128^3/1e7 after 2 sweeps, checked against
# the oracle) alternately.  Usage: PARITY="a b" bash tools/energy_ab.sh <tag> <variant>...
set -o pipefail
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for v in $PARITY; do
  PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "energy_paths or full_sweeps_parity_16 or slab_driver_equals" > $O/parity_$v.log 2>&1 || { echo "parity FAILED for $v"; tail -30 $O/parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.log)"
done
for r in ${REPS:-1 2}; do
  for v in "$@"; do
    PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python tools/energy_timing.py > $O/${v}_$r.log 2>&1 || { tail -20 $O/${v}_$r.log; exit 1; }
    echo "$v $(tail -1 $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["equal"], round(d["ms_per_call_incl_sync"],4))')"
  done
done | tee $O/ab.txt
