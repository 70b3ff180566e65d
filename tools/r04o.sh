#!/bin/bash
# Round 4 probe: the 8-rank rehearsal without the per-phase fallback launches (PMC_PROBE_NO_FALLBACK:
# wrong results only if a cell overflows the main capacity) -- how much of the rank sweep the empty
# fallback launches cost on the chains.  Usage (GPU box, repo root): bash tools/r04o.sh <tag>
set -o pipefail
T=${1:-r04o}; O=gpurun_out/$T; mkdir -p $O
V=$PWD/parallel-monte-carlo_amd/build/variants
PMC_LIB_PATH=$V/lib_nofb.so timeout -k 10 300 python bench.py --config 4 --emulate-ranks 8 --steps 40 --warmup 5 > $O/nofb_parity.log 2>&1 || { tail -20 $O/nofb_parity.log; exit 1; }
grep '^{' $O/nofb_parity.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity']; print('nofb parity', p['state_bitwise_equal'], p['counters_equal'], d['ms_per_step'])"
R=8 DELAYS="0 80" REPS="1 2 3" bash tools/r04_variants_ab.sh ${T}_ab "cur:PMC_LIB_PATH=$V/lib_cur.so" "nofb:PMC_LIB_PATH=$V/lib_nofb.so" || exit 1
