#!/bin/bash
# Round 4: direct halo writes for the single-rank slab (PMC_SLAB_DIRECT_HALO=1: the boundary launches
# also write each stored row into the halo plane of its periodic image; the run exchange copies
# nothing) -- parity of the world-1 slab tests with it on, then the 8-rank rehearsal A/B.
# Usage (GPU box, repo root): bash tools/r04w.sh <tag>
set -o pipefail
T=${1:-r04w}; O=gpurun_out/$T; mkdir -p $O
PMC_SLAB_DIRECT_HALO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "slab_driver_equals or forced_fallback or timing_and_restart or rewarm" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
PMC_SLAB_DIRECT_HALO=1 timeout -k 10 300 python bench.py --config 4 --emulate-ranks 8 --steps 40 --warmup 5 > $O/parity_direct.log 2>&1 || { tail -20 $O/parity_direct.log; exit 1; }
grep '^{' $O/parity_direct.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity']; print('direct halo rehearsal parity', p['state_bitwise_equal'], p['counters_equal'], d['ms_per_step'])"
R=8 DELAYS="0 80" REPS="1 2 3" bash tools/r04_variants_ab.sh ${T}_ab "copy:PMC_SLAB_DIRECT_HALO=0" "direct:PMC_SLAB_DIRECT_HALO=1" || exit 1
