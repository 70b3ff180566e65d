#!/bin/bash
# Round 4: the world-1 slab driver against the oracle (one- and two-plane halos, local and one-rank
# RCCL transport); one cell per wave for mid-size phases (PMC_DIRECT_CELLS) on config 2 and on the
# 8-rank rehearsal's interior launches, with a config-2 parity run of that form.
# Usage (GPU box, repo root): bash tools/r04k.sh <tag>
set -o pipefail
T=${1:-r04k}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "c_slab_driver_equals_whole_box" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
PMC_DIRECT_CELLS=40000 timeout -k 10 300 python bench.py --config 2 --steps 16 --warmup 8 > $O/bench2_direct.log 2>&1 || { tail -20 $O/bench2_direct.log; exit 1; }
grep '^{' $O/bench2_direct.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['parity']; print('direct config 2 parity', p['state_bitwise_equal'], p['counters_equal'], d['value'])"
CONFIG=2 STEPS=160 REPS="1 2 3" bash tools/r04_env_ab.sh ${T}_c2 "main:PMC_DIRECT_CELLS=0" "direct:PMC_DIRECT_CELLS=40000" || exit 1
R=8 DELAYS="0" REPS="1 2" bash tools/r04_variants_ab.sh ${T}_e8 "main:PMC_DIRECT_CELLS=0" "direct:PMC_DIRECT_CELLS=40000" || exit 1
