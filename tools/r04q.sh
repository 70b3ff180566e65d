#!/bin/bash
# Round 4: k_shift with 32-bit byte offsets (PMC_SHIFT_OFF32=1, default) against the 64-bit form --
# shift/slab parity tests, then the whole-box bench A/B (shift_ms is the k_shift launch time).
# Usage (GPU box, repo root): bash tools/r04q.sh <tag>
set -o pipefail
T=${1:-r04q}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread \
    -k "shift or full_sweeps or slab_driver_equals or halo2 or config4_world8_128_equals or small" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
REPS="1 2 3 4" bash tools/r04_env_ab.sh ${T}_ab "off32:PMC_SHIFT_OFF32=1" "off64:PMC_SHIFT_OFF32=0" || exit 1
