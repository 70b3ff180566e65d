#!/bin/bash
# Round 4, final kernel: the 8-rank rehearsal (local halo copies) with and without the injected 80 us
# delay, default schedule / full-capacity boundary launches / two-plane halos; the halo validation test.
# Usage (GPU box, repo root): bash tools/r04n.sh <tag>
set -o pipefail
T=${1:-r04n}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "halo_parameter" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
R=8 DELAYS="0 80" REPS="1 2 3" bash tools/r04_variants_ab.sh ${T}_ab "base:PMC_SLAB_HALO=1" "bfull:PMC_BOUNDARY_FULL=1" "h2:PMC_SLAB_HALO=2" || exit 1
