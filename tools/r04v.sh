#!/bin/bash
# Round 4: two-plane halos with the boundary plane and the redundant halo plane in ONE launch per
# phase on the exchange stream (PMC_SLAB_H2_MERGE=1, default) -- the halo-2 GPU tests, then the
# 8-rank rehearsal: one-plane halos, two-plane merged, two-plane with the R stream, at 0/40/80 us.
# Usage (GPU box, repo root): bash tools/r04v.sh <tag>
set -o pipefail
T=${1:-r04v}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "halo2 or restart or slab_driver_equals or halo_parameter or chain_count" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
R=8 DELAYS="0 40 80" REPS="1 2" bash tools/r04_variants_ab.sh ${T}_ab "h1:PMC_SLAB_HALO=1" "h2m:PMC_SLAB_HALO=2,PMC_SLAB_H2_MERGE=1" "h2r:PMC_SLAB_HALO=2,PMC_SLAB_H2_MERGE=0" || exit 1
