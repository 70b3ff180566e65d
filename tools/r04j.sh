#!/bin/bash
# Round 4: two-plane halos (pmc_params.halo = 2, one exchange per sweep) -- GPU tests, then the
# 8-rank rehearsal A/B against one-plane halos with and without an injected 80 us exchange delay,
# then the whole-box bench with and without the global-z wrap cell_geo gained for halo planes.
# Usage (GPU box, repo root): bash tools/r04j.sh <tag>
set -o pipefail
T=${1:-r04j}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread \
    -k "halo2 or restart or config4_world8_128_equals or chain_count" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
R=8 DELAYS="0 80" REPS="1 2" bash tools/r04_variants_ab.sh ${T}_ab "h1:PMC_SLAB_HALO=1" "h2:PMC_SLAB_HALO=2" || exit 1
REPS="1 2 3" bash tools/bench_ab.sh cur nowrap 2>&1 | tee $O/wrap_ab.txt
