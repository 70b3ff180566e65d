#!/bin/bash
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k "chain_count or config4 or world_equals" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04_variants_ab.sh r04d_ab "bfirst:PMC_SLAB_B_FIRST=1" "blast:PMC_SLAB_B_FIRST=0" \
  "crit:PMC_BOUNDARY_FULL=1,PMC_SLAB_SPLIT_SHIFT=1,PMC_SLAB_DEFER_Z=1" "critnf:PMC_SLAB_SPLIT_SHIFT=1,PMC_SLAB_DEFER_Z=1" \
  "critnf_bl:PMC_SLAB_SPLIT_SHIFT=1,PMC_SLAB_DEFER_Z=1,PMC_SLAB_B_FIRST=0"
