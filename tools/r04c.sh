#!/bin/bash
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k "chain_count" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/r04_variants_ab.sh r04c_ab "base:PMC_SLAB_CHAINS=2" "bfull:PMC_BOUNDARY_FULL=1" \
  "crit:PMC_BOUNDARY_FULL=1,PMC_SLAB_SPLIT_SHIFT=1,PMC_SLAB_DEFER_Z=1" "critnf:PMC_SLAB_SPLIT_SHIFT=1,PMC_SLAB_DEFER_Z=1"
