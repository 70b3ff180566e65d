#!/bin/bash
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread -k "chain_count" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
PMC_SLAB_RUNK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k "config4 or world_equals" > $O/tests_runk.log 2>&1 || { tail -40 $O/tests_runk.log; exit 1; }
tail -3 $O/tests_runk.log
bash tools/r04_variants_ab.sh r04f_ab "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1"
