#!/bin/bash
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread -k "chain_count and env7 or chain_count and env8 or chain_count and env9 or chain_count and env10" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PMC_SLAB_RUNK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k "config4 or world_equals or parity_leg" > $O/tests_runk.log 2>&1 || { tail -40 $O/tests_runk.log; exit 1; }
tail -2 $O/tests_runk.log
bash tools/r04_variants_ab.sh r04g_ab "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1"
