#!/bin/bash
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
PMC_SHIFT_YCHUNK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "shift or full_sweeps or slab" > $O/tests_ychunk.log 2>&1 || { tail -30 $O/tests_ychunk.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "slab or multirank or chain_count or world or config4 or parity_leg or rewarm" > $O/tests_slab.log 2>&1 || { tail -30 $O/tests_slab.log; exit 1; }
tail -1 $O/tests_slab.log
tail -1 $O/tests_ychunk.log
REPS="1 2 3" bash tools/r04_env_ab.sh r04e_ab "plain:PMC_SHIFT_YCHUNK=0" "ychunk:PMC_SHIFT_YCHUNK=1"
bash tools/r04_variants_ab.sh r04e_s8 "plain:PMC_SHIFT_YCHUNK=0" "ychunk:PMC_SHIFT_YCHUNK=1"
