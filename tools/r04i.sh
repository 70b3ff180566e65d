#!/bin/bash
set -o pipefail
V=$PWD/parallel-monte-carlo_amd/build/variants
PMC_SLAB_RUNK=1 PMC_LIB_PATH=$V/lib_runk_static.so timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -k "config4" > gpurun_out/r04i_static_tests.log 2>&1 || { tail -30 gpurun_out/r04i_static_tests.log; exit 1; }
tail -1 gpurun_out/r04i_static_tests.log
R=8 DELAYS="0" REPS="1 2" bash tools/r04_variants_ab.sh r04i_ab8 "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1" "static:PMC_SLAB_RUNK=1,PMC_LIB_PATH=$V/lib_runk_static.so"
R=1 DELAYS="0" REPS="1 2" STEPS=30 bash tools/r04_variants_ab.sh r04i_ab1 "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1" "static:PMC_SLAB_RUNK=1,PMC_LIB_PATH=$V/lib_runk_static.so"
