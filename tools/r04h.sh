#!/bin/bash
set -o pipefail
V=$PWD/parallel-monte-carlo_amd/build/variants
DELAYS="0" REPS="1 2" bash tools/r04_variants_ab.sh r04h_ab "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1" \
  "plain:PMC_SLAB_RUNK=1,PMC_LIB_PATH=$V/lib_runk_plain.so" "nowait:PMC_SLAB_RUNK=1,PMC_LIB_PATH=$V/lib_runk_nowait.so" \
  "both:PMC_SLAB_RUNK=1,PMC_LIB_PATH=$V/lib_runk_both.so"
R=4 DELAYS="0" REPS="1 2" bash tools/r04_variants_ab.sh r04h_ab4 "base:PMC_SLAB_RUNK=0" "runk:PMC_SLAB_RUNK=1"
