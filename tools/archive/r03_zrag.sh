#!/bin/bash
# Ragged z-groups: parity (slab tests) then config 5 and the 8-rank config-4 rehearsal A/B.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_zrag.so timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "world or config4 or slab or single_colour_parity_64" > $O/parity_zrag.log 2>&1 || { tail -30 $O/parity_zrag.log; exit 1; }
echo "zrag parity: $(tail -1 $O/parity_zrag.log)"
CONFIG=5 STEPS=10 bash tools/bench_ab_cfg.sh base zrag
CONFIG=4 EXTRA="--emulate-ranks 8 --self-rccl" STEPS=40 bash tools/bench_ab_cfg.sh base zrag
