#!/bin/bash
# Round 4: Philox round keys formed on the fly in the rare in-visit paths (PMC_RARE_KEYS=1: fewer
# SGPR spills in the move loop) -- parity subset, then the whole-box bench A/B against the
# precomputed keys everywhere (PMC_RARE_KEYS=0).  Usage (GPU box, repo root): bash tools/r04l.sh <tag>
set -o pipefail
T=${1:-r04l}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "full_sweeps or acceptance or move_count or odd_colour or single_colour or all_colour or fallback or small" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
REPS="1 2 3 4" bash tools/bench_ab.sh cur oldkeys 2>&1 | tee $O/keys_ab.txt
