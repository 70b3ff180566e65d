#!/bin/bash
# Round 4: the move loop's last partner block in one pass when it holds <= 32 partners
# (PMC_HALF_BLOCK=1) -- parity subset, then the whole-box bench A/B against PMC_HALF_BLOCK=0.
# Usage (GPU box, repo root): bash tools/r04p.sh <tag>
set -o pipefail
T=${1:-r04p}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "full_sweeps or acceptance or move_count or odd_colour or single_colour or all_colour or fallback or small or nmax" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
REPS="1 2 3 4" bash tools/bench_ab.sh cur nohalf 2>&1 | tee $O/half_ab.txt
