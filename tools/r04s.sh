#!/bin/bash
# Round 4 probe: the whole-box bench without the per-phase fallback launches (PMC_PROBE_NO_FALLBACK).
# Usage (GPU box, repo root): bash tools/r04s.sh <tag>
set -o pipefail
T=${1:-r04s}; O=gpurun_out/$T; mkdir -p $O
REPS="1 2 3 4" bash tools/bench_ab.sh cur nofb 2>&1 | tee $O/nofb_box_ab.txt
