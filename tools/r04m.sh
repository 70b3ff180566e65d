#!/bin/bash
# Round 4 A/B: LLVM's max-memory-clause scheduler on the round-4 kernel (tools/build_variant.sh mmc).
# Usage (GPU box, repo root): bash tools/r04m.sh <tag>
set -o pipefail
T=${1:-r04m}; O=gpurun_out/$T; mkdir -p $O
REPS="1 2 3" bash tools/bench_ab.sh cur mmc 2>&1 | tee $O/mmc_ab.txt
