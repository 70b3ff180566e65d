#!/bin/bash
# Kernel trace of the one-rank RCCL slab bench (weak-scaling rank) for tools/timeline.py.
# Usage (GPU box, repo root): bash tools/slab_trace.sh <tag>
set -o pipefail
OUT=gpurun_out/slabtr_${1:-a}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --slab --self-rccl --no-cpu-baseline --steps 4 --warmup 2 > $OUT/trace.log 2>&1 || exit 1
echo ok
