#!/bin/bash
# GPU-box round check: all GPU tests, the default bench line, the one-rank RCCL slab bench and the
# strong-scaling rehearsal at 8 and 4 ranks.  Usage (GPU box, repo root): bash tools/round_check.sh <tag>
set -o pipefail
TAG=${1:-k}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
timeout -k 10 300 python bench.py --slab --self-rccl --no-cpu-baseline > $OUT/bench_slab.log 2>&1 || { tail -30 $OUT/bench_slab.log; exit 1; }
timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/emu8.log 2>&1 || { tail -30 $OUT/emu8.log; exit 1; }
timeout -k 10 200 python tools/strong_emulation.py --p2p rccl --ranks 4 > $OUT/emu4.log 2>&1 || { tail -30 $OUT/emu4.log; exit 1; }
for f in bench bench_slab emu8 emu4; do grep '^{' $OUT/$f.log | cut -c1-300; done
