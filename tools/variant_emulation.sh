#!/bin/bash
# A/B of the strong-scaling rehearsal (8 ranks): the default build against a variant library from
# tools/build_variant.sh.  Usage (GPU box, repo root): bash tools/variant_emulation.sh <variant> [tag]
set -o pipefail
V=$1
OUT=gpurun_out/var_${2:-a}; mkdir -p $OUT
timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/base.log 2>&1 || exit 1
PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$V.so timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/$V.log 2>&1 || exit 1
for f in base $V; do grep '^{' $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'])"; done
