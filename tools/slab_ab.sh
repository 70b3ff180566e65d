#!/bin/bash
# A/B of the slab paths (one-rank RCCL weak sweep and the 8-rank strong rehearsal) over library
# variants from tools/build_variant.sh, alternating twice.  Usage: bash tools/slab_ab.sh <variant>...
set -o pipefail
OUT=gpurun_out/slab_ab; mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    L=parallel-monte-carlo_amd/build/variants/lib_$v.so
    PMC_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/${v}_plain_$r.log 2>&1 || exit 1
    PMC_LIB_PATH=$L timeout -k 10 200 python bench.py --slab --self-rccl --no-cpu-baseline > $OUT/${v}_slab_$r.log 2>&1 || exit 1
    PMC_LIB_PATH=$L timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/${v}_emu_$r.log 2>&1 || exit 1
    p=$(grep '^{' $OUT/${v}_plain_$r.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    w=$(grep '^{' $OUT/${v}_slab_$r.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    e=$(grep '^{' $OUT/${v}_emu_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['rank_sweep_ms'], d['full_box_sweep_ms'])")
    echo "$v plain $p slab $w emu8 $e"
  done
done
