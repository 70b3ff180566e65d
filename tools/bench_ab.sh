#!/bin/bash
# A/B of the default bench (full sweeps, the driver's --steps 20 --warmup 5) over library variants
# from tools/build_variant.sh, run alternately (REPS rounds, default 3).
# Usage (GPU box, repo root): bash tools/bench_ab.sh <variant>...
set -o pipefail
OUT=gpurun_out/bench_ab; mkdir -p $OUT
for r in ${REPS:-1 2 3}; do
  for v in "$@"; do
    PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${v}_$r.log 2>&1 || exit 1
    grep '^{' $OUT/${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['launch_ms'], r['shift_ms'])"
  done
done
