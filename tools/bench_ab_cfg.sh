#!/bin/bash
# bench_ab.sh for another bench config: CONFIG=5box bash tools/bench_ab_cfg.sh <variant>...
set -o pipefail
OUT=gpurun_out/bench_ab_cfg; mkdir -p $OUT
for r in ${REPS:-1 2}; do
  for v in "$@"; do
    PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 300 python bench.py --config ${CONFIG:-5box} ${EXTRA} --steps ${STEPS:-10} --no-cpu-baseline > $OUT/${CONFIG}_${v}_$r.log 2>&1 || exit 1
    grep '^{' $OUT/${CONFIG}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('${CONFIG:-5box} $v', d['value'], d['ms_per_step'], r['launch_ms'], r['shift_ms'])"
  done
done
