#!/bin/bash
# Strong-scaling rehearsal (8 ranks) over library variants, alternating.  Usage: bash tools/strong_ab.sh <variant>...
set -o pipefail
O=gpurun_out/strong_ab; mkdir -p $O
for r in ${REPS:-1 2}; do for v in "$@"; do
  PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -k 10 200 python tools/strong_emulation.py --ranks 8 > $O/${v}_$r.log 2>&1 || exit 1
  grep '^{' $O/${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v R8 full %.4f rank %.4f speedup %.2f host %.3f' % (d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'], d['host_issue_ms_per_sweep']))"
done; done
