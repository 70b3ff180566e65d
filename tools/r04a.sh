#!/bin/bash
# Round 4, first GPU call: chain-count / split-shift parity, energy + small-box + parity-leg tests,
# strong-scaling A/B (chains x split x injected delay), config 2 line.
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "chain_count or config4 or energy or small_box or parity_leg" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
CHAINS="2 3" DELAYS="0 80" REPS="1 2" bash tools/r04_strong_ab.sh r04a_strong || exit 1
PMC_SLAB_SPLIT_SHIFT=1 CHAINS="2 3" DELAYS="0 80" REPS="1" bash tools/r04_strong_ab.sh r04a_strong_split || exit 1
timeout -k 10 300 python bench.py --config 2 --steps 160 --warmup 8 > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity'])"
