#!/bin/bash
# Round 4: kernel traces of the 8-rank rehearsal (per-stream timelines): 2 chains + split shift +
# 80 us injected delay, 2 chains no delay, 3 chains no delay.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 bench.py --config 4 --emulate-ranks 8 --steps 20 --warmup 5 --no-cpu-baseline $XARGS > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  tail -1 $O/$tag.log | cut -c1-200
}
XARGS="--xfer-delay-us 80" run c2s1d80 PMC_SLAB_CHAINS=2 PMC_SLAB_SPLIT_SHIFT=1
XARGS="" run c2s0d0 PMC_SLAB_CHAINS=2 PMC_SLAB_SPLIT_SHIFT=0
XARGS="" run c3s0d0 PMC_SLAB_CHAINS=3 PMC_SLAB_SPLIT_SHIFT=0
find $O -name "*kernel_trace.csv" | head
# one cell per wave for mid-size phases (PMC_DIRECT_LAUNCH): config 2 (32768 cells per phase) and
# the 8-rank rehearsal's interior chain launches (~14k cells), alternating
for r in 1 2; do for dl in 0 40000; do
  PMC_DIRECT_LAUNCH=$dl timeout -k 10 200 python bench.py --config 2 --steps 160 --warmup 8 --no-cpu-baseline > $O/b2_dl${dl}_$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$O/b2_dl${dl}_$r.json').read().strip().splitlines()[-1]); print('config2 direct=$dl', d['ms_per_step'], d['roofline']['launch_ms'])"
  PMC_DIRECT_LAUNCH=$dl timeout -k 10 200 python bench.py --config 4 --emulate-ranks 8 --steps 100 --warmup 5 --no-cpu-baseline > $O/e8_dl${dl}_$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('$O/e8_dl${dl}_$r.json').read().strip().splitlines()[-1]); print('emu8 direct=$dl', d['ms_per_step'], d['roofline']['launch_ms'])"
done; done
