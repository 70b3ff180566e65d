#!/bin/bash
# Round 4: kernel traces of the 8-rank rehearsal without and with 80 us injected per exchange, and
# their timeline statistics (tools/timeline_stats.py).  Usage (GPU box, repo root): bash tools/r04x.sh <tag>
set -o pipefail
T=${1:-r04x}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for dl in 0 80; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_d$dl -o run -- python3 bench.py --config 4 --emulate-ranks 8 --steps 40 --warmup 5 --no-cpu-baseline --xfer-delay-us $dl > $O/tr_d$dl.log 2>&1 || { tail -20 $O/tr_d$dl.log; exit 1; }
  python3 tools/timeline_stats.py $(find $O/tr_d$dl -name "*kernel_trace.csv" | head -1) 10 | tee $O/timeline_d$dl.txt
done
