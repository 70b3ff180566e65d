#!/bin/bash
set -o pipefail
OUT=gpurun_out/series; mkdir -p $OUT
for p in 0 300 2000; do
  timeout -k 10 200 python tools/sweep_series.py --prewarm-ms $p > $OUT/p$p.log 2>&1 || exit 1
  grep '^{' $OUT/p$p.log
done
