#!/bin/bash
# Round 3 bench lines: config 3 (driver command), config 4 slab at one rank and as an 8-rank
# rehearsal, config 5 rehearsal -- each with CPU baseline and parity leg.
# Usage (GPU box, repo root): bash tools/archive/r03_bench.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log > $O/$n.json; python3 - $O/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; p = d.get("parity") or {}; c = d.get("cpu_baseline") or {}
print(sys.argv[1].split("/")[-1], "value %.4g ms %.4f launch %s frac %.4f traffic %s parity %s/%s cpu %s vs %s" % (
    d["value"], d["ms_per_step"], r["launch_ms"], r["frac"] or 0, r["traffic"], p.get("state_bitwise_equal"),
    p.get("counters_equal"), c.get("socket_estimate"), d.get("vs_baseline")))
PY
}
run bench3 --gpus 1 --steps 20 --warmup 5
run bench4slab1 --config 4 --slab --self-rccl --steps 20 --warmup 5
run bench4emu8 --config 4 --emulate-ranks 8 --self-rccl --steps 40 --warmup 5
run bench5 --config 5 --steps 10 --warmup 3
