#!/bin/bash
# Instruction-cache behaviour of k_subsweep (one colour-phase workload, tools/ablate.py): SQC
# instruction-cache requests, hits, misses and the instruction-fetch counters, one rocprofv3 pass.
# Usage (GPU box): bash tools/icache_counters.sh <tag>
set -o pipefail
OUT=gpurun_out/icc_$1; mkdir -p $OUT
export TMPDIR=/tmp MOVES=10 REPS=3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES -T --output-format csv -d $OUT/p1 -o run -- python3 tools/ablate.py > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].split("<")[0].split("(")[0].endswith("k_subsweep"):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for c in sorted(agg):
    print(f"{c:30s} mean per dispatch {agg[c] / len(n[c]):16.1f}   n={len(n[c])}")
req, miss = agg.get("SQC_ICACHE_REQ", 0), agg.get("SQC_ICACHE_MISSES", 0)
if req:
    print(f"icache miss rate {miss / req:.4f}")
PY
