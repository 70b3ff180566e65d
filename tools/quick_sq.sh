#!/bin/bash
# One rocprofv3 counter pass over a short bench run: per-wave VALU/SALU/LDS counts, busy cycles.
# Usage (GPU box, repo root): bash tools/quick_sq.sh <tag>
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU -T --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/run.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in ("k_subsweep", "k_shift"):
    d = {c: sum(v) / len(v) for (kk, c), v in agg.items() if kk == k}
    if not d:
        continue
    w = d.get("SQ_WAVES", 1)
    print(k, {c: round(v / w, 1) if c.startswith("SQ_INSTS") else v for c, v in sorted(d.items())})
PY
