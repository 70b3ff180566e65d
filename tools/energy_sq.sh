#!/bin/bash
# SQ instruction mix and wait cycles of k_energy (tools/energy_timing.py, 128^3 / 1e7).
# Usage (GPU box, repo root): bash tools/energy_sq.sh <tag>
set -o pipefail
OUT=gpurun_out/esq_$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -T --output-format csv -d $OUT/p1 -o run -- python3 tools/energy_timing.py > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/p2 -o run -- python3 tools/energy_timing.py > $OUT/p2.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_energy" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
cells = 128 ** 3
for c in sorted(agg):
    m = agg[c] / len(n[c])
    print(f"{c:24s} per dispatch {m:14.1f}  per cell {m / cells:9.2f}")
PY
