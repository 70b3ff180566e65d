#!/bin/bash
# Two rocprofv3 counter passes over one colour-phase workload (tools/ablate.py, 128^3/1e7, 10
# moves): instruction mix and issue/wait cycles of k_subsweep.  Usage: bash tools/sq_counters.sh tag
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/sqc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp MOVES=10 REPS=3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INST_CYCLES_SALU -T --output-format csv -d $OUT/p1 -o run -- python3 tools/ablate.py > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv -d $OUT/p2 -o run -- python3 tools/ablate.py > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/p3 -o run -- python3 tools/ablate.py > $OUT/p3.log 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
rows = [(f, r) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1] == "k_subsweep"]
# whole colour phases only: the equilibration sweeps may split phases over plane chains (smaller grids)
grid = max(int(r["Grid_Size"]) for _, r in rows)
for f, r in rows:
    if int(r["Grid_Size"]) == grid:
        agg[((f, r["Dispatch_Id"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (d, c), v in agg.items():
    per[c].append(sum(v))
mean = {c: sum(v) / len(v) for c, v in per.items()}
for c in sorted(mean):
    print(f"{c:28s} mean per dispatch {mean[c]:14.1f}   n={len(per[c])}")
cells = 2 * mean.get("SQ_WAVES", 0)   # two cells per wave in the main launch
if cells:
    print("per cell visit: " + ", ".join(f"{c} {mean[c] / cells:.1f}" for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS") if c in mean))
PY
