#!/bin/bash
# Memory-side traffic per k_shift launch (shiftCells) in the default bench workload (128^3/1e7):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes, FETCH_SIZE doubled (gfx950).
# Usage (GPU box): bash tools/shift_traffic.sh <tag>
set -o pipefail
O=gpurun_out/shtcc_$1; mkdir -p $O
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 bench.py --steps 4 --warmup 2 --rewarm 0 --no-cpu-baseline > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections, json
root = sys.argv[1]
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = collections.defaultdict(float)
    for f in glob.glob(f"{root}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_shift<" in r["Kernel_Name"] and r["Counter_Name"] == c:
                v[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    out[c] = (sum(v.values()) / len(v), len(v)) if v else (None, 0)
rd = 2 * out["FETCH_SIZE"][0] * 1024; wr = out["WRITE_SIZE"][0] * 1024
print(json.dumps({"k_shift_read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "dispatches": out["FETCH_SIZE"][1]}))
PY
