#!/bin/bash
# Memory-side traffic of k_subsweep per launch over the one-phase workload of tools/ablate.py
# (128^3 / 1e7, 10 moves), collected as MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes (they do not fit one pass), FETCH_SIZE doubled (gfx950
# tallies 128 B requests at 64 B), plus the TCC_EA0 request-size split that checks that correction.
# Infinity-Cache hits are counted (fabric traffic, an upper bound on HBM bytes).
# Usage (GPU box, repo root): bash tools/tcc_traffic.sh <tag>  -> gpurun_out/tcc_<tag>/summary.json
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out/tcc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp MOVES=10 REPS=3
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
           "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d $OUT/p$i -o run -- python3 tools/ablate.py > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
rows = [(f, r) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if "k_subsweep" in r["Kernel_Name"] and "fallback" not in r["Kernel_Name"]]
# whole colour phases only: the equilibration sweeps may split phases over plane chains (smaller grids)
grid = max(int(r["Grid_Size"]) for _, r in rows)
for f, r in rows:
    if int(r["Grid_Size"]) == grid:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
per = {c: tot[c] / len(disp[c]) for c in tot}
per["grid_size"] = grid
fetch = 2 * per.get("FETCH_SIZE", 0) * 1024          # KiB, doubled (gfx950 correction)
write = per.get("WRITE_SIZE", 0) * 1024              # KiB
req = per.get("TCC_EA0_RDREQ_32B", 0) * 32 + per.get("TCC_EA0_RDREQ_64B", 0) * 64 + per.get("TCC_EA0_RDREQ_128B", 0) * 128
out = {"kernel": "k_subsweep", "counters_per_launch": per,
       "read_bytes_per_launch": fetch, "write_bytes_per_launch": write,
       "traffic_bytes_per_launch": fetch + write,
       "read_bytes_from_request_sizes": req,
       "note": "FETCH_SIZE x 2 x 1024 (KiB; gfx950 tallies 128 B requests at 64 B) + WRITE_SIZE x 1024, "
               "separate passes (MI355X_MICROARCH.md HBM section); read_bytes_from_request_sizes = "
               "TCC_EA0_RDREQ_{32,64,128}B x size cross-checks the doubling; Infinity-Cache hits included"}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
