#!/bin/bash
# Memory-side traffic of k_subsweep by request size (TCC_EA0_* counters, separate passes of <= 4 TCC
# counters each) over the one-phase workload of tools/ablate.py (128^3 / 1e7, 10 moves).
# Usage (GPU box, repo root): bash tools/tcc_traffic.sh <tag>  -> gpurun_out/tcc_<tag>/summary.json
set -o pipefail
TAG=${1:-t}
OUT=gpurun_out/tcc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp MOVES=10 REPS=3
i=0
for set in "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
           "TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B" \
           "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" \
           "TCC_EA0_WRREQ_WRITE_DRAM TCC_EA0_WRREQ_WRITE_DRAM_32B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d $OUT/p$i -o run -- python3 tools/ablate.py > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if k.startswith("k_subsweep") and "fallback" not in k:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
per = {c: tot[c] / len(disp[c]) for c in tot}
rd = per.get("TCC_EA0_RDREQ_32B", 0) * 32 + per.get("TCC_EA0_RDREQ_64B", 0) * 64 + per.get("TCC_EA0_RDREQ_128B", 0) * 128
wr = (per.get("TCC_EA0_WRREQ", 0) - per.get("TCC_EA0_WRREQ_64B", 0)) * 32 + per.get("TCC_EA0_WRREQ_64B", 0) * 64
dram_rd = per.get("TCC_EA0_RDREQ_DRAM_32B", 0) * 32 + (per.get("TCC_EA0_RDREQ_DRAM", 0) - per.get("TCC_EA0_RDREQ_DRAM_32B", 0)) * 64
out = {"kernel": "k_subsweep", "counters_per_launch": per,
       "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
       "dram_read_bytes_per_launch_est": dram_rd,
       "note": "memory-side (L2->fabric) requests by size: RDREQ_32B*32 + RDREQ_64B*64 + RDREQ_128B*128, "
               "WRREQ: 64B requests*64 + the rest*32; Infinity-Cache hits are included (MI355X_MICROARCH.md)"}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
