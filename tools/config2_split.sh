#!/bin/bash
# rocprofv3 counter passes over tools/config2_split.py (separate passes per the MI355X guide's HBM
# section): per dispatch FETCH_SIZE (x2 for gfx950), WRITE_SIZE, TCC hits and misses, for the full
# config-2 phase and its two plane halves.  Usage (GPU box, repo root): bash tools/config2_split.sh TAG
set -o pipefail
O=gpurun_out/c2split_$1; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/config2_split.py > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, json, sys, collections
root = sys.argv[1]
by = collections.defaultdict(lambda: collections.defaultdict(list))   # grid -> counter -> values
for f in glob.glob(root + "/p*/**/*counter_collection.csv", recursive=True):
    vals = collections.defaultdict(float)
    grids = {}
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void pmc::(anonymous namespace)::k_subsweep<"):
            vals[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            grids[r["Dispatch_Id"]] = int(r["Grid_Size"])
    for (d, c), v in vals.items():
        by[grids[d]][c].append(v)
out = {}
for grid, cs in sorted(by.items(), reverse=True):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {"dispatches": max(len(v) for v in cs.values()), "counters": m}
    if "FETCH_SIZE" in m: e["read_MB"] = 2 * m["FETCH_SIZE"] * 1024 / 1e6
    if "WRITE_SIZE" in m: e["write_MB"] = m["WRITE_SIZE"] * 1024 / 1e6
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        e["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    out[f"grid {grid}"] = e
print(json.dumps(out, indent=1))
json.dump(out, open(root + "/summary.json", "w"), indent=1)
PY
