"""Per-launch averages of rocprofv3 --pmc counters by kernel: python tools/sq_summary.py <counter_collection.csv> [name filter] [cells per launch]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cells = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"]
    if flt not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for k, v in agg.items():
    n = len(disp[k]) or 1
    out = {c: v[c] / n for c in sorted(v)}
    print(k[:90], "launches", n)
    for c, x in out.items():
        print(f"   {c:22s} {x:16.1f}" + (f"   per cell {x / cells:10.2f}" if cells else ""))
