"""Summarise rocprofv3 counter CSVs: mean counter value per dispatch for each kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if k.startswith("k_"):
        print(f"{k:28s} {c:28s} n={len(v):3d} mean={sum(v)/len(v):.6g}")
