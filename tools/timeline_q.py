"""Per-queue kernel timeline of sweep k (counted from the end) in a rocprofv3 --kernel-trace CSV of
a slab run: the kernels between two consecutive context-stream shiftCells launches.

  python tools/timeline_q.py <kernel_trace.csv> [k_from_end=3]
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
main_q = min(int(r["Queue_Id"]) for r in rows if "k_shift" in r["Kernel_Name"])
shifts = [r for r in rows if "k_shift" in r["Kernel_Name"] and int(r["Queue_Id"]) == main_q]
a, b = int(shifts[-k - 1]["End_Timestamp"]), int(shifts[-k]["End_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= a or s >= b:
        continue
    m = re.search(r"(k_\w+|ncclKernel\w*|\w*[Cc]opy\w*|rccl\w*)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    print(f"Q{r['Queue_Id']} {name:28s} {(s - a) / 1e3:8.1f} -> {(e - a) / 1e3:8.1f} us  ({(e - s) / 1e3:6.1f})  grid {r['Grid_Size_X']}")
print(f"sweep {(b - a) / 1e3:.1f} us")
