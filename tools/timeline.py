"""Per-stream kernel timeline of the last sweep in a rocprofv3 --kernel-trace CSV.

  python tools/timeline.py <kernel_trace.csv> [n_last]
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n_last:]
t0 = int(rows[0]["Start_Timestamp"])
qcol = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
for r in rows:
    name = r["Kernel_Name"]
    m = re.search(r"(k_\w+|ncclKernel\w*|\w*[Cc]opy\w*|rccl\w*)", name)
    short = m.group(1) if m else name[:40]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{qcol[:1]}{r[qcol]:>3} {short:34s} start {s/1e3:9.1f} us  dur {(e-s)/1e3:7.1f} us  grid {r.get('Grid_Size', r.get('Grid_Size_X', ''))}")
