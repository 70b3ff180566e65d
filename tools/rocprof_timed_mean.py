"""Mean k_subsweep duration over the bench's timed launches in a rocprofv3 kernel trace (the last
steps*8 main launches; the warm-up launches run colder), for comparison with the bench's own
HIP-event launch time.  python tools/rocprof_timed_mean.py <kernel_trace.csv> <steps>"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if r["Kernel_Name"].startswith("void pmc::(anonymous namespace)::k_subsweep<")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
n = 8 * int(sys.argv[2])
t = d[-n:]
print(f"k_subsweep launches {len(d)}; timed {len(t)}: mean {statistics.mean(t):.4f} ms, "
      f"median {statistics.median(t):.4f} ms, min {min(t):.4f} ms; all launches mean {statistics.mean(d):.4f} ms")
