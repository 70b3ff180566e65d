"""Mean k_subsweep duration over the bench's timed launches in a rocprofv3 kernel trace (the last
steps*8*chains main launches; the warm-up launches run colder), for comparison with the bench's own
HIP-event launch time.  pmc_sweep's plane chains split each colour phase into `chains` launches.
  python tools/rocprof_timed_mean.py <kernel_trace.csv | rocprofv3 output dir> [steps] [chains]"""
import csv
import glob
import os
import statistics
import sys

src = sys.argv[1]
if os.path.isdir(src):
    src = sorted(glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True))[-1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
chains = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = [r for r in csv.DictReader(open(src))
        if r["Kernel_Name"].startswith("void pmc::(anonymous namespace)::k_subsweep<")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
t = d[-8 * steps * chains:]
print(f"{src}: k_subsweep launches {len(d)}; timed {len(t)}: mean {statistics.mean(t):.4f} ms, "
      f"median {statistics.median(t):.4f} ms, min {min(t):.4f} ms; all launches mean {statistics.mean(d):.4f} ms")
