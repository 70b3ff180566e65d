"""Summarise a tools/profile_subsweep.sh run into profiles/.

  python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied verbatim)
  profiles/<tag>_pmc.txt            per-kernel mean of every collected counter
  profiles/<tag>_fetch_write_size.json   FETCH_SIZE / WRITE_SIZE per k_subsweep launch (a cross-check:
                                    bench.py's roofline.traffic comes from profiles/pmc_traffic.json,
                                    written from tools/tcc_traffic.sh's TCC_EA0 request counts)

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch and come from separate passes (they cannot share
one on gfx950).  MI355X_MICROARCH.md: FETCH_SIZE reads exactly half the bytes of a 16-B-per-lane
streaming read; other access widths are uncalibrated.  The subsweep's loads are 4-B-per-lane
dword rows (64 B per 16 lanes), so both the raw value and the x2-corrected upper estimate are
recorded; bench.py reports the raw sum and names the caveat.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(root):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main():
    root, tag = sys.argv[1], sys.argv[2]
    out = os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(root, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats.csv"))
    agg = counters(root)
    lines = []
    for (k, c), v in sorted(agg.items()):
        if k.startswith("k_"):
            lines.append(f"{k:24s} {c:26s} n={len(v):4d} mean={sum(v) / len(v):.6g}")
    with open(os.path.join(out, f"{tag}_pmc.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    fetch = agg.get(("k_subsweep", "FETCH_SIZE"))
    write = agg.get(("k_subsweep", "WRITE_SIZE"))
    if fetch and write:
        fkb = sum(fetch) / len(fetch)
        wkb = sum(write) / len(write)
        traffic = {
            "kernel": "k_subsweep",
            "tag": tag,
            "fetch_bytes_per_launch": fkb * 1024.0,
            "write_bytes_per_launch": wkb * 1024.0,
            "subsweep_bytes_per_launch": (fkb + wkb) * 1024.0,
            "subsweep_bytes_per_launch_fetch_x2": (2.0 * fkb + wkb) * 1024.0,
            "note": "rocprofv3 FETCH_SIZE+WRITE_SIZE (KiB x 1024), separate passes; raw, the gfx950 x2 "
                    "FETCH correction is calibrated only for 16-B/lane streams (upper estimate given)",
        }
        with open(os.path.join(out, f"{tag}_fetch_write_size.json"), "w") as f:
            json.dump(traffic, f, indent=1)
        print(json.dumps(traffic))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
