#!/bin/bash
# Memory-side traffic per interior k_subsweep launch of the slab driver, for the launch shapes of the
# N>1 bench lines: config 4 at 2/4/8 ranks (one rank's slab, bench.py --emulate-ranks R: the same
# interior launches a rank of the R-GPU run issues) and config 5 (a 256x256x32 slab).  FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes, FETCH_SIZE doubled (MI355X_MICROARCH.md, gfx950).
# Usage (GPU box, repo root): bash tools/slab_traffic.sh <tag> -> gpurun_out/slabtcc_<tag>/summary.json
set -o pipefail
O=gpurun_out/slabtcc_$1; mkdir -p $O
export TMPDIR=/tmp
B="bench.py --steps 4 --warmup 2 --rewarm 0 --no-cpu-baseline"
for shape in "4:16:--config 4 --emulate-ranks 8" "4:32:--config 4 --emulate-ranks 4" "4:64:--config 4 --emulate-ranks 2" "5:32:--config 5"; do
  key=${shape%%:--*}; args=--${shape#*:--}; d=$O/${key/:/_}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -T --output-format csv -d $d/$c -o run -- python3 $B $args > $d.$c.log 2>&1 || { tail -20 $d.$c.log; exit 1; }
  done
  echo "$key done"
done
python3 - "$O" <<'PY'
import csv, glob, json, os, re, sys, collections
root = sys.argv[1]
out = {}
for d in sorted(glob.glob(root + "/*_*/")):
    key = os.path.basename(d.rstrip("/")).replace("_", ":")
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(float)
        for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"(k_\w+)", r["Kernel_Name"])
                if m and m.group(1) == "k_subsweep" and r["Counter_Name"] == c:
                    vals[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
        per[c] = (sum(vals.values()) / len(vals), len(vals)) if vals else (None, 0)
    rd = 2 * per["FETCH_SIZE"][0] * 1024 if per["FETCH_SIZE"][0] is not None else None
    wr = per["WRITE_SIZE"][0] * 1024 if per["WRITE_SIZE"][0] is not None else None
    out[key] = {"kernel": "k_subsweep (slab interior launches)", "dispatches": per["FETCH_SIZE"][1],
                "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                "subsweep_bytes_per_launch": (rd + wr) if rd is not None and wr is not None else None}
json.dump(out, open(root + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
