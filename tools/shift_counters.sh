#!/bin/bash
# Counters of k_shift (shiftCells) in the default bench workload (128^3/1e7): memory-side traffic
# (FETCH_SIZE x 2 for gfx950, WRITE_SIZE; separate rocprofv3 passes) and the wave-state counters
# that say what a shift wave spends its life on (issue vs waiting).  Usage (GPU box): bash tools/shift_counters.sh <tag>
set -o pipefail
O=gpurun_out/shcnt_$1; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps 4 --warmup 2 --rewarm 0 --no-cpu-baseline > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
}
run p1 FETCH_SIZE || exit 1
run p2 WRITE_SIZE || exit 1
run p3 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU || exit 1
run p4 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections, json
root = sys.argv[1]
per = collections.defaultdict(dict)
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_shift<" in r["Kernel_Name"] or "k_shift_run<" in r["Kernel_Name"]:
            vals[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in vals.items():
        per[c].setdefault(f, []).append(v)
mean = {c: sum(sum(v) for v in fs.values()) / sum(len(v) for v in fs.values()) for c, fs in per.items()}
out = {"kernel": "k_shift_run<16,4> (shiftCells, 128^3 / 1e7; k_shift<16,8> with PMC_SHIFT_RUN=0)", "counters_per_launch": mean}
if "FETCH_SIZE" in mean:
    out["read_bytes_per_launch"] = 2 * mean["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in mean:
    out["write_bytes_per_launch"] = mean["WRITE_SIZE"] * 1024
if "SQ_WAVE_CYCLES" in mean:
    wc = mean["SQ_WAVE_CYCLES"]
    out["wait_any_fraction_of_wave_cycles"] = mean.get("SQ_WAIT_ANY", 0) / wc
    out["wait_inst_any_fraction_of_wave_cycles"] = mean.get("SQ_WAIT_INST_ANY", 0) / wc
    out["active_valu_fraction_of_wave_cycles"] = mean.get("SQ_ACTIVE_INST_VALU", 0) / wc
    out["active_any_fraction_of_wave_cycles"] = mean.get("SQ_ACTIVE_INST_ANY", 0) / wc
if "SQ_BUSY_CYCLES" in mean and "SQ_WAVE_CYCLES" in mean:
    out["mean_resident_waves_per_busy_cycle"] = mean["SQ_WAVE_CYCLES"] / mean["SQ_BUSY_CYCLES"]
if "GRBM_GUI_ACTIVE" in mean:
    out["launch_cycles_per_xcd"] = mean["GRBM_GUI_ACTIVE"] / 8
out["note"] = ("rocprofv3 sums over the 8 XCDs; SQ_*_CYCLES count in units of the SQ clock per the MI355X guide's "
               "caveats; fractions are of the summed wave lifetime (SQ_WAVE_CYCLES)")
json.dump(out, open(f"{root}/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
