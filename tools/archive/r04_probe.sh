#!/bin/bash
# Round-4 costing probe of VERDICT r3 item 3(i): the default kernel against PMC_PROBE_NO_REPEAT_OLD
# (no old-position terms for a particle's repeat moves: the upper bound of an old-energy cache),
# alternating bench runs; and PMC_SHIFT_NT=1 (nontemporal shiftCells output stores).  Usage (GPU box, repo root): bash tools/archive/r04_probe.sh <tag>
set -o pipefail
T=$1; O=gpurun_out/$T; mkdir -p $O
REPS="1 2 3" bash tools/bench_ab.sh cur norepold shiftnt 2>&1 | tee $O/probe_ab.txt
