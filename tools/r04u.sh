#!/bin/bash
# Round 4 probe: the 8-rank rehearsal without the boundary chain's phase launches (PMC_PROBE_SKIP_B=1,
# wrong results; exchanges kept) -- the most that folding the boundary planes into the interior chains
# could save.  Usage (GPU box, repo root): bash tools/r04u.sh <tag>
set -o pipefail
T=${1:-r04u}
R=8 DELAYS="0 80" REPS="1 2 3" bash tools/r04_variants_ab.sh ${T}_ab "base:PMC_PROBE_SKIP_B=0" "skipb:PMC_PROBE_SKIP_B=1"
