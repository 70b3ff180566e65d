#!/bin/bash
# Profile the default bench command on one MI355X: kernel trace + stats, then HBM counters in
# separate passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), then SQ counters.
# Usage (on the GPU box, from the repo root): bash tools/profile_subsweep.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -T --output-format csv -d $OUT/sq -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/sq2 -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq2.log 2>&1 || exit $?
echo done > $OUT/ok
