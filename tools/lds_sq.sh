#!/bin/bash
# LDS-pipe counters of the subsweep per library variant (one rocprofv3 --pmc pass each over a short
# bench run).  Usage (GPU box, repo root): bash tools/lds_sq.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/lds_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for v in "$@"; do
  PMC_LIB_PATH=$PWD/parallel-monte-carlo_amd/build/variants/lib_$v.so timeout -s KILL 200 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES} --output-format csv -d $OUT/$v -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/run_$v.log 2>&1 || exit $?
  f=$(find $OUT/$v -name "*counter_collection.csv" | head -1)
  echo "== $v"; python3 tools/sq_summary.py "$f" k_subsweepILi16ELi16ELb1 262144
done
