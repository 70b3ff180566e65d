#!/bin/bash
# SQ / LDS / TA counter passes on bench.py (one counter group per pass).
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACCUM_PREV_HIRES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -T --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/fail.txt; }
done
echo done > $OUT/ok
