#!/bin/bash
# SQ instruction mix and wave cycles of the energy kernels (tools/energy_timing.py workload), one
# rocprofv3 --pmc pass.  Usage (GPU box): bash tools/energy_sq.sh <tag>
set -o pipefail
O=gpurun_out/esq_$1; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p -o run -- python3 tools/energy_timing.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
python3 tools/pmc_summary.py $O/p | grep k_energy
