#!/bin/bash
# GPU box: energy parity tests, timing (tools/energy_timing.py) and SQ instruction counts of k_energy.
# Usage: bash tools/energy_check.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 150 --timeout-method thread -k "full_sweeps or energy or slab or world or lattice or odd" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/energy_timing.py || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/energy_timing.py > /dev/null 2>&1 || exit 1
grep -rh energy $GRAFT_REPO_ROOT/$O/prof --include="*kernel_stats.csv" | cut -c1-250
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM -T --output-format csv -d $GRAFT_REPO_ROOT/$O/sq -o run -- python3 $GRAFT_REPO_ROOT/tools/energy_timing.py > /dev/null 2>&1 || exit 1
