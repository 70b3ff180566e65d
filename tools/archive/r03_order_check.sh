#!/bin/bash
# Round 3: the create-ordering test against the round-2 library (expected to expose the race) and
# the current one, then the whole GPU suite.  Usage (GPU box, repo root): bash tools/archive/r03_order_check.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
T="python -u -m pytest tests/test_gpu_parity.py -k busy_null_stream -v --timeout 120 --timeout-method thread"
PMC_LIB_PATH=$PWD/tools/old_lib/libpmc_r02.so timeout -k 10 150 $T > $O/order_old.log 2>&1
echo "old library: exit $?"; grep -E "PASS|FAIL|assert" $O/order_old.log | head -5
timeout -k 10 150 $T > $O/order_new.log 2>&1 || { tail -30 $O/order_new.log; exit 1; }
echo "new library: pass"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
