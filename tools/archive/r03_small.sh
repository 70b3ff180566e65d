#!/bin/bash
# Small-box persistent sweeps: parity tests, then timing at 16^3 (and 8^3, 24^3)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "small_box or full_sweeps_parity_16" > $O/small_tests.log 2>&1 || { tail -40 $O/small_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/small_tests.log
for a in "16 10000" "8 1500" "24 40000"; do
  timeout -k 10 120 python tools/small_box_timing.py $a > $O/small_timing_${a// /_}.log 2>&1 || { tail -20 $O/small_timing_${a// /_}.log; exit 1; }
  tail -1 $O/small_timing_${a// /_}.log
done
