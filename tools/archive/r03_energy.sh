#!/bin/bash
# Round 3 energy: the energy path tests, timing of pmc_energy (new default vs PMC_ENERGY_LEGACY=1,
# alternating) with the oracle check, and rocprofv3 kernel stats of the default.
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "energy_paths or full_sweeps_parity_16 or acceptance or slab_driver_equals" > $O/energy_tests.log 2>&1 || { tail -40 $O/energy_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/energy_tests.log | tail -12
for i in 1 2; do
  timeout -k 10 200 python tools/energy_timing.py > $O/energy_new_$i.log 2>&1 || { tail -20 $O/energy_new_$i.log; exit 1; }
  PMC_ENERGY_LEGACY=1 timeout -k 10 200 python tools/energy_timing.py > $O/energy_legacy_$i.log 2>&1 || { tail -20 $O/energy_legacy_$i.log; exit 1; }
  echo "new:    $(tail -1 $O/energy_new_$i.log | cut -c1-300)"
  echo "legacy: $(tail -1 $O/energy_legacy_$i.log | cut -c1-300)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/energy_timing.py > $O/energy_prof.log 2>&1 || { tail -20 $O/energy_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
