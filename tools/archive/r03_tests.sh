#!/bin/bash
# Round 3: the whole GPU suite (with a heartbeat file: the config-5 oracle test is quiet for ~1 min)
# Usage (GPU box, repo root): bash tools/archive/r03_tests.sh <tag> [pytest args]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
( while sleep 20; do date +%T >> $O/heartbeat; done ) & HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 "$@" > $O/tests.log 2>&1
rc=$?
kill $HB
tail -25 $O/tests.log
exit $rc
