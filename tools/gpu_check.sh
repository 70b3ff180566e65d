#!/bin/bash
# GPU-box check: parity tests then the default bench line.  Usage: bash tools/gpu_check.sh <tag> [bench args]
set -o pipefail
TAG=${1:-chk}; shift
OUT=gpurun_out/chk_$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py "$@" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value %.4g ms/step %.4f phase %.4f shift %.4f frac %.4f cpu %s' % (d['value'], d['ms_per_step'], r['launch_ms'], r['shift_ms'], r['frac'], (d.get('cpu_baseline') or {}).get('value')))"
