set -o pipefail
OUT=gpurun_out/weak_b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k slab --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/plain.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --slab --self-rccl --no-cpu-baseline > $OUT/slab.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --slab --self-rccl --no-cpu-baseline > $OUT/slab2.log 2>&1 || exit 1
for f in plain slab slab2; do grep '^{' $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
bash tools/slab_trace.sh b
