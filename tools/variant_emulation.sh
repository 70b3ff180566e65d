set -o pipefail
OUT=gpurun_out/var_a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k forced_fallback --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/base.log 2>&1 || exit 1
PMC_LIB_PATH=parallel-monte-carlo_amd/build/variants/lib_cpw1.so timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/cpw1.log 2>&1 || exit 1
for f in base cpw1; do grep '^{' $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'])"; done
