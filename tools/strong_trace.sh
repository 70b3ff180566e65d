set -o pipefail
OUT=gpurun_out/strong_${1:-a}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k slab --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/strong_emulation.py --p2p rccl > $OUT/emu8.log 2>&1 || { tail -30 $OUT/emu8.log; exit 1; }
tail -1 $OUT/emu8.log
timeout -k 10 200 rocprofv3 --kernel-trace -T --output-format csv -d $OUT/trace -o run -- python3 tools/strong_emulation.py --p2p rccl --steps 5 > $OUT/trace.log 2>&1 || exit 1
echo ok
