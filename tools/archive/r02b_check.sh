set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
(lscpu; nproc; cat /sys/fs/cgroup/cpu.max; echo OMP=$OMP_NUM_THREADS) > $O/host.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench3.log 2>&1 || { tail -30 $O/bench3.log; exit 1; }
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $O/bench5.log 2>&1 || { tail -30 $O/bench5.log; exit 1; }
timeout -k 10 400 python bench.py --config 5box --steps 10 > $O/bench5box.log 2>&1 || { tail -30 $O/bench5box.log; exit 1; }
for f in bench3 bench5 bench5box; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; p=d.get('parity') or {}; print('$f value %.4g ms/step %.4f phase %s frac %s cpu %s serial %s parity %s' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], c.get('value'), (c.get('serial') or {}).get('value'), p.get('state_bitwise_equal')))"; done
