#!/bin/bash
# Round 3: strong-scaling rehearsal at 8 ranks with the host restricted to 2 CPUs (an 8-GPU node's
# 16-CPU quota / 8 ranks) against the unrestricted one, alternating.  Usage: bash tools/archive/r03_host.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for c in 0 2; do
    timeout -k 10 200 python tools/strong_emulation.py --ranks 8 --cpus $c > $O/emu8_cpus$c.$i.log 2>&1 || { tail -20 $O/emu8_cpus$c.$i.log; exit 1; }
    grep '^{' $O/emu8_cpus$c.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cpus=$c run $i: full %.4f rank %.4f speedup %.2f host_issue %.3f host_only %.3f aff %s' % (d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'], d['host_issue_ms_per_sweep'], d['host_only_ms_per_sweep'], d['cpu_affinity']))"
  done
done
timeout -k 10 200 python tools/strong_emulation.py --ranks 4 --cpus 2 > $O/emu4_cpus2.log 2>&1 && grep '^{' $O/emu4_cpus2.log | cut -c1-400
