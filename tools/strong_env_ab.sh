# Strong-scaling rehearsal A/B over an environment switch of the product library (same build).
# Usage: ENVVAR=PMC_SLAB_SPLIT_SHIFT VALUES="0 1" REPS="1 2 3" bash tools/strong_env_ab.sh
set -o pipefail
O=gpurun_out/strong_env_ab; mkdir -p $O
for r in ${REPS:-1 2 3}; do for v in ${VALUES:-0 1}; do
  env $ENVVAR=$v timeout -k 10 200 python tools/strong_emulation.py --ranks ${RANKS:-8} > $O/${ENVVAR}_${v}_$r.log 2>&1 || exit 1
  grep '^{' $O/${ENVVAR}_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ENVVAR=$v R${RANKS:-8} full %.4f rank %.4f speedup %.2f host %.3f' % (d['full_box_sweep_ms'], d['rank_sweep_ms'], d['projected_speedup'], d['host_issue_ms_per_sweep']))"
done; done
