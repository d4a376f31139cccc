#!/bin/bash
# Concurrent weight gradients on / off: the per-rank N = 2 workload and the bench step.
set -o pipefail
OUT=gpurun_out/wg; mkdir -p $OUT
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), round(d['ms_per_step'],1), 'gen', round(t['gen'],3), 'upd', round(t['update_actor'],3))"; }
for W in 0 1; do
  DRL_CONCURRENT_WGRAD=$W timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/n2_$W.log 2>&1 || { tail -30 $OUT/n2_$W.log; exit 1; }
  show $OUT/n2_$W.log "N=2 wgrad_concurrent=$W"
done
DRL_CONCURRENT_WGRAD=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/b512_0.log 2>&1 || { tail -30 $OUT/b512_0.log; exit 1; }
show $OUT/b512_0.log "B512 wgrad_concurrent=0"
