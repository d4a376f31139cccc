#!/bin/bash
# The per-rank N = 2 workload: device allocations inside the timed region, default allocator vs expandable segments.
set -o pipefail
OUT=gpurun_out/n2mem; mkdir -p $OUT
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['ms_per_step'],1), 'gen', round(t['gen'],3), 'upd', round(t['update_actor'],3), d['memory'])"; }
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/a.log 2>&1 || { tail -30 $OUT/a.log; exit 1; }
show $OUT/a.log "N=2 default"
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/b.log 2>&1 || { tail -30 $OUT/b.log; exit 1; }
show $OUT/b.log "N=2 expandable"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/c.log 2>&1 || { tail -30 $OUT/c.log; exit 1; }
show $OUT/c.log "B512 default"
