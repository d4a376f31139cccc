#!/bin/bash
set -o pipefail
OUT=gpurun_out/alloct; mkdir -p $OUT
for i in 1 2; do
DRL_ALLOC_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/a$i.log 2>&1 || { tail -30 $OUT/a$i.log; exit 1; }
grep '^{' $OUT/a$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v,3) for k,v in d['timing_s'].items()}, d['memory'])"
done
