#!/bin/bash
# per-rank N=2 workload (256 sequences) under different fused-execution budgets
set -o pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3), {k: round(v, 1) for k, v in d['memory'].items()})"; }
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  summ $OUT/$name.log $name
}
run n2_default
run n2_a60 actor_rollout_ref.actor.exec_activation_gb=60
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True run n2_expandable
summ0() { :; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/n1.log 2>&1 || { tail -20 $OUT/n1.log; exit 1; }
summ $OUT/n1.log n1_default
