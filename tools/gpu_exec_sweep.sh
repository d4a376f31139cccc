#!/bin/bash
# bench step rate vs the fused-execution group sizes (actor / critic exec_activation_gb, log-prob pass tokens)
set -o pipefail
OUT=gpurun_out/execsweep; mkdir -p $OUT
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'ref', round(t.get('ref',0),3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3))"; }
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --override "$@" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  summ $OUT/$name.log $name
}
if [ "${SWEEP:-1}" = 1 ]; then
run base
run a60 actor_rollout_ref.actor.exec_activation_gb=60
run a60_lp98k actor_rollout_ref.actor.exec_activation_gb=60 actor_rollout_ref.actor.exec_log_prob_tokens=98304 actor_rollout_ref.ref.exec_log_prob_tokens=98304
run a120 actor_rollout_ref.actor.exec_activation_gb=120
else
run m16 actor_rollout_ref.actor.exec_micro_batches=16
run m32 actor_rollout_ref.actor.exec_micro_batches=32
run m16_lp196k actor_rollout_ref.actor.exec_micro_batches=16 actor_rollout_ref.actor.exec_log_prob_tokens=196608 actor_rollout_ref.ref.exec_log_prob_tokens=196608
fi
