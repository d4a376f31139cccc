#!/bin/bash
# Configs #5 / #4 architectures at FULL size on one MI355X (GRPO step, tiny batch): Qwen2.5-7B (head_dim 128, 28 / 4
# heads) and Llama-3-8B (no qkv bias, untied lm_head), random init; the step's timings and peak memory.
set -o pipefail
OUT=gpurun_out/size; mkdir -p $OUT
COMMON="data.train_batch_size=4 actor_rollout_ref.rollout.n=2 actor_rollout_ref.actor.ppo_mini_batch_size=4 \
actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=2 actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=4 \
actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=4 data.max_response_length=64 actor_rollout_ref.rollout.response_length=64"
for M in ${MODELS:-llama-3-8b qwen2.5-7b}; do
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --override actor_rollout_ref.model.path=random:$M $COMMON \
    > $OUT/$M.log 2>&1 || { tail -20 $OUT/$M.log; exit 1; }
  grep '^{' $OUT/$M.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$M', round(d['ms_per_step']), 'ms/step', {k: round(v, 3) for k, v in d['timing_s'].items()})"
done
