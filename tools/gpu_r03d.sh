#!/bin/bash
# Decode-path A/B at 512 rows (packed decode GEMMs vs the unpacked step on drl_gemm) and at 64 rows (per-rank N=8).
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'prefill', round(t['generate_prefill'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3))"; }
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override actor_rollout_ref.rollout.packed_decode_max_rows=256 > $OUT/unpacked512.log 2>&1 || { tail -30 $OUT/unpacked512.log; exit 1; }
summ $OUT/unpacked512.log unpacked512
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > $OUT/packed64.log 2>&1 || { tail -30 $OUT/packed64.log; exit 1; }
summ $OUT/packed64.log packed64
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 actor_rollout_ref.rollout.packed_decode=False > $OUT/unpacked64.log 2>&1 || { tail -30 $OUT/unpacked64.log; exit 1; }
summ $OUT/unpacked64.log unpacked64
