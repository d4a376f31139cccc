#!/bin/bash
# Fused micro-batch execution: actor-update parity tests, then the bench A/B (exec_micro_batches auto vs 1).
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_critic_gpu.py tests/test_actor_update_gpu.py tests/test_rmpad_gpu.py tests/test_gemm_sk_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -5 $OUT/t.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -30; exit 1; }
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3))"; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench_fused.log 2>&1 || { tail -30 $OUT/bench_fused.log; exit 1; }
summ $OUT/bench_fused.log fused
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd --override actor_rollout_ref.actor.exec_micro_batches=1 actor_rollout_ref.actor.exec_log_prob_tokens=0 actor_rollout_ref.ref.exec_log_prob_tokens=0 > $OUT/bench_plain.log 2>&1 || { tail -30 $OUT/bench_plain.log; exit 1; }
summ $OUT/bench_plain.log per_micro_batch
DRL_GEMM=hipblaslt timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench_lib.log 2>&1 || { tail -30 $OUT/bench_lib.log; exit 1; }
summ $OUT/bench_lib.log hipblaslt_fused
