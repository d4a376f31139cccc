#!/bin/bash
# Decode row lanes: parity tests, then the bench step and the per-rank N=8 workload at 1 / 2 / 4 lanes.
set -o pipefail
OUT=gpurun_out/lanes; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_decode_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), round(d['ms_per_step'],1), 'gen', round(t['gen'],3), 'prefill', round(t['generate_prefill'],3), 'upd', round(t['update_actor'],3))"; }
for L in ${LANES:-1 2 4}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --override actor_rollout_ref.rollout.decode_lanes=$L > $OUT/bench_l$L.log 2>&1 || { tail -30 $OUT/bench_l$L.log; exit 1; }
  show $OUT/bench_l$L.log "B512 lanes=$L"
done
for L in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 actor_rollout_ref.rollout.decode_lanes=$L > $OUT/n8_l$L.log 2>&1 || { tail -30 $OUT/n8_l$L.log; exit 1; }
  show $OUT/n8_l$L.log "B64 lanes=$L"
done
