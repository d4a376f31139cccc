#!/bin/bash
# Concurrent weight gradients only for whole-tile ones: tests, the bench, per-rank N = 2 / 4.
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_estimators_gpu.py tests/test_actor_update_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), round(d['ms_per_step'],1), {k: round(v,3) for k,v in t.items()})"; }
for n in 2 4; do
  tb=$((64 / n)); mb=$((32 / n))
  timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=$tb actor_rollout_ref.actor.ppo_mini_batch_size=$mb > $OUT/n$n.log 2>&1 || { tail -30 $OUT/n$n.log; exit 1; }
  show $OUT/n$n.log N=$n
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
show $OUT/bench.log B512
