#!/bin/bash
# Decode planner change (qkv + RoPE and short-K partials on the one-round-trip kernel, one-block workgroups):
# decode / rollout parity tests, the planner sweep, the bench, the per-rank N=8 workload.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_decode_gemm_gpu.py tests/test_full_depth_gpu.py tests/test_model_gpu.py tests/test_llama_gpu.py tests/test_vt_blocked_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python tools/decode_cfg_sweep.py --rows 512 256 64 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -30 $OUT/sweep.err; exit 1; }
python -c "
import json
for l in open('$OUT/sweep.jsonl'):
    d=json.loads(l); print(d['rows'], d['proj'], 'planner', d['planner'], 'mb1', d.get('untiled_mb1'))"
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), round(d['ms_per_step'],1), {k: round(v,3) for k,v in t.items()})"; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
show $OUT/bench.log B512
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > $OUT/n8.log 2>&1 || { tail -30 $OUT/n8.log; exit 1; }
show $OUT/n8.log N8
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/n2.log 2>&1 || { tail -30 $OUT/n2.log; exit 1; }
show $OUT/n2.log N2
