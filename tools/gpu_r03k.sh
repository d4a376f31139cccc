#!/bin/bash
# Concurrent weight-gradient stream A/B under fused micro-batch execution.
set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3))"; }
for c in 0 1 0 1; do
  DRL_CONCURRENT_WGRAD=$c timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench_c$c.log 2>&1 || { tail -30 $OUT/bench_c$c.log; exit 1; }
  summ $OUT/bench_c$c.log concurrent$c
done
