#!/bin/bash
# drl_gemm whole-tile chaining: GEMM tests (race screens included), fixed-cost probe, bench.
set -o pipefail
OUT=gpurun_out/r03q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|assert|Error" $OUT/t.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/probes/sk_overhead.py > $OUT/o.jsonl 2> $OUT/o.err || { tail $OUT/o.err; exit 1; }
cat $OUT/o.jsonl
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3))"; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --roofline-kernel drl_flash_attn_fwd > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
summ $OUT/bench.log chained
