#!/bin/bash
# whole-tile drl_gemm as one workgroup per tile: GEMM tests, then the bench with and without the side-stream weight
# gradient
set -o pipefail
OUT=gpurun_out/r03aa; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_decode_gemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/t.log | head -20; exit 1; }
summ() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print('$2', round(d['value'],4), 'gen', round(t['gen'],3), 'logp', round(t['old_log_prob'],3), 'upd', round(t['update_actor'],3), 'step', round(t['step'],3), round(d['roofline']['frac'],3))"; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b0.log 2>&1 || { tail -20 $OUT/b0.log; exit 1; }
summ $OUT/b0.log concurrent_off
DRL_CONCURRENT_WGRAD=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b1.log 2>&1 || { tail -20 $OUT/b1.log; exit 1; }
summ $OUT/b1.log concurrent_on
