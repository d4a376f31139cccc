#!/bin/bash
# concurrent weight gradients by default + union-of-intervals roofline: model-level suites and a bench line
set -o pipefail
OUT=gpurun_out/r03ab; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_actor_update_gpu.py tests/test_critic_gpu.py tests/test_rmpad_gpu.py tests/test_dp_gpu.py tests/test_llama_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/t.log | head -20; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; r=d['roofline']; print(round(d['value'],4), {k: round(v,3) for k,v in t.items()}, round(r['frac'],3), round(r['mean_launch_us'],1), round(r['busy_us_per_launch'],1), d['memory'])"
