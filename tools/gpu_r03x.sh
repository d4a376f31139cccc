#!/bin/bash
# model-level suites on the current library, then a bench line
set -o pipefail
OUT=gpurun_out/r03x; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_actor_update_gpu.py tests/test_llama_gpu.py tests/test_gemm_gpu.py tests/test_wide_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/t.log | head -20; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing_s']; print(round(d['value'],4), d['roofline']['frac'], {k: round(v,3) for k,v in t.items()})"
