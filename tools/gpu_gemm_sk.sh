#!/bin/bash
# drl_gemm parity tests then the shape sweep vs hipBLASLt (run through gpurun from the repo root).
set -o pipefail
OUT=gpurun_out/gemm_sk; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -15 $OUT/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python -u tools/gemm_sk_bench.py ${BENCH_ARGS} > $OUT/bench.jsonl 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    r=json.loads(l); print(f\"{r['shape']:22s} {r['M']:6d} {r['N']:6d} {r['K']:6d}  lib {r['hipblaslt_us']:8.1f}us {r['hipblaslt_TF']:6.0f}TF  ours {r['ours_us']:8.1f}us {r['ours_TF']:6.0f}TF\", r.get('sweep_us',''))
"
