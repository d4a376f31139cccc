#!/bin/bash
# drl_gemm epilogue changes: GEMM tests (layouts, decompositions, race screens), then the per-tile fixed-cost probe
set -o pipefail
OUT=gpurun_out/r03w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gemm_sk_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/t.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/probes/sk_overhead.py > $OUT/o.jsonl 2> $OUT/o.err || { tail $OUT/o.err; exit 1; }
cat $OUT/o.jsonl
