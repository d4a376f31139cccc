#!/bin/bash
# decode projections: tests, then every configuration at 512 / 256 rows in situ (24 layers' weights per graph)
set -o pipefail
OUT=gpurun_out/r03z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_decode_gemm_gpu.py tests/test_vt_blocked_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $OUT/t.log | head -20; exit 1; }
timeout -k 10 400 python -u tools/decode_cfg_sweep.py --rows 512 256 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
