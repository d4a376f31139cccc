#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 300 python -u tools/decode_cfg_sweep.py > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
