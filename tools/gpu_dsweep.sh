#!/bin/bash
set -o pipefail
OUT=gpurun_out/dsweep; mkdir -p $OUT
timeout -k 10 400 python tools/decode_cfg_sweep.py --rows 512 256 64 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail -30 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
