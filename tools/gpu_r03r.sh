#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 300 python -u tools/probes/sk_overhead.py > $OUT/o.jsonl 2> $OUT/o.err || { tail $OUT/o.err; exit 1; }
cat $OUT/o.jsonl
