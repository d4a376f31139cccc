#!/bin/bash
set -o pipefail
OUT=gpurun_out/decattn; mkdir -p $OUT
timeout -k 10 400 python tools/kernel_bench.py --only decode_cold > $OUT/cold.jsonl 2> $OUT/cold.err || { tail -30 $OUT/cold.err; exit 1; }
python -c "
import json
for l in open('$OUT/cold.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['B'], 'auto', d['auto_us'], 'best', d['best'], d['best_us'], d['best_GBps'], sorted(d['sweep_us'].items(), key=lambda x: x[1])[:5])"
