#!/bin/bash
# drl_gemm decomposition sweep at the fused-micro-batch row counts (24576 update rows, 49152 log-prob rows).
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
timeout -k 10 600 python -u tools/gemm_sk_bench.py --quick --tune --rows 24576 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail $OUT/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.jsonl'):
    r=json.loads(l); sw=sorted(r['sweep_us'].items(), key=lambda x:x[1])
    print(f\"{r['shape']:20s} {r['M']:6d} {r['N']:6d} {r['K']:6d} lib {r['hipblaslt_us']:7.1f} ours {r['ours_us']:7.1f} ({r['ours_TF']:5.0f}TF) best {sw[0][0]} {sw[0][1]:.1f} | {' '.join(f'{k}:{v:.0f}' for k,v in r['sweep_us'].items())}\")
"
