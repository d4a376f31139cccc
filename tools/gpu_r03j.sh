#!/bin/bash
# Decode projections at 512 / 256 rows: drl_gemm decompositions vs the packed decode kernels (cold weights).
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
for M in 512 256; do
  timeout -k 10 300 python -u tools/gemm_sk_bench.py --tune --decode $M > $OUT/dec$M.jsonl 2> $OUT/dec$M.err || { tail $OUT/dec$M.err; exit 1; }
done
timeout -k 10 400 python -u tools/kernel_bench.py --only decode_gemm > $OUT/packed.jsonl 2> $OUT/packed.err || { tail $OUT/packed.err; exit 1; }
python3 -c "
import json
for M in (512, 256):
    for l in open(f'$OUT/dec{M}.jsonl'):
        r=json.loads(l); sw=sorted(r['sweep_us'].items(), key=lambda x:x[1])
        print(f\"{r['shape']:20s} {r['M']:5d} lib {r['hipblaslt_us']:7.1f} ours {r['ours_us']:7.1f} best {sw[0][0]} {sw[0][1]:.1f} | {' '.join(f'{k}:{v:.0f}' for k,v in r['sweep_us'].items())}\")
"
grep -E '"M": (256|512)' $OUT/packed.jsonl | cut -c1-300
