#!/bin/bash
# GPU suite + bench with every model GEMM on drl_gemm, then the GEMM shape sweep.
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputests.log 2>&1; rc=$?; tail -25 $OUT/gputests.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timing_s'], d['roofline']['frac'], d['roofline']['mean_launch_us'])"
timeout -k 10 400 python -u tools/gemm_sk_bench.py > $OUT/gemm.jsonl 2> $OUT/gemm.err || { tail $OUT/gemm.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/gemm.jsonl'):
    r=json.loads(l); print(f\"{r['shape']:22s} {r['M']:6d} {r['N']:6d} {r['K']:6d}  lib {r['hipblaslt_us']:8.1f}us  ours {r['ours_us']:8.1f}us\")
"
