#!/bin/bash
# Deterministic embedding backward + SwiGLU-backward epilogue fast path: the GPU suite, the bench, a step profile.
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['timing_s'].items()}, d['roofline']['frac'])"
bash tools/step_profile.sh r03b_prof && grep -A1 -E 'gemm_sk_kernel<4|gemm_sk_kernel<2|indexFunc|embedding' gpurun_out/r03b_prof/trace_summary.txt
