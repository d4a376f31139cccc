#!/bin/bash
# Round-3 first GPU pass: the GPU suite, the default bench line, then config #5 (Qwen2.5-7B DAPO) one step.
set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timing_s'], d['roofline']['frac'], d['roofline_k1']['frac'], d['roofline_k1_two_pass']['frac'])"
timeout -k 10 500 python bench.py --dapo --steps 1 --warmup 1 --no-cpu-baseline > $OUT/dapo.log 2>&1 || { tail -30 $OUT/dapo.log; exit 1; }
grep '^{' $OUT/dapo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'], d['value'], d['ms_per_step'], d['timing_s'])"
