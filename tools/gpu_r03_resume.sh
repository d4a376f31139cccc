#!/bin/bash
# Round-3 re-entry check on the rebuilt library: the GPU suite, smoke(), the default bench line.
set -o pipefail
OUT=gpurun_out/r03_resume; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timing_s'], d['roofline']['frac'], d['roofline_k1']['frac'])"
