#!/bin/bash
# Closing check of the committed tree: the GPU suite, smoke(), the default bench line (no flags).
set -o pipefail
OUT=gpurun_out/close; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['steps'], d['warmup'], round(d['ms_per_step'],1), {k: round(v,3) for k,v in d['timing_s'].items()}, d['roofline']['frac'], d['roofline_k1']['frac'], d['memory'])"
