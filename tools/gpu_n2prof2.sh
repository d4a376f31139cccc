#!/bin/bash
set -o pipefail
OUT=gpurun_out/n2p; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep '^{' $OUT/prof.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), {k: round(v,3) for k,v in d['timing_s'].items()})"
python3 tools/trace_summary.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) 16 > $OUT/trace_summary.txt
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/trace.csv.gz; find $OUT/prof -name "*kernel_trace.csv" -delete
head -40 $OUT/trace_summary.txt
