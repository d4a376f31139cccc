#!/bin/bash
# rocprofv3 kernel statistics of the N = 8 per-rank workload (64 sequences: 8 prompts x 8) -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:-prof64}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 bench.py --steps 2 --warmup 2 \
  --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > "$OUT/prof.log" 2>&1 \
  || { tail -20 "$OUT/prof.log"; exit 1; }
TR=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$TR" 30 > "$OUT/trace_summary.txt" || exit 1
python3 tools/decode_gaps.py "$TR" > "$OUT/decode_step.txt" 2>&1 || true
find "$OUT/prof" -name "*kernel_trace.csv" -delete
head -30 "$OUT/decode_step.txt"
