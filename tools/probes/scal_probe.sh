# Per-rank workload of the strong-scaling runs (global batch 512 split over N ranks), emulated on one GPU:
# bench lines at 256/128/64 sequences and a rocprofv3 kernel summary of the 64-sequence (N=8) rank.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/scal
mkdir -p "$OUT"
for tb in ${TBS:-32 16 8}; do
  mb=$((tb/2))
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=$tb actor_rollout_ref.actor.ppo_mini_batch_size=$mb > "$OUT/tb$tb.json" 2> "$OUT/tb$tb.err" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > "$OUT/prof.log" 2>&1 || exit 1
python3 "$ROOT/tools/trace_summary.py" $(find "$OUT/prof" -name "*kernel_trace.csv" | head -1) 25 > "$OUT/trace_summary.txt"
find "$OUT/prof" -name "*kernel_trace.csv" -delete
