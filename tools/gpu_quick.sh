# Full GPU test suite + N=1 bench line + per-rank (64-sequence) bench line (run through gpurun).
set -o pipefail
OUT=gpurun_out/q
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -1 $OUT/gputests.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b512.json 2> $OUT/b512.err || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > $OUT/b64.json 2> $OUT/b64.err || exit 1
