#!/bin/bash
# Round-3 closing record on the final library: GPU suite, smoke(), the bench line (driver-like steps), the step's
# rocprof kernel stats, decode anatomy at 64 / 512 rows, per-rank N = 2 / 4 / 8 emulation.
set -o pipefail
OUT=gpurun_out/final3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { tail -30 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], {k: round(v,3) for k,v in d['timing_s'].items()}, d['roofline']['frac'], d['roofline_k1']['frac'], d['cpu_baseline']['value'])"
bash tools/step_profile.sh final3_prof || exit 1
cp gpurun_out/final3_prof/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
ANAT=final3_anat bash tools/gpu_decode_anatomy.sh || exit 1
for n in 2 4 8; do
  tb=$((64 / n)); mb=$((32 / n)); [ $mb -lt 4 ] && mb=4
  timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --override data.train_batch_size=$tb actor_rollout_ref.actor.ppo_mini_batch_size=$mb > $OUT/n$n.log 2>&1 || { tail -30 $OUT/n$n.log; exit 1; }
  grep '^{' $OUT/n$n.log > $OUT/per_rank_n$n.json
  python -c "import json; d=json.load(open('$OUT/per_rank_n$n.json')); print('N=$n', round(d['ms_per_step'],1), {k: round(v,3) for k,v in d['timing_s'].items()})"
done
