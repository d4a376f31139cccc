# Decode-step anatomy (wall vs kernel-busy per decode step) at 64 rows (the per-rank N=8 workload) and 512 rows.
set -o pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${ANAT:-anat}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
for tag in ${TAGS:-64 512}; do
  if [ $tag = 64 ]; then ov="--override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4"; else ov=""; fi
  timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $OUT/p$tag -o run -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline $ov > $OUT/b$tag.log 2>&1 || { tail -20 $OUT/b$tag.log; exit 1; }
  f=$(find $OUT/p$tag -name "*kernel_trace.csv" | head -1)
  python3 tools/decode_gaps.py $f > $OUT/decode_$tag.txt || exit 1
  python3 tools/trace_summary.py $f 25 > $OUT/summary_$tag.txt || exit 1
  cp $f $OUT/trace_$tag.csv
  rm -f $f; gzip -f $OUT/trace_$tag.csv
  cat $OUT/decode_$tag.txt
done
