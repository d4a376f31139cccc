# Per-rank workload of the strong-scaling runs (global batch 512 split over N ranks), emulated on one GPU:
# bench lines at 256/128/64 sequences and a rocprofv3 kernel summary of the 64-sequence (N=8) rank.
set -e
cd /root/repo
mkdir -p gpurun_out/scal
make -C dots.rl_amd/csrc -j16 >/dev/null
for tb in ${TBS:-32 16 8}; do
  mb=$((tb/2))
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --override data.train_batch_size=$tb actor_rollout_ref.actor.ppo_mini_batch_size=$mb > gpurun_out/scal/tb$tb.json 2> gpurun_out/scal/tb$tb.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /root/repo/gpurun_out/scal/prof -o run -- python3 /root/repo/bench.py --steps 1 --warmup 1 --no-cpu-baseline --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > /root/repo/gpurun_out/scal/prof.log 2>&1
python /root/repo/tools/trace_summary.py $(find /root/repo/gpurun_out/scal/prof -name "*kernel_trace.csv" | head -1) 25 > /root/repo/gpurun_out/scal/trace_summary.txt
find /root/repo/gpurun_out/scal/prof -name "*kernel_trace.csv" -delete
