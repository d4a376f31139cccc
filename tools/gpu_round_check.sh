mkdir -p gpurun_out/r11
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r11/gputests.log 2>&1
tail -3 gpurun_out/r11/gputests.log
grep -q " passed" gpurun_out/r11/gputests.log && ! grep -q " failed\|[0-9] error" gpurun_out/r11/gputests.log || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r11/b512.json 2> gpurun_out/r11/b512.err || exit 1
bash tools/step_profile.sh r11p64 --override data.train_batch_size=8 actor_rollout_ref.actor.ppo_mini_batch_size=4 > gpurun_out/r11/b64.json
