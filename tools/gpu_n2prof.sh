#!/bin/bash
set -o pipefail
bash tools/step_profile.sh r03_n2prof --override data.train_batch_size=32 actor_rollout_ref.actor.ppo_mini_batch_size=16 && head -40 gpurun_out/r03_n2prof/trace_summary.txt
