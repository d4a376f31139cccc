"""dots.rl_amd — MI355X-native PPO/GRPO actor-learner hot path (drop-in for verl's
RayPPOTrainer.fit() / ActorRolloutRefWorker dataflow, rednote-hilab/dots.rl @ 2025-09-19).

Host code is Python mirroring the reference's interfaces; every numeric hot-path step runs in the
gfx950 HIP kernels of ``libdotsrl_amd.so`` (C-ABI: ``include/dotsrl_amd.h``). See DESIGN.md.
"""

__version__ = "0.1.0"
