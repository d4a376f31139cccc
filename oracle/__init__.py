"""CPU oracle for the PPO/GRPO actor-learner hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference algorithms (dots.rl / verl 0.5.0.dev at
/root/reference). It exists to CHECK the HIP product path: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and never as the thing measured or shipped.
The product path (``dots.rl_amd``) never imports it and fails loudly when its HIP library is missing.

Pinning: every function here is checked against golden vectors produced by running the reference
itself (``tests/golden/make_golden.py``, committed with its fixtures) — see ``tests/test_oracle_golden.py``.
"""

from .ppo_oracle import *  # noqa: F401,F403
