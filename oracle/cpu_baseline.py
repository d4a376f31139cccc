"""CPU baseline of the GRPO step — TEST / BENCH INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg).

Times the reference's hot path restated on the host CPU (``oracle.qwen2_ref`` HF-Qwen2 math in eager
torch fp32 + the PPO clip loss) on a BOUNDED sample of the benchmark workload, then scales the
per-token costs to one full step of the benchmark configuration:

  rollout   : prefill of B x P prompt tokens  + B x (R-1) decode tokens      (hf_rollout.py:112-160)
  old / ref : 2 x teacher-forced forward of B x (P+R) tokens                 (dp_actor.py:232-280)
  update    : forward + backward of B x (P+R) tokens, PPO loss (vanilla clip, token-mean) + one AdamW
              step per PPO mini-batch
                                                                             (dp_actor.py:282-420)
Sample (~10-30 s on 16 host threads): forward and forward+backward over 2 sequences of 128 tokens,
greedy decode of 32 sequences x 8 steps after a 16-token prompt, AdamW over 1/8 of the parameters.
Per-token costs are taken at those lengths (attention is <10 % of a token's FLOPs at 768 tokens for
Qwen2.5-0.5B, so the length scaling is near-linear); the result is a CPU estimate, reported next to the
GPU number, never the measured product.
"""

from __future__ import annotations

import time

import torch

from . import qwen2_ref


def _timeit(fn, reps=1):
    fn()  # warm (allocator, thread pool)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def measure(cfg, B, P, R, n_optimizer_steps=2, seed=0, threads=None):
    """Returns dict(step_s=estimated seconds per full GRPO step, parts..., sample=description)."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    Pm = qwen2_ref.init_params(cfg, seed)
    V = cfg.vocab_size
    # --- forward (teacher-forced log-probs + entropy) on 2 x 128 tokens
    Ts, Bs, Rs = 128, 2, 64
    ids = torch.randint(0, V, (Bs, Ts))
    am = torch.ones(Bs, Ts, dtype=torch.int64)
    pos = torch.arange(Ts)[None].expand(Bs, Ts).contiguous()
    resp = ids[:, -Rs:]
    with torch.no_grad():
        t_fwd = _timeit(lambda: qwen2_ref.logp_entropy(cfg, Pm, ids, am, pos, resp))
    # --- forward + backward with the PPO loss (oracle formulas restated in torch for autograd)
    Pg = {k: v.clone().requires_grad_(True) for k, v in Pm.items()}
    old = torch.randn(Bs, Rs) * 0.1 - 3.0
    adv = torch.randn(Bs, Rs)

    def fb():
        lp, ent = qwen2_ref.logp_entropy(cfg, Pg, ids, am, pos, resp)
        ratio = torch.exp(lp - old)
        pg = torch.maximum(-adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.28)).mean()
        pg.backward()

    t_fb = _timeit(fb)
    # --- greedy decode: 32 sequences, 16-token prompt, 8 new tokens (prefill included, then removed)
    Bd, Pd, Rd = 32, 16, 8
    pid = torch.randint(0, V, (Bd, Pd))
    pam = torch.ones(Bd, Pd, dtype=torch.int64)
    ppos = torch.arange(Pd)[None].expand(Bd, Pd).contiguous()
    t_pre = _timeit(lambda: qwen2_ref.generate_greedy(cfg, Pm, pid, pam, ppos, 1, [-1], 0))
    t_gen = _timeit(lambda: qwen2_ref.generate_greedy(cfg, Pm, pid, pam, ppos, Rd, [-1], 0))
    c_dec = max(t_gen - t_pre, 1e-9) / (Bd * (Rd - 1))
    # --- AdamW (oracle-equivalent torch.optim on 1/8 of the parameter count, fp32)
    n_params = sum(v.numel() for v in Pm.values())
    w = torch.zeros(n_params // 8)
    w.grad = torch.randn_like(w)
    opt = torch.optim.AdamW([w], lr=1e-6, weight_decay=0.01, foreach=False)
    t_adam = _timeit(opt.step) * 8
    c_fwd = t_fwd / (Bs * Ts)
    c_fb = t_fb / (Bs * Ts)
    T = P + R
    parts = {
        "rollout_s": B * P * c_fwd + B * (R - 1) * c_dec,
        "old_log_prob_s": B * T * c_fwd,
        "ref_s": B * T * c_fwd,
        "update_actor_s": B * T * c_fb + n_optimizer_steps * t_adam,
    }
    parts["step_s"] = sum(parts.values())
    parts["per_token_s"] = {"fwd": c_fwd, "fwd_bwd": c_fb, "decode": c_dec, "adamw_full": t_adam}
    parts["sample"] = (f"Qwen2.5-0.5B-shaped random fp32 model on CPU: fwd and fwd+bwd over {Bs}x{Ts} tokens, greedy "
                       f"decode {Bd} seqs x {Rd} steps after a {Pd}-token prompt, AdamW over 1/8 of {n_params} params; "
                       f"per-token costs scaled to B={B}, P={P}, R={R}")
    parts["threads"] = torch.get_num_threads()
    return parts
