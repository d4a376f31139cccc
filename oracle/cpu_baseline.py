"""CPU baseline of the GRPO step — TEST / BENCH INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg).

Times the reference's hot path restated on the host CPU (``oracle.qwen2_ref`` HF-Qwen2 math in eager
torch fp32 + the PPO clip loss) on a BOUNDED sample of the benchmark workload, then scales the
per-token costs to one full step of the benchmark configuration:

  rollout   : prefill of B x P prompt tokens  + B x (R-1) decode tokens      (hf_rollout.py:112-160)
  old / ref : 2 x teacher-forced forward of B x (P+R) tokens                 (dp_actor.py:232-280)
  update    : forward + backward of B x (P+R) tokens, PPO loss (vanilla clip, token-mean) + one AdamW
              step per PPO mini-batch
                                                                             (dp_actor.py:282-420)
Sample (~40-60 s on 16 host threads): forward and forward+backward over 4 sequences of 512 tokens, greedy
decode of 32 sequences x 32 steps after a 64-token prompt, AdamW over 1/8 of the parameters; each timed 3 times
after a warm-up, the median used and the (min, max) spread reported.
Per-token costs are taken at those lengths (attention is <10 % of a token's FLOPs at 768 tokens for
Qwen2.5-0.5B, so the length scaling is near-linear); the result is a CPU estimate, reported next to the
GPU number, never the measured product.
"""

from __future__ import annotations

import time

import torch

from . import qwen2_ref


def _timeit(fn, reps=3):
    """Median and (min, max) of ``reps`` timed calls after one warm-up call."""
    fn()  # warm (allocator, thread pool)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], (ts[0], ts[-1])


def measure(cfg, B, P, R, n_optimizer_steps=2, seed=0, threads=None, reps=3, group=1):
    """Returns dict(step_s=estimated seconds per full GRPO step (median sample), step_s_range=(min, max) over the
    repetitions, parts..., sample=description). The headline prices every row's P + R tokens, as the reference's
    CPU FSDP path computes them (no prompt sharing). With ``group`` > 1 (GRPO's n samples per prompt, interleaved)
    ``shared`` adds the estimate for the work the GPU line executes with prompt groups run once: the prefill over
    B / group prompts, and the full-sequence passes over B / group x (P - 1) shared prompt tokens + B x (R + 1) own
    tokens (qwen2.PrefixShare); the decode is unchanged."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    Pm = qwen2_ref.init_params(cfg, seed)
    V = cfg.vocab_size
    # --- forward (teacher-forced log-probs + entropy) on 4 x 512 tokens (the last 256 predict the response)
    Ts, Bs, Rs = 512, 4, 256
    ids = torch.randint(0, V, (Bs, Ts))
    am = torch.ones(Bs, Ts, dtype=torch.int64)
    pos = torch.arange(Ts)[None].expand(Bs, Ts).contiguous()
    resp = ids[:, -Rs:]
    with torch.no_grad():
        t_fwd, r_fwd = _timeit(lambda: qwen2_ref.logp_entropy(cfg, Pm, ids, am, pos, resp), reps)
    # --- forward + backward with the PPO loss (oracle formulas restated in torch for autograd)
    Pg = {k: v.clone().requires_grad_(True) for k, v in Pm.items()}
    old = torch.randn(Bs, Rs) * 0.1 - 3.0
    adv = torch.randn(Bs, Rs)

    def fb():
        lp, ent = qwen2_ref.logp_entropy(cfg, Pg, ids, am, pos, resp)
        ratio = torch.exp(lp - old)
        pg = torch.maximum(-adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.28)).mean()
        pg.backward()
        for v in Pg.values():
            v.grad = None

    t_fb, r_fb = _timeit(fb, reps)
    # --- greedy decode: 32 sequences, 64-token prompt, 32 new tokens (the prefill-only run is subtracted)
    Bd, Pd, Rd = 32, 64, 32
    pid = torch.randint(0, V, (Bd, Pd))
    pam = torch.ones(Bd, Pd, dtype=torch.int64)
    ppos = torch.arange(Pd)[None].expand(Bd, Pd).contiguous()
    t_pre, r_pre = _timeit(lambda: qwen2_ref.generate_greedy(cfg, Pm, pid, pam, ppos, 1, [-1], 0), reps)
    t_gen, r_gen = _timeit(lambda: qwen2_ref.generate_greedy(cfg, Pm, pid, pam, ppos, Rd, [-1], 0), reps)
    c_dec = max(t_gen - t_pre, 1e-9) / (Bd * (Rd - 1))
    c_dec_rng = (max(r_gen[0] - r_pre[1], 1e-9) / (Bd * (Rd - 1)), max(r_gen[1] - r_pre[0], 1e-9) / (Bd * (Rd - 1)))
    # --- AdamW (oracle-equivalent torch.optim on 1/8 of the parameter count, fp32)
    n_params = sum(v.numel() for v in Pm.values())
    w = torch.zeros(n_params // 8)
    w.grad = torch.randn_like(w)
    opt = torch.optim.AdamW([w], lr=1e-6, weight_decay=0.01, foreach=False)
    t_adam, r_adam = _timeit(opt.step, reps)
    t_adam, r_adam = t_adam * 8, (r_adam[0] * 8, r_adam[1] * 8)
    T = P + R

    def parts_of(c_fwd, c_fb, c_d, ta):
        p = {"rollout_s": B * P * c_fwd + B * (R - 1) * c_d, "old_log_prob_s": B * T * c_fwd,
             "ref_s": B * T * c_fwd, "update_actor_s": B * T * c_fb + n_optimizer_steps * ta}
        return p, sum(p.values())

    parts, step = parts_of(t_fwd / (Bs * Ts), t_fb / (Bs * Ts), c_dec, t_adam)
    _, lo = parts_of(r_fwd[0] / (Bs * Ts), r_fb[0] / (Bs * Ts), c_dec_rng[0], r_adam[0])
    _, hi = parts_of(r_fwd[1] / (Bs * Ts), r_fb[1] / (Bs * Ts), c_dec_rng[1], r_adam[1])
    parts["step_s"] = step
    parts["step_s_range"] = (lo, hi)
    parts["tokens_per_row"] = T
    if group > 1:
        tok_shared = (B // group) * (P - 1) + B * (R + 1)
        c_fwd, c_fb = t_fwd / (Bs * Ts), t_fb / (Bs * Ts)
        sh = {"rollout_s": (B // group) * P * c_fwd + B * (R - 1) * c_dec, "old_log_prob_s": tok_shared * c_fwd,
              "ref_s": tok_shared * c_fwd, "update_actor_s": tok_shared * c_fb + n_optimizer_steps * t_adam}
        parts["shared"] = {"step_s": sum(sh.values()), "tokens_per_row": tok_shared / B, "group": group,
                           **{k + "_shared": v for k, v in sh.items()}}
    parts["per_token_s"] = {"fwd": t_fwd / (Bs * Ts), "fwd_bwd": t_fb / (Bs * Ts), "decode": c_dec,
                            "adamw_full": t_adam}
    parts["sample"] = (f"Qwen2.5-0.5B-shaped random fp32 model on CPU: fwd and fwd+bwd over {Bs}x{Ts} tokens, greedy "
                       f"decode {Bd} seqs x {Rd} steps after a {Pd}-token prompt, AdamW over 1/8 of {n_params} params; "
                       f"median of {reps} repetitions each; per-token costs scaled to B={B}, P={P}, R={R}")
    parts["threads"] = torch.get_num_threads()
    return parts
