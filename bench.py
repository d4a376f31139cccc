"""PPO steps/sec + rollout tokens/sec for Qwen2.5-0.5B GRPO on MI355X (BASELINE.json config #2 / #3).

One "step" is one full GRPO iteration of RayPPOTrainer.fit(): rollout of 64 prompts x n=8 (512-token
prompts, 256-token responses, sampling) -> old log-probs + entropy -> ref log-probs -> GRPO advantages ->
two PPO mini-batch updates (micro 8/GPU) with AdamW. Global batch is fixed (512 sequences/step) and split
across the N ranks: "scaling" is strong. Random-init Qwen2.5-0.5B weights, synthetic prompts.

  python bench.py [--gpus N] [--steps K] [--warmup W]          (N>1 under torch.distributed.run)

Besides the step rate the JSON line carries
  roofline     : the dominant eagerly launched hand-written kernel (--roofline-kernel; default drl_gemm, the
                 stream-K ping-pong GEMM that runs every projection of the full-sequence passes — forward,
                 dgrad and wgrad — and the lm_head; MFMA-bound; the fused attention forward is the other
                 MFMA-bound kernel),
                 every launch inside the timed region bracketed by HIP events on its launch stream;
                 achieved = algorithmic work per launch (ROOFLINE below) / mean launch
                 duration, against its bound's peak (2.5 PFLOP/s dense bf16 MFMA or 8 TB/s HBM);
                 traffic = HBM bytes per launch from the committed rocprofv3 PMC pass
                 (profiles/pmc_<kernel>.json, FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE) or null;
  cpu_baseline : rank 0 at N=1 only — oracle/cpu_baseline.py (the same step restated in eager torch fp32
                 on the host cores) on a bounded sample, scaled to PPO steps/s.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "PPO steps/sec + rollout tokens/sec, Qwen2.5-0.5B GRPO @1/2/4/8 MI355X"
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (AMD's 5 PF figure counts 2:1 sparsity)


def _softmax_fwd_bytes(a):
    # drl_masked_softmax_fwd(scores, probs, dt, valid, ld_valid, B, HG, Tq, Tk, qoff, scale, stream):
    # read fp32 scores + write probs (bf16 / fp32) per element, key-valid row once per (b, key)
    dt, B, HG, Tq, Tk = a[2], a[5], a[6], a[7], a[8]
    return B * HG * Tq * Tk * (4 + (2 if dt == 4 else 4)) + B * Tk


def _decode_attn_bytes(a):
    # drl_decode_attention(q, k, v, dt, valid, ld, qpos_ptr, qpos, B, Hkv, G, D, Tk, L, ...): K and V rows
    # of every allowed key once + q and out rows
    dt, B, Hkv, G, D, L = a[3], a[8], a[9], a[10], a[11], a[13]
    e = 2 if dt == 4 else 4
    return B * Hkv * (2 * L * D + 2 * G * D) * e


def _flash_fwd_flops(a):
    # drl_flash_attn_fwd(q, k, vt, dt, valid, ld_valid, B, Hkv, G, D, Tq, Tk, ld_k, ld_vt, qoff, ...):
    # QK^T and PV over the causally allowed (query, key) pairs: 4 * D FLOP per pair and query head
    B, Hkv, G, D, Tq, Tk, qoff = a[6], a[7], a[8], a[9], a[10], a[11], a[14]
    pairs = sum(min(Tk, t + qoff + 1) for t in range(Tq))
    return 4.0 * B * Hkv * G * D * pairs


def _swiglu_fwd_bytes(a):
    # drl_swiglu_fwd(gate_up, out, dt, N, I, stream): read gate and up rows, write the product (one element each)
    dt, N, I = a[2], a[3], a[4]
    return 3 * N * I * (2 if dt == 4 else 4)


def _gemm_sk_flops(a):
    # drl_gemm(a, lda, a_layout, b, ldb, b_layout, c, ldc, c_dtype, beta, M, N, K, bias, epilogue, ...): 2 M N K
    return 2.0 * a[10] * a[11] * a[12]


def _gemm_sk_dispatches(a):
    """Kernel dispatches of one drl_gemm call (rocprof counts these; the KernelTimer counts calls): a layout-T operand
    past the 2 GB buffer range is split over K blocks, one dispatch each (csrc/gemm_sk.hip, drl_gemm); a layout-K A
    past it runs as one dispatch with its descriptor rebased per tile."""
    from dots.rl_amd import _lib, native

    lda, a_layout, ldb, b_layout, M, N, K = a[1], a[2], a[4], a[5], a[10], a[11], a[12]
    lim = 1 << 31
    tb = [K * ld * 2 + 320 * ld * 2 if lay == 1 else 0 for lay, ld in ((a_layout, lda), (b_layout, ldb))]
    # round 6: a layout-T A past the range (B within it, fp32 plain output, a whole-tile plan) walks its K blocks
    # inside ONE launch (the lm_head weight gradient)
    if (a_layout == 1 and tb[0] >= lim and tb[1] < lim and a[8] == _lib.DRL_F32 and a[14] == 0
            and native.gemm_plan(M, N, K, 0)[0] == 2):
        return 1
    if max(tb) >= lim:
        ld = max(lda if a_layout == 1 else 0, ldb if b_layout == 1 else 0)
        kb = max(128, (lim // (ld * 2) - 320) // 128 * 128)
        return -(-K // kb)
    return 1


def _gemm_sk_tag(a):
    # (M, N, K, a_layout, b_layout, c_dtype, epilogue, dispatches)
    return (a[10], a[11], a[12], a[2], a[5], a[8], a[14], _gemm_sk_dispatches(a))


TAGS = {"drl_gemm": _gemm_sk_tag}

# symbol -> (work per launch from the call's arguments, per-unit statement, bound, peak, unit)
ROOFLINE = {
    "drl_gemm": (_gemm_sk_flops, "2*M*N*K FLOP per launch (bf16 operands, fp32 accumulation): every projection GEMM "
                 "of the full-sequence passes — forward (bias / SwiGLU epilogues), dgrad, wgrad into the fp32 "
                 "gradient, lm_head forward and backward", "mfma", PEAK_BF16_TFLOPS, "TFLOP/s"),
    "drl_swiglu_fwd": (_swiglu_fwd_bytes, "6 B per (token, intermediate column): gate + up read, product written (bf16)",
                       "hbm", PEAK_HBM_GBPS, "GB/s"),
    "drl_flash_attn_fwd": (_flash_fwd_flops, "4*D FLOP per causal (query, key) pair per query head", "mfma",
                           PEAK_BF16_TFLOPS, "TFLOP/s"),
    "drl_masked_softmax_fwd": (_softmax_fwd_bytes, "6 B per attention score (fp32 in, bf16 out)", "hbm",
                               PEAK_HBM_GBPS, "GB/s"),
    "drl_decode_attention": (_decode_attn_bytes, "4*D B per cached key (bf16 K+V rows)", "hbm", PEAK_HBM_GBPS,
                             "GB/s"),
}


def _pmc_traffic(symbol):
    path = os.path.join(ROOT, "profiles", f"pmc_{symbol}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


K1_TOKENS = 1 << 26
K1_PER_UNIT = ("36 B per token: old_log_prob, log_prob, advantages, entropy, ref_log_prob read (5 x 4 B fp32), "
               "response_mask read (8 B int64), dlog_prob and dentropy written (2 x 4 B fp32)")


def k1_roofline(form="two_pass", reps=20, warmup=3):
    """North-star kernel K1 (fused PPO loss fwd+bwd, drl_ppo_loss_fwd_bwd) at 2^26 tokens, token-mean, low_var_kl,
    entropy bonus, int64 mask: every launch bracketed by HIP events on its stream. ``one_pass`` is the form the
    actor runs (dp_actor.update_policy hands over every micro-batch's sum(mask)); ``two_pass`` folds the count by
    the K1a pre-pass inside the same call (callers without the count)."""
    import torch

    from dots.rl_amd import native

    N, R = K1_TOKENS, 1024
    B = N // R
    g = torch.Generator(device="cuda").manual_seed(26)
    old = -torch.rand(B, R, device="cuda", generator=g) * 5
    lp = old + torch.randn(B, R, device="cuda", generator=g) * 0.3
    adv = torch.randn(B, R, device="cuda", generator=g)
    mask = (torch.rand(B, R, device="cuda", generator=g) > 0.05).to(torch.int64)
    ent = torch.rand(B, R, device="cuda", generator=g)
    ref = lp + 0.1
    out = torch.empty(8, device="cuda")
    dlp, dent = torch.empty_like(lp), torch.empty_like(lp)
    kw = dict(entropy_coeff=0.001, kl_loss_coef=0.001, kl_loss_type="low_var_kl", loss_agg_mode="token-mean",
              want_dentropy=True, out=out, dlogp=dlp, dentropy=dent)
    if form == "one_pass":
        kw["token_count"] = mask.to(torch.float64).sum().reshape(1)
    for _ in range(warmup):
        native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, **kw)
    # one HIP event pair on the launch stream around `reps` back-to-back calls (per-call event pairs would add
    # their own gaps to a ~450 us kernel): mean call duration, kernel boundaries included
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, **kw)
    b.record(s)
    b.synchronize()
    t = a.elapsed_time(b) * 1e-3 / reps
    work = 36.0 * N
    sym = "drl_ppo_loss_fwd_bwd" + ("_one_pass" if form == "one_pass" else "")
    traffic, src = _pmc_traffic(sym)
    achieved = work / t / 1e9
    del old, lp, adv, mask, ent, ref, dlp, dent
    torch.cuda.empty_cache()
    return {"kernel": "drl_ppo_loss_fwd_bwd", "form": form, "tokens": N, "bound": "hbm", "achieved": achieved,
            "peak": PEAK_HBM_GBPS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBPS, "traffic": traffic,
            "algorithmic_work_per_launch": work, "mean_launch_us": t * 1e6, "launches": reps, "per_unit": K1_PER_UNIT,
            "traffic_source": src}


def cpu_baseline(cfg):
    from oracle import cpu_baseline as cb

    from dots.rl_amd.workers import resolve_model_config

    ar = cfg.actor_rollout_ref
    B = cfg.data.train_batch_size * ar.rollout.n
    n_mini = max(1, cfg.data.train_batch_size // ar.actor.ppo_mini_batch_size)
    r = cb.measure(resolve_model_config(ar.model), B, cfg.data.max_prompt_length, cfg.data.max_response_length,
                   n_optimizer_steps=n_mini, group=int(ar.rollout.n))
    out = {"value": 1.0 / r["step_s"], "unit": "PPO steps/s", "cores": r["threads"], "kind": "port",
           "sample": r["sample"], "est_step_s": r["step_s"],
           "value_range": [1.0 / r["step_s_range"][1], 1.0 / r["step_s_range"][0]],
           "est_parts_s": {k: v for k, v in r.items() if k.endswith("_s") and k != "step_s"},
           # what the headline priced: every row's prompt + response tokens, no prompt sharing (the reference's CPU
           # FSDP path); the GPU line runs prompt groups once, so the shared-prompt estimate is given beside it
           "tokens_per_row_priced": r["tokens_per_row"], "prompts_shared": False}
    if "shared" in r:
        sh = r["shared"]
        out["shared_prompt_estimate"] = {"value": 1.0 / sh["step_s"], "unit": "PPO steps/s",
                                         "est_step_s": sh["step_s"], "tokens_per_row_priced": sh["tokens_per_row"],
                                         "prompts_shared": True, "group": sh["group"]}
    return out


def build_config(args):
    from dots.rl_amd.config import apply_overrides, default_config

    cfg = default_config()
    apply_overrides(cfg, [
        "data.train_batch_size=64", "data.max_prompt_length=512", "data.max_response_length=256",
        "actor_rollout_ref.rollout.n=8", "actor_rollout_ref.rollout.response_length=256",
        "actor_rollout_ref.rollout.prompt_length=512", "actor_rollout_ref.rollout.ignore_eos=True",
        "actor_rollout_ref.actor.ppo_mini_batch_size=32", "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=8",
        "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=16",
        "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=16",
        "actor_rollout_ref.actor.use_kl_loss=True", "actor_rollout_ref.actor.kl_loss_coef=0.001",
        "actor_rollout_ref.actor.kl_loss_type=low_var_kl", "actor_rollout_ref.actor.entropy_coeff=0",
        "algorithm.adv_estimator=grpo", "trainer.balance_batch=False", "trainer.gc_freeze=True",
    ])
    if args.tiny:
        apply_overrides(cfg, ["+actor_rollout_ref.model.override_config.num_hidden_layers=2",
                              "data.train_batch_size=8", "actor_rollout_ref.actor.ppo_mini_batch_size=4",
                              "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=4",
                              "data.max_response_length=32", "actor_rollout_ref.rollout.response_length=32",
                              "data.max_prompt_length=64", "actor_rollout_ref.rollout.prompt_length=64"])
    if args.dapo:
        # BASELINE config #5 on one GPU: Qwen2.5-7B, the DAPO recipe (clip-higher, token-mean, dynamic sampling with
        # filter_groups on acc, overlong buffer), group size 8, 1024-token responses; 8 prompts x 8 per step
        from dots.rl_amd.dapo_trainer import dapo_overrides

        apply_overrides(cfg, dapo_overrides(1024) + [
            "actor_rollout_ref.model.path=random:qwen2.5-7b", "data.train_batch_size=8",
            "data.max_response_length=1024", "actor_rollout_ref.rollout.response_length=1024",
            "actor_rollout_ref.actor.ppo_mini_batch_size=4", "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=2",
            "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=8",
            "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=8",
            "reward_model.reward_manager=dapo_synthetic"])
    apply_overrides(cfg, args.override)
    return cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    # two warmup steps: after a single one, the first timed step's old_log_prob stage measured 1.2-1.4 s instead of
    # 0.36 s (profiles/r03_decode_lanes.jsonl, warmup-1 runs)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tiny", action="store_true", help="2-layer model, small batch (bring-up only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-kernel", default="drl_gemm", choices=sorted(ROOFLINE))
    ap.add_argument("--override", nargs="*", default=[])
    ap.add_argument("--dapo", action="store_true",
                    help="BASELINE config #5 on one GPU: Qwen2.5-7B DAPO, n=8, 1024-token responses (RayDAPOTrainer)")
    ap.add_argument("--k1-only", choices=["two_pass", "one_pass"], default=None,
                    help="only the K1 roofline at 2^26 tokens (rocprofv3 PMC passes for profiles/pmc_drl_ppo_loss_*)")
    ap.add_argument("--launch-log", default=None,
                    help="write every timed launch of the roofline kernel in the LAST timed step (start / end us, "
                         "stream, work, shape) as JSON lines to this path: the roofline's per-dispatch and union "
                         "fractions recompute from it")
    ap.add_argument("--dist-backend", default=None,
                    help="default: nccl (RCCL) on GPU; gloo lets several ranks share one GPU for a rehearsal")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from dots.rl_amd import native

    if args.k1_only:
        print(json.dumps(k1_roofline(args.k1_only)), flush=True)
        return
    from dots.rl_amd.single_controller import init_process_group_from_env
    from dots.rl_amd.trainer import RayPPOTrainer

    init_process_group_from_env(args.dist_backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    cfg = build_config(args)
    if args.dapo:
        from dots.rl_amd.dapo_trainer import RayDAPOTrainer

        trainer = RayDAPOTrainer(cfg)
    else:
        trainer = RayPPOTrainer(cfg)
    trainer.init_workers()
    trainer.global_steps = 1
    for _ in range(args.warmup):
        trainer.step(None if args.dapo else trainer.train_dataloader.next())
        trainer.global_steps += 1
    # DAPO draws its own generation batches inside step() (dynamic sampling)
    prompts = [None if args.dapo else trainer.train_dataloader.next() for _ in range(args.steps)]
    if cfg.trainer.get("gc_freeze", False):  # the long-running job's host heap, frozen once warm (trainer.freeze_host_heap)
        from dots.rl_amd.trainer import freeze_host_heap

        freeze_host_heap()
    timer = native.KernelTimer(args.roofline_kernel, ROOFLINE[args.roofline_kernel][0], TAGS.get(args.roofline_kernel))
    mark = os.environ.get("DRL_TRACE_MARK") == "1"  # a spin kernel on each side of the timed steps (trace windows)
    dist.barrier()  # (the first barrier of a run builds the communicator: seconds, kept out of the trace window)
    torch.cuda.synchronize()
    if mark:
        torch.cuda._sleep(1000)
    ms0 = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    hist = []
    last_step_first_launch = 0
    with timer:
        for p in prompts:
            last_step_first_launch = len(timer.events)
            hist.append(trainer.step(p))
            trainer.global_steps += 1
    torch.cuda.synchronize()
    if mark:
        torch.cuda._sleep(1000)
    dist.barrier()
    ms1 = torch.cuda.memory_stats()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    steps_per_s = args.steps / elapsed
    gen_tokens = sum(h["perf/total_num_tokens"] for h in hist)  # prompt + response tokens processed
    resp_tokens = sum(h["perf/rollout_tokens_per_sec"] * h["timing_s/gen"] for h in hist)
    gen_time = sum(h["timing_s/gen"] for h in hist)
    n_launch, t_launch, b_launch = timer.summary()
    # the rate of the kernel's work while any of its launches runs: launches on the side stream (weight gradients)
    # overlap the current stream's, so the mean per-launch interval (mean_launch_us, comparable to rocprof's
    # per-kernel average) counts shared time twice; achieved uses the union of the intervals instead
    t_busy = timer.busy_seconds() / n_launch if n_launch else None
    dispatches = sum(t[-1] for t in timer.tags) if timer.tags and n_launch else None
    if args.launch_log and rank == 0 and n_launch:
        with open(args.launch_log, "w") as f:
            for st, en, stream, work, tag in timer.intervals()[last_step_first_launch:]:
                f.write(json.dumps({"start_us": round(st, 3), "end_us": round(en, 3), "stream": stream, "work": work,
                                    "tag": tag}) + "\n")
    if rank == 0:
        ar = cfg.actor_rollout_ref
        preset = str(ar.model.get("path", "random:qwen2.5-0.5b"))
        model_name = {"random:qwen2.5-0.5b": "Qwen2.5-0.5B", "random:llama-3-8b": "Llama-3-8B",
                      "random:qwen2.5-7b": "Qwen2.5-7B", "random:": "Qwen2.5-0.5B"}.get(preset, preset)
        if args.tiny:
            model_name += " (2 layers)"
        algo = {"grpo": "GRPO", "gae": "PPO"}.get(str(cfg.algorithm.adv_estimator), str(cfg.algorithm.adv_estimator))
        if args.dapo:
            algo = "DAPO"
        # BASELINE.json's metric for the default workload; the same sentence with the model / algorithm that ran
        metric = METRIC.replace("Qwen2.5-0.5B GRPO", f"{model_name} {algo}")
        _, per_unit, bound, peak, unit = ROOFLINE[args.roofline_kernel]
        scale = 1e12 if unit == "TFLOP/s" else 1e9
        # frac: the work over the summed launch durations (each call's HIP-event interval; the rocprof view: the
        # mean kernel duration x dispatches); frac_union: over the union of those intervals (launches on the side
        # stream — weight gradients beside their input gradients — share the CUs with the current stream's)
        achieved = b_launch / t_launch / scale if n_launch else None
        achieved_union = b_launch / t_busy / scale if n_launch else None
        # the committed PMC pass is of the default workload (N=1 config #2): attach it only to that workload
        default_workload = not args.tiny and not args.override and args.gpus == 1
        traffic, traffic_src = _pmc_traffic(args.roofline_kernel) if default_workload else (None, None)
        roofline = {"kernel": args.roofline_kernel, "bound": bound, "achieved": achieved, "peak": peak,
                    "unit": unit, "frac": achieved / peak if achieved else None,
                    "frac_per_dispatch": achieved / peak if achieved else None,
                    "achieved_union": achieved_union, "frac_union": achieved_union / peak if achieved_union else None,
                    "traffic": traffic,
                    "algorithmic_work_per_launch": b_launch if n_launch else None,
                    "mean_launch_us": t_launch * 1e6 if n_launch else None, "launches": n_launch,
                    "dispatches": dispatches,
                    "mean_dispatch_us": t_launch * n_launch / dispatches * 1e6 if dispatches else None,
                    "busy_us_per_launch": t_busy * 1e6 if n_launch else None,
                    "per_unit": per_unit, "traffic_source": traffic_src}
        line = {
            "metric": metric,
            "value": steps_per_s,
            "unit": "PPO steps/s",
            "rollout_tokens_per_sec": resp_tokens / gen_time,
            "perf/throughput_tokens_per_sec_per_gpu": gen_tokens / elapsed / world,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"workload": (f"{model_name} {algo}, {cfg.data.train_batch_size} prompts x n={ar.rollout.n}, "
                                    f"{cfg.data.max_prompt_length}-tok prompts / {cfg.data.max_response_length}-tok responses"),
                       "model": f"{model_name} (random init)", "global_batch": cfg.data.train_batch_size * ar.rollout.n,
                       "seq_len": cfg.data.max_prompt_length + cfg.data.max_response_length,
                       "parallelism": f"dp{world}", "tiny": bool(args.tiny)},
            "timing_s": {k.split("/", 1)[1]: sum(h[k] for h in hist) / len(hist) for k in hist[0] if k.startswith("timing_s/")},
            # per stage over the timed steps: [min, median, max] seconds (a bimodal stage shows as max >> median)
            "timing_spread_s": {k.split("/", 1)[1]: [min(v), sorted(v)[len(v) // 2], max(v)]
                                for k in hist[0] if k.startswith("timing_s/")
                                for v in [[h[k] for h in hist]]},
            # headline MFU: the FLOPs update_actor executed (flops_counter.executed_flops: prompt groups counted once,
            # lm_head over the response rows) over its time and the dense bf16 peak
            "mfu_actor": sum(h.get("perf/mfu/actor_executed", 0.0) for h in hist) / len(hist),
            "mfu_actor_basis": "executed FLOPs of update_actor / its time / 2.5 PFLOP/s dense bf16",
            # the reference's perf/mfu/actor (flops_counter.estimate_flops over every row's prompt + response
            # tokens): with prompt groups run once (prompt_groups below) it counts FLOPs that were never executed
            "reference_formula": {"mfu_actor": sum(h.get("perf/mfu/actor", 0.0) for h in hist) / len(hist),
                                  "basis": "verl flops_counter.estimate_flops over every row's tokens (perf/mfu/actor)"},
            "prompt_groups": {"rollout.enable_prefix_caching": bool(ar.rollout.get("enable_prefix_caching", True)),
                              "model.share_prompt_prefix": bool(ar.model.get("share_prompt_prefix", True))},
            "roofline": roofline,
            "roofline_k1": None,
            "cpu_baseline": None,
            # device memory of this rank over the run (caching allocator): a high retry count means the passes are
            # sized past what the pool can serve without freeing and re-allocating
            "memory": {"max_allocated_gb": torch.cuda.max_memory_allocated() / 2 ** 30,
                       "max_reserved_gb": torch.cuda.max_memory_reserved() / 2 ** 30,
                       "alloc_retries": torch.cuda.memory_stats().get("num_alloc_retries", 0),
                       # device allocations / frees by torch's caching allocator inside the timed region
                       "timed_device_allocs": ms1.get("num_device_alloc", 0) - ms0.get("num_device_alloc", 0),
                       "timed_device_frees": ms1.get("num_device_free", 0) - ms0.get("num_device_free", 0)},
        }
        if not args.tiny:
            # the actor's form: update_policy hands K1 every micro-batch's sum(response_mask) (one pass over HBM)
            line["roofline_k1"] = k1_roofline("one_pass")
            line["roofline_k1_two_pass"] = k1_roofline("two_pass")
        if world == 1 and not args.no_cpu_baseline and not args.tiny:
            line["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(line), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
