"""DataParallelPPOActor on MI355X (mirror of verl/workers/actor/dp_actor.py:53-482).

Same micro-batching, loss composition, gradient accumulation and metric keys as the reference; the
numerics per micro-batch are: transformer forward (drl_gemm GEMMs) -> lm_head on the R response
positions only -> K2 log-prob/entropy over the vocabulary -> K1 fused actor loss (forward + backward in
one launch) -> backward of the model from (d logp, d entropy). The optimizer step is the flat-buffer
RCCL all-reduce + HIP grad-norm + HIP AdamW (FlatAdamW). Metric scalars stay on device until the end
of update_policy (one host sync per call instead of one per micro-batch, dp_actor.py:468-479).
"""

from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import native
from .core_algos import cov_loss_kw, fused_actor_loss
from .protocol import DataProto
from .seqlen_balancing import prepare_dynamic_batch, restore_dynamic_batch
from .qwen2 import PrefixShare, Qwen2Model, RmPad, gather_rows, pad_seq_columns
from .torch_functional import logprobs_and_entropy_from_logits


def append_to_dict(data: dict, new: dict):
    for k, v in new.items():
        data.setdefault(k, []).append(v)


def lr_schedule(optim_cfg):
    """The LambdaLR multiplier fsdp_workers.py:461-486 builds from an optim config section: warmup steps from
    ``lr_warmup_steps`` (or ``lr_warmup_steps_ratio`` x ``total_training_steps`` when negative / None), then
    ``warmup_style`` "constant" (get_constant_schedule_with_warmup, torch_functional.py:553-575) or "cosine"
    (get_cosine_schedule_with_warmup with ``min_lr_ratio`` / ``num_cycles``, torch_functional.py:509-550).
    Any other style raises NotImplementedError, as the reference does."""
    total = optim_cfg.get("total_training_steps", 0)
    total = 0 if total is None else int(total)
    warm = optim_cfg.get("lr_warmup_steps", -1)
    warm = -1 if warm is None else int(warm)
    ratio = float(optim_cfg.get("lr_warmup_steps_ratio", 0.0) or 0.0)
    style = optim_cfg.get("warmup_style", "constant")
    # the reference always hands the schedule a positive horizon (ray_trainer.py:557-571: the dataloader length x
    # total_epochs unless trainer.total_training_steps overrides it); without one a cosine schedule would flip
    # between lr and min_lr every step and a ratio warmup would silently be zero steps
    if total <= 0 and (style == "cosine" or (warm < 0 and ratio > 0)):
        raise ValueError(f"warmup_style={style!r} / lr_warmup_steps_ratio={ratio} need a positive "
                         f"total_training_steps (set trainer.total_training_steps, or give the trainer a "
                         f"train_dataloader with a length)")
    if warm < 0:
        warm = int(ratio * total)
    if style == "constant":
        def lam(step):
            if step < warm:
                return float(step) / float(max(1.0, warm))
            return 1.0
    elif style == "cosine":
        min_lr_ratio = optim_cfg.get("min_lr_ratio", 0.0)
        min_lr_ratio = 0.0 if min_lr_ratio is None else float(min_lr_ratio)
        assert 0.0 <= min_lr_ratio <= 1.0
        num_cycles = float(optim_cfg.get("num_cycles", 0.5))
        coef, intercept = (1 - min_lr_ratio) * 0.5, (1 + min_lr_ratio) * 0.5

        def lam(step):
            if step < warm:
                return min_lr_ratio + (1.0 - min_lr_ratio) * (float(step) / float(max(1, warm)))
            progress = float(step - warm) / float(max(1, total - warm))
            return max(min_lr_ratio, math.cos(math.pi * num_cycles * 2.0 * progress) * coef + intercept)
    else:
        raise NotImplementedError(f"Warmup style {style} is not supported")
    return lam


class FlatAdamW:
    """torch.optim.AdamW over the ParamStore's flat fp32 buffers (fsdp_workers.py:454-459 hyper-parameters),
    with clip_grad_norm_ + skip-if-non-finite (dp_actor.py:282-298) fused into the HIP step kernel.
    LR schedule: ``lr_lambda`` (``lr_schedule(optim_cfg)``: constant or cosine with warmup, as LambdaLR) evaluated
    at ``sched_step``, which the worker advances once per update call (fsdp_workers.py:717-719); default: constant
    with ``warmup_steps`` of linear warmup."""

    def __init__(self, store, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=1.0,
                 warmup_steps=0, group=None, lr_lambda=None):
        self.store = store
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.warmup_steps = warmup_steps
        self.lr_lambda = lr_lambda or lr_schedule({"lr_warmup_steps": warmup_steps})
        self.group = group
        # moments cover what the master holds: everything (replicated) or [small region | own shard]
        self.exp_avg = torch.zeros_like(store.master)
        self.exp_avg_sq = torch.zeros_like(store.master)
        self.step_count = 0
        self.sched_step = 0
        self.norm = torch.zeros(1, dtype=torch.float32, device=store.master.device)
        self._pending = []
        # sharded store: the reduce-scattered gradient of [small region | own shard], aligned with the master
        self.grad_work = torch.zeros_like(store.master) if store.sharded else None

    def current_lr(self):
        return self.lr * self.lr_lambda(self.sched_step)

    def zero_grad(self):
        self.store.zero_grad()

    # ------------------------------------------------------------------ gradient averaging across DP ranks
    def distributed(self):
        return dist.is_initialized() and dist.get_world_size(self.group) > 1

    def begin_overlap(self, model):
        """Before the LAST micro-batch's backward of an optimizer step: every decoder layer's gradient slice
        is all-reduced (async, RCCL's own stream, ordered after the layer's backward kernels) as soon as its
        backward finishes, so the 24 slices (73 % of the bytes for Qwen2.5-0.5B) travel under the rest of the
        backward. The embedding / lm_head and final-norm slices are complete only at the end (allreduce_rest)."""
        self._pending = []
        if not self.distributed() or self.store.sharded:  # sharded: one reduce-scatter in step()
            return

        def hook(i):
            a, b = self.store.layer_range(i)
            self._pending.append((a, b, dist.all_reduce(self.store.grad[a:b], op=dist.ReduceOp.AVG, group=self.group,
                                                        async_op=True)))

        model.grad_ready_hook = hook

    def end_overlap(self, model):
        model.grad_ready_hook = None

    def allreduce_grads(self):
        """AVG-all-reduce every gradient byte not already reduced by begin_overlap's per-layer work, then
        wait for all of it (the optimizer kernels run after this on the current stream)."""
        if not self.distributed():
            self._pending = []
            return
        g = self.store.grad
        done = sorted((a, b) for a, b, _ in getattr(self, "_pending", []))
        gaps, pos = [], 0
        for a, b in done:
            if a > pos:
                gaps.append((pos, a))
            pos = max(pos, b)
        if pos < g.numel():
            gaps.append((pos, g.numel()))
        works = [w for _, _, w in getattr(self, "_pending", [])]
        works += [dist.all_reduce(g[a:b], op=dist.ReduceOp.AVG, group=self.group, async_op=True) for a, b in gaps]
        for w in works:
            w.wait()
        self._pending = []

    def step(self):
        """All-reduce (average) the flat gradient across DP ranks, then norm -> clip -> AdamW in HIP.
        Returns the device grad-norm tensor (the reference returns clip_grad_norm_'s total norm)."""
        if self.store.sharded:
            return self._step_sharded()
        g = self.store.grad
        self.allreduce_grads()
        native.grad_norm(g, out=self.norm)
        self.step_count += 1
        params_bf16 = None if self.store.compute is self.store.master else self.store.compute
        self.store.version += 1  # the compute copy changes below
        native.adamw_step(self.store.master, g, self.exp_avg, self.exp_avg_sq, lr=self.current_lr(),
                          beta1=self.betas[0], beta2=self.betas[1], eps=self.eps, weight_decay=self.weight_decay,
                          step=self.step_count, max_grad_norm=self.max_grad_norm, grad_norm_t=self.norm,
                          params_bf16=params_bf16)
        return self.norm

    def _step_sharded(self):
        """ZeRO-style step over a sharded store (what FSDP FULL_SHARD's optimizer step does for the reference,
        fsdp_workers.py:397-418 + dp_actor.py:282-298): AVG reduce-scatter of the GEMM region's gradient into
        this rank's shard, AVG all-reduce of the (replicated, tiny) small region; clip_grad_norm_'s total norm
        = sqrt(|small|^2 + sum over ranks |shard|^2) (FSDP's sharded norm: local squares, SUM all-reduce);
        HIP AdamW on [small | shard] (bf16 compute shard written in the same pass); all-gather of the
        compute copy's GEMM region."""
        st, g, gw = self.store, self.store.grad, self.grad_work
        ns = st.n_small
        lo, hi = st.master_range()
        dist.all_reduce(g[:ns], op=dist.ReduceOp.AVG, group=self.group)
        if dist.get_backend(self.group) == "nccl" or g.device.type == "cpu":
            dist.reduce_scatter_tensor(gw[ns:], g[ns:], op=dist.ReduceOp.AVG, group=self.group)
        else:  # gloo on device tensors (ranks sharing one GPU in a test): AVG all-reduce, own shard kept
            dist.all_reduce(g[ns:], op=dist.ReduceOp.AVG, group=self.group)
            gw[ns:].copy_(g[lo:hi])
        gw[:ns].copy_(g[:ns])
        n_small = native.grad_norm(gw[:ns])
        n_shard = native.grad_norm(gw[ns:])
        sq = n_shard * n_shard
        dist.all_reduce(sq, op=dist.ReduceOp.SUM, group=self.group)
        torch.sqrt(sq + n_small * n_small, out=self.norm)
        self.step_count += 1
        bf16 = st.compute is not st.master and st.compute.dtype == torch.bfloat16
        hp = dict(lr=self.current_lr(), beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                  weight_decay=self.weight_decay, step=self.step_count, max_grad_norm=self.max_grad_norm,
                  grad_norm_t=self.norm)
        st.version += 1  # the compute copy changes below
        m, v, p = self.exp_avg, self.exp_avg_sq, st.master
        native.adamw_step(p[:ns], gw[:ns], m[:ns], v[:ns], params_bf16=None, **hp)
        native.adamw_step(p[ns:], gw[ns:], m[ns:], v[ns:], params_bf16=st.compute[lo:hi] if bf16 else None, **hp)
        if not bf16:
            st.compute[lo:hi].copy_(p[ns:])
        st.all_gather_compute()
        return self.norm

    def state_dict(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self.step_count,
                "sched_step": self.sched_step}

    def load_state_dict(self, sd):
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        self.sched_step = int(sd.get("sched_step", 0))


def _concat_rows(group):
    """The forward inputs of consecutive micro-batches as one batch of rows (all share the padded width T)."""
    if len(group) == 1:
        return group[0].batch
    return {k: torch.cat([mb.batch[k] for mb in group], 0)
            for k in ("input_ids", "attention_mask", "position_ids", "responses")}


def exec_groups(cfg, model_cfg, micro_batches, shared_tokens=0.0, resident_bytes=0):
    """Micro-batches that run through the model in one pass. The reference runs one per forward / backward
    (dp_actor.py:392-466, dp_critic.py:214-250); their gradients only add up (each micro-batch's loss carries its own
    scale factor and token count), so consecutive micro-batches may share one pass over their concatenated rows: the
    GEMMs see 2-4x the rows (at 6144 rows the N = 896 projections fill 96 of 256 CUs). ``exec_micro_batches`` fixes
    the group size (1 = the reference's schedule); 0 groups as many as keep the saved activations under
    ``exec_activation_gb``. ``shared_tokens``: the fraction of a micro-batch's tokens that prefix sharing runs once
    for several rows (they hold no per-token activations of their own; the attention's stay padded), the smallest
    over the micro-batches. ``resident_bytes``: device memory the worker holds for the whole run (parameter stores,
    gradient, AdamW moments, the reference policy): the plan keeps within 70 % of what they leave."""
    n = int(cfg.get("exec_micro_batches", 1) or 0)
    if n <= 0:
        H, I, L = model_cfg.hidden_size, model_cfg.intermediate_size, model_cfg.num_hidden_layers
        nq = (model_cfg.num_attention_heads + 2 * model_cfg.num_key_value_heads) * model_cfg.head_dim
        # saved per token and layer: x, x2 (fp32), h1, h2, attn (bf16), gate|up and SwiGLU out per packed token;
        # q / k / v / k^T (and the padded attention output) per padded position
        per_tok = L * ((8 * H + 6 * H + 6 * I) * (1.0 - shared_tokens) + 4 * nq)
        budget = float(cfg.get("exec_activation_gb", 110)) * 2 ** 30
        if torch.cuda.is_available():
            # never plan past 40 % of the device — a static bound (not what happens to be free at the call), so the
            # group size, and with it the GEMM shapes and the fp32 gradient summation order, is the same on every
            # rank, run and resume
            total = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory
            budget = min(budget, 0.4 * total)
            if resident_bytes:  # what the resident state leaves (the same on every rank: a static bound too)
                budget = min(budget, 0.7 * max(0, total - resident_bytes))
        toks = max(mb.batch["input_ids"].numel() for mb in micro_batches)
        n = max(1, int(budget // max(1, per_tok * toks)))
    return balanced_groups(micro_batches, n)


def balanced_groups(items, n):
    """Consecutive groups of at most n items, as few as possible and of near-equal size (32 items at n = 17 -> two
    groups of 16, not 17 + 15): every pass's GEMMs then see about the same row count."""
    if not items:
        return []
    k = -(-len(items) // max(1, n))
    base, extra = divmod(len(items), k)
    out, i = [], 0
    for j in range(k):
        m = base + (1 if j < extra else 0)
        out.append(items[i:i + m])
        i += m
    return out


class DataParallelPPOActor:
    """dp_actor.py:53-482. ``actor_optimizer`` None -> reference policy."""

    def __init__(self, config, actor_module: Qwen2Model, actor_optimizer: FlatAdamW | None = None):
        self.config = config
        self.actor_module = actor_module
        self.actor_optimizer = actor_optimizer
        self.use_remove_padding = config.get("use_remove_padding", False)
        self.use_fused_kernels = config.get("use_fused_kernels", False)
        self.share_prompt_prefix = config.get("share_prompt_prefix", True)
        self.exec_stats = {"tokens": 0, "attn_pairs": 0, "lm_rows": 0}

    def _forward_micro_batch(self, micro_batch, temperature, calculate_entropy=False):
        """dp_actor.py:90-280: full-sequence forward, logits only at the R positions that predict the response
        ([:, -R-1:-1]), then K2. Returns (entropy or None, log_probs), (bs, R) fp32.

        use_remove_padding (dp_actor.py:119-247): the backbone runs on the nnz attended tokens only (RmPad), the R
        predicting rows are gathered from the packed hidden states and the outputs at pad positions are 0 (the
        reference's pad_input). The reference takes the label of the last attended token from the next packed
        sequence; that position is outside the response mask in both.

        share_prompt_prefix (qwen2.PrefixShare): rows of the pass that share a prompt — the n samples of a GRPO
        group — run the prompt's tokens once; their attention still reads every row's full sequence."""
        m = self.actor_module
        responses = micro_batch["responses"]
        B, R = responses.shape
        # T % 8 != 0 (e.g. max_response_length 250): pad columns the fused attention needs, sliced away below
        ids, am, pos, padc = pad_seq_columns(m, micro_batch["input_ids"], micro_batch["attention_mask"],
                                             micro_batch["position_ids"])
        keep = None
        # the pad columns count as response positions for prefix sharing (never shared)
        share = PrefixShare.build(ids, am, R + padc, keep_pads=not self.use_remove_padding) \
            if self.share_prompt_prefix else None
        T = am.shape[1]
        T0 = T - padc
        if m.training:  # executed work of the update passes (exec_stats: the executed-FLOP MFU beside the reference's)
            st = self.exec_stats
            pairs = B * T * (T + 1) // 2  # causal (query, key) pairs the fused attention computes per head
            if share is not None:
                # q_start: the copies skip the shared prompt's query tiles — whole 32-row tiles below q_start only
                # (csrc/flash_attn.hip starts at q_start & ~31), so the skipped pairs are those of S0 = S & ~31 rows
                S0 = share.S & ~31
                pairs -= (B - share.groups) * S0 * (S0 + 1) // 2
            st["tokens"] += share.nnz if share is not None else (int(am.sum()) if self.use_remove_padding else B * T)
            st["attn_pairs"] += pairs
            st["lm_rows"] += B * R
        if share is not None or self.use_remove_padding:
            rm = share if share is not None else RmPad(am)
            h = m.hidden_states(ids, am, pos, rm=rm)
            sel = rm.inv.view(B, T)[:, T0 - R - 1:T0 - 1].reshape(-1).contiguous()
            h = gather_rows(h.view(rm.nnz, h.shape[-1]), sel)
            keep = (sel >= 0).view(B, R)
        else:
            h = m.hidden_states(ids, am, pos)
            h = h[:, T0 - R - 1:T0 - 1, :].reshape(B * R, h.shape[-1])
        if self.use_fused_kernels:  # A21: no (B*R, V) logits (dp_actor.py:173-186 fused branch)
            logp, ent = m.fused_logprob(h, responses.reshape(-1), temperature, calculate_entropy)
        else:
            logits = m.logits(h)
            logp, ent = logprobs_and_entropy_from_logits(logits, responses.reshape(-1), temperature,
                                                         calculate_entropy, inplace_backward=True)
        logp, ent = logp.view(B, R), (ent.view(B, R) if ent is not None else None)
        if keep is not None:
            logp = torch.where(keep, logp, 0.0)
            ent = torch.where(keep, ent, 0.0) if ent is not None else None
        return ent, logp

    def _shared_fraction(self, data, rows_per_micro_batch=None):
        """Fraction of the tokens that prefix sharing runs once for several rows: the first P - 1 tokens of every row
        whose prompt equals the previous row's (the trainer's interleaved repeat). With ``rows_per_micro_batch`` the
        smallest fraction over the micro-batches of that many rows (a row that opens a micro-batch counts as
        unshared): the activation plan then holds for the least-shared pass. One device read."""
        if not self.share_prompt_prefix or data is None or len(data) < 2:
            return 0.0
        ids = data.batch["input_ids"]
        B, T = ids.shape
        S = T - data.batch["responses"].shape[1] - 1
        if S <= 0:
            return 0.0
        same = torch.zeros(B, dtype=torch.int64, device=ids.device)
        same[1:] = (ids[1:, :S] == ids[:-1, :S]).all(-1)
        n = int(rows_per_micro_batch or B)
        if n >= B:
            return int(same.sum()) * S / (B * T)
        same[::n] = 0
        k = B // n * n
        per = same[:k].view(-1, n).sum(-1).tolist() + ([int(same[k:].sum())] if k < B else [])
        sizes = [n] * (k // n) + ([B - k] if k < B else [])
        return min(c * S / (m * T) for c, m in zip(per, sizes))

    def resident_bytes(self):
        """Device memory held for the whole run: this actor's parameter store and AdamW moments plus what the worker
        registered beside it (``extra_resident_bytes``: the reference policy's store)."""
        b = self.actor_module.store.memory_bytes() + getattr(self, "extra_resident_bytes", 0)
        opt = self.actor_optimizer
        if opt is not None:
            b += sum(t.numel() * t.element_size() for t in (getattr(opt, "exp_avg", None),
                                                          getattr(opt, "exp_avg_sq", None)) if t is not None)
        return b

    def _exec_groups(self, micro_batches, mini_batch=None):
        rows = len(micro_batches[0]) if micro_batches and not self.config.get("use_dynamic_bsz", False) else None
        return exec_groups(self.config, self.actor_module.cfg, micro_batches,
                           self._shared_fraction(mini_batch, rows), self.resident_bytes())

    def _log_prob_groups(self, micro_batches, data=None):
        """Forward-only passes: rows are independent, so consecutive micro-batches run as one pass of at most
        ``exec_log_prob_tokens`` tokens (0: one micro-batch per pass, as the reference) — bigger GEMMs, same rows.
        Tokens prefix sharing runs once per group count once."""
        budget = int(self.config.get("exec_log_prob_tokens", 0) or 0)
        if budget <= 0:
            return [[mb] for mb in micro_batches]
        toks = max(mb.batch["input_ids"].numel() for mb in micro_batches) if micro_batches else 1
        toks = max(1, int(toks * (1.0 - self._shared_fraction(data))))
        return balanced_groups(micro_batches, max(1, budget // toks))

    @torch.no_grad()
    def compute_log_prob(self, data: DataProto, calculate_entropy=False):
        """dp_actor.py:300-359."""
        self.actor_module.training = False
        micro_batch_size = data.meta_info["micro_batch_size"]
        temperature = data.meta_info["temperature"]
        use_dynamic_bsz = data.meta_info.get("use_dynamic_bsz", False)
        data = data.select(batch_keys=["responses", "input_ids", "attention_mask", "position_ids"])
        if use_dynamic_bsz:  # token-budget micro-batches (seqlen_balancing.prepare_dynamic_batch)
            micro_batches, batch_idx_list = prepare_dynamic_batch(data, max_token_len=data.meta_info["max_token_len"])
        else:
            micro_batches = data.split(micro_batch_size)
        lps, ents = [], []
        for group in self._log_prob_groups(micro_batches, data if not use_dynamic_bsz else None):
            ent, lp = self._forward_micro_batch(_concat_rows(group), temperature, calculate_entropy)
            lps.append(lp)
            if calculate_entropy:
                ents.append(ent)
        log_probs = torch.cat(lps, 0)
        entropys = torch.cat(ents, 0) if calculate_entropy else None
        if use_dynamic_bsz:
            log_probs = restore_dynamic_batch(log_probs, batch_idx_list)
            if entropys is not None:
                entropys = restore_dynamic_batch(entropys, batch_idx_list)
        return log_probs, entropys

    def update_policy(self, data: DataProto):
        """dp_actor.py:361-482."""
        cfg = self.config
        m = self.actor_module
        m.training = True
        temperature = data.meta_info["temperature"]
        keys = ["responses", "response_mask", "input_ids", "attention_mask", "position_ids", "old_log_probs",
                "advantages"]
        if cfg.use_kl_loss:
            keys.append("ref_log_prob")
        data = data.select(batch_keys=keys)
        mini_batches = data.split(cfg.ppo_mini_batch_size)
        loss_mode = cfg.policy_loss.get("loss_mode", "vanilla")
        if loss_mode not in ("vanilla", "gpg", "gspo", "geo_mean", "clip_cov", "kl_cov"):
            raise NotImplementedError(f"policy loss {loss_mode}: the fused K1 modes are vanilla (PPO clip + dual clip), "
                                      "gpg, gspo, geo_mean, clip_cov and kl_cov")
        lo = cfg.clip_ratio_low if cfg.get("clip_ratio_low") is not None else cfg.clip_ratio
        hi = cfg.clip_ratio_high if cfg.get("clip_ratio_high") is not None else cfg.clip_ratio
        mb_out, mb_lsf, grad_norms = [], [], []
        for _ in range(cfg.ppo_epochs):
            for mini_batch in mini_batches:
                if cfg.get("use_dynamic_bsz", False):
                    micro_batches, _ = prepare_dynamic_batch(mini_batch, max_token_len=cfg.ppo_max_token_len_per_gpu)
                else:
                    grad_accum = cfg.ppo_mini_batch_size // cfg.ppo_micro_batch_size_per_gpu
                    micro_batches = mini_batch.split(cfg.ppo_micro_batch_size_per_gpu)
                self.actor_optimizer.zero_grad()
                counts = None
                if cfg.loss_agg_mode == "token-mean" and loss_mode in ("vanilla", "gpg"):
                    # every micro-batch's sum(response_mask) in one launch (exact in fp64): K1 runs one-pass
                    sizes = {len(mb) for mb in micro_batches}
                    if cfg.get("use_dynamic_bsz", False) or len(sizes) != 1:
                        counts = torch.stack([mb.batch["response_mask"].sum(dtype=torch.float64)
                                              for mb in micro_batches])
                    else:
                        rm = mini_batch.batch["response_mask"]
                        counts = rm.reshape(len(micro_batches), -1).sum(-1, dtype=torch.float64)
                groups = self._exec_groups(micro_batches, mini_batch)
                k = 0
                for gi, group in enumerate(groups):
                    if gi == len(groups) - 1:  # gradients final after this backward: overlap the all-reduce
                        self.actor_optimizer.begin_overlap(m)
                    calculate_entropy = cfg.entropy_coeff != 0
                    entropy_all, log_prob_all = self._forward_micro_batch(_concat_rows(group), temperature,
                                                                          calculate_entropy)
                    total, r0 = None, 0
                    for micro_batch in group:
                        mb = micro_batch.batch
                        n = mb["responses"].shape[0]
                        if cfg.get("use_dynamic_bsz", False):  # relative to the dynamic bsz (dp_actor.py:413-414)
                            lsf = mb["response_mask"].shape[0] / cfg.ppo_mini_batch_size
                        else:
                            lsf = 1.0 / grad_accum
                        log_prob = log_prob_all[r0:r0 + n] if len(group) > 1 else log_prob_all
                        entropy = entropy_all[r0:r0 + n] if (entropy_all is not None and len(group) > 1) else entropy_all
                        r0 += n
                        out = fused_actor_loss(
                            log_prob, entropy, mb["old_log_probs"], mb["advantages"], mb["response_mask"],
                            mb.get("ref_log_prob"), clip_ratio_low=lo, clip_ratio_high=hi,
                            clip_ratio_c=cfg.get("clip_ratio_c", 3.0), entropy_coeff=cfg.entropy_coeff,
                            use_kl_loss=cfg.use_kl_loss, kl_loss_type=cfg.kl_loss_type, kl_loss_coef=cfg.kl_loss_coef,
                            loss_agg_mode=cfg.loss_agg_mode, loss_scale_factor=lsf, policy_loss=loss_mode,
                            token_count=counts[k:k + 1] if counts is not None else None,
                            cov_kw=(cov_loss_kw(cfg.policy_loss, loss_mode,
                                                seed_key=(cfg.policy_loss.get("seed", 1234),
                                                          self.actor_optimizer.step_count, k))
                                    if loss_mode in ("clip_cov", "kl_cov") else None))
                        total = out[6] if total is None else total + out[6]
                        mb_out.append(out.detach())
                        mb_lsf.append(lsf)
                        k += 1
                    total.backward()
                self.actor_optimizer.end_overlap(m)
                grad_norms.append(self.actor_optimizer.step().clone())
        self.actor_optimizer.zero_grad()
        m.training = False
        # one device->host copy for every metric of the call
        stats = torch.stack(mb_out).cpu().tolist() if mb_out else []
        gn = torch.cat(grad_norms).cpu().tolist() if grad_norms else []
        metrics: dict = {}
        for row, lsf in zip(stats, mb_lsf):
            mbm = {}
            if cfg.use_kl_loss:
                mbm["actor/kl_loss"] = row[5] * lsf
                mbm["actor/kl_coef"] = cfg.kl_loss_coef
            mbm.update({"actor/pg_loss": row[0] * lsf, "actor/pg_clipfrac": row[1], "actor/ppo_kl": row[2],
                        "actor/pg_clipfrac_lower": row[3]})
            append_to_dict(metrics, mbm)
        for g in gn:
            if not math.isfinite(g):
                print(f"WARN: grad_norm is not finite: {g}")
            append_to_dict(metrics, {"actor/grad_norm": g})
        return metrics
