"""DataParallelPPOCritic on MI355X (mirror of verl/workers/critic/dp_critic.py:46-263).

Same micro-batching, loss scaling, gradient accumulation and metric keys as the reference. Per micro-batch:
Qwen2 backbone forward (the actor's kernels) -> the value head on the R positions that predict the
response ([:, -R-1:-1], ``csrc/value_loss.hip`` drl_value_head_fwd, output in the compute dtype like the
reference's autocast Linear) -> K6 fused clipped value loss, forward + backward in one launch
(drl_value_loss_fwd_bwd) -> value-head backward (drl_value_head_bwd, weight/bias gradients accumulated in
fp32) -> the backbone's hand-written backward. Optimizer: the flat-buffer RCCL all-reduce + HIP grad-norm +
HIP AdamW of the actor (FlatAdamW), with the critic's own hyper-parameters (critic.yaml: lr 1e-5).
"""

from __future__ import annotations

import math

import torch

from . import native
from .dp_actor import FlatAdamW, _concat_rows, append_to_dict, exec_groups
from .protocol import DataProto
from .seqlen_balancing import prepare_dynamic_batch, restore_dynamic_batch
from .qwen2 import PrefixShare, Qwen2Model, RmPad, gather_rows, pad_seq_columns


class _ValueHead(torch.autograd.Function):
    """values (N,) = h (N, H) . score.weight + score.bias; backward dh = dv w, dW/db += (fp32, in place)."""

    @staticmethod
    def forward(ctx, h, w, b, gw, gb, dummy):
        h = h.contiguous()
        ctx.save_for_backward(h, w)
        ctx.gw, ctx.gb = gw, gb
        return native.value_head_fwd(h, w, b)

    @staticmethod
    def backward(ctx, dv):
        h, w = ctx.saved_tensors
        dh = native.value_head_bwd(h, w, dv, dweight=ctx.gw.reshape(-1) if ctx.gw is not None else None,
                                   dbias=ctx.gb if ctx.gb is not None else None)
        return dh, None, None, None, None, None


def value_head(m: Qwen2Model, h):
    """The critic's score head over hidden rows h (N, H) -> (N,) values in the compute dtype."""
    s = m.store
    train = m.training and s.trainable
    return _ValueHead.apply(h, s.w("score.weight"), s.w("score.bias"), s.g("score.weight") if train else None,
                            s.g("score.bias") if train else None, m._dummy)


class DataParallelPPOCritic:
    """dp_critic.py:46-263 (padded and use_remove_padding paths; ulysses SP is out of scope)."""

    def __init__(self, config, critic_module: Qwen2Model, critic_optimizer: FlatAdamW | None = None):
        self.config = config
        self.critic_module = critic_module
        self.critic_optimizer = critic_optimizer
        self.use_remove_padding = config.model.get("use_remove_padding", False) if "model" in config else False
        # prefix sharing (qwen2.PrefixShare, as the actor's): a prompt group's prompt tokens run once
        self.share_prompt_prefix = config.model.get("share_prompt_prefix", True) if "model" in config else True

    def _forward_micro_batch(self, micro_batch):
        """dp_critic.py:57-145: values = score(h)[:, -R-1:-1] (compute dtype, (bs, R)); use_remove_padding
        (dp_critic.py:69-107) runs the backbone on the attended tokens only and gives 0 at pad positions."""
        m = self.critic_module
        R = micro_batch["responses"].size(-1)
        # T % 8 != 0: pad columns for the fused attention (qwen2.pad_seq_columns), sliced away below
        ids, am, pos, padc = pad_seq_columns(m, micro_batch["input_ids"], micro_batch["attention_mask"],
                                             micro_batch["position_ids"])
        B, T = am.shape
        T0 = T - padc
        share = PrefixShare.build(ids, am, R + padc, keep_pads=not self.use_remove_padding) \
            if self.share_prompt_prefix else None
        if share is not None or self.use_remove_padding:
            rm = share if share is not None else RmPad(am)
            h = m.hidden_states(ids, am, pos, rm=rm)
            sel = rm.inv.view(B, T)[:, T0 - R - 1:T0 - 1].reshape(-1).contiguous()
            v = value_head(m, gather_rows(h.view(rm.nnz, h.shape[-1]), sel)).view(B, R)
            return torch.where((sel >= 0).view(B, R), v, 0.0)
        h = m.hidden_states(ids, am, pos)
        h = h[:, T0 - R - 1:T0 - 1, :].reshape(B * R, h.shape[-1])
        return value_head(m, h).view(B, R)

    @torch.no_grad()
    def compute_values(self, data: DataProto) -> torch.Tensor:
        """dp_critic.py:163-197."""
        self.critic_module.training = False
        micro_batch_size = data.meta_info["micro_batch_size"]
        use_dynamic_bsz = data.meta_info.get("use_dynamic_bsz", False)
        keys = ["responses", "input_ids", "attention_mask", "position_ids"]
        if "response_mask" in data.batch:
            keys.append("response_mask")
        data = data.select(batch_keys=keys)
        if use_dynamic_bsz:
            micro_batches, batch_idx_list = prepare_dynamic_batch(data, max_token_len=data.meta_info["max_token_len"])
        else:
            micro_batches = data.split(micro_batch_size)
        values = torch.cat([self._forward_micro_batch(mb.batch) for mb in micro_batches], 0)
        if use_dynamic_bsz:
            values = restore_dynamic_batch(values, batch_idx_list)
        if "response_mask" in data.batch:
            values = values * data.batch["response_mask"]  # only action tokens have values (bf16 * int64 -> bf16)
        return values

    def update_critic(self, data: DataProto):
        """dp_critic.py:199-263."""
        cfg = self.config
        m = self.critic_module
        m.training = True
        data = data.select(batch_keys=["input_ids", "responses", "response_mask", "attention_mask", "position_ids",
                                       "values", "returns"])
        mini_batches = data.split(cfg.ppo_mini_batch_size)
        mb_out, mb_lsf, grad_norms = [], [], []
        for _ in range(cfg.ppo_epochs):
            for mini_batch in mini_batches:
                if cfg.get("use_dynamic_bsz", False):
                    micro_batches, _ = prepare_dynamic_batch(mini_batch, max_token_len=cfg.ppo_max_token_len_per_gpu)
                else:
                    grad_accum = cfg.ppo_mini_batch_size // cfg.ppo_micro_batch_size_per_gpu
                    micro_batches = mini_batch.split(cfg.ppo_micro_batch_size_per_gpu)
                self.critic_optimizer.zero_grad()
                # micro-batches sharing one pass (dp_actor), planned within what the critic's resident state leaves
                opt = self.critic_optimizer
                resident = m.store.memory_bytes() + sum(t.numel() * t.element_size()
                                                        for t in (opt.exp_avg, opt.exp_avg_sq))
                groups = exec_groups(cfg, m.cfg, micro_batches, resident_bytes=resident)
                for gi, group in enumerate(groups):
                    if gi == len(groups) - 1:
                        self.critic_optimizer.begin_overlap(m)
                    vpreds_all = self._forward_micro_batch(_concat_rows(group))
                    total, r0 = None, 0
                    for micro_batch in group:
                        mb = micro_batch.batch
                        n = mb["responses"].shape[0]
                        if cfg.get("use_dynamic_bsz", False):  # dp_critic.py:232-234
                            lsf = mb["response_mask"].shape[0] / cfg.ppo_mini_batch_size
                        else:
                            lsf = 1.0 / grad_accum
                        vpreds = vpreds_all[r0:r0 + n] if len(group) > 1 else vpreds_all
                        r0 += n
                        out = fused_value_loss(vpreds, mb["values"], mb["returns"], mb["response_mask"],
                                               cliprange_value=cfg.cliprange_value, loss_agg_mode=cfg.loss_agg_mode,
                                               loss_scale_factor=lsf)
                        total = out[3] if total is None else total + out[3]
                        mb_out.append(out.detach())
                        mb_lsf.append(lsf)
                    total.backward()
                self.critic_optimizer.end_overlap(m)
                grad_norms.append(self.critic_optimizer.step().clone())
        self.critic_optimizer.zero_grad()
        m.training = False
        stats = torch.stack(mb_out).cpu().tolist() if mb_out else []
        gn = torch.cat(grad_norms).cpu().tolist() if grad_norms else []
        metrics: dict = {}
        for row, lsf in zip(stats, mb_lsf):
            append_to_dict(metrics, {"critic/vf_loss": row[0] * lsf, "critic/vf_clipfrac": row[1],
                                     "critic/vpred_mean": row[2]})
        for g in gn:
            if not math.isfinite(g):
                print(f"WARN: grad_norm is not finite: {g}")
            append_to_dict(metrics, {"critic/grad_norm": g})
        return metrics


class _FusedValueLoss(torch.autograd.Function):
    """K6: forward AND backward in the forward launch; backward scales the stored d loss / d vpreds."""

    @staticmethod
    def forward(ctx, vpreds, values, returns, response_mask, kw):
        out, dv = native.value_loss_fwd_bwd(vpreds.detach(), values, returns, response_mask,
                                            want_dvpreds=vpreds.requires_grad, **kw)
        ctx.save_for_backward(dv if dv is not None else out.new_empty(0))
        ctx.has = dv is not None
        return out

    @staticmethod
    def backward(ctx, g):
        (dv,) = ctx.saved_tensors
        return (dv * g[3] if ctx.has else None), None, None, None, None


def fused_value_loss(vpreds, values, returns, response_mask, *, cliprange_value, loss_agg_mode="token-mean",
                     loss_scale_factor=1.0):
    """float32[8]: vf_loss, vf_clipfrac, vpred_mean, loss (= vf_loss * loss_scale_factor, the differentiable
    slot), mask count (DRL_VALUE_OUT_*)."""
    return _FusedValueLoss.apply(vpreds, values, returns, response_mask,
                                 dict(cliprange_value=cliprange_value, loss_agg_mode=loss_agg_mode,
                                      loss_scale_factor=loss_scale_factor))
