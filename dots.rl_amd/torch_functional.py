"""Vocabulary-side and rollout-bookkeeping functions with the reference's names (verl/utils/torch_functional.py,
verl/utils/model.py), computed by the HIP kernels K2 (logp/entropy over the vocabulary) and A4/A5.
"""

from __future__ import annotations

import torch

from . import native


class _LogprobEntropy(torch.autograd.Function):
    """K2 forward (one pass: logp of the label, entropy, logsumexp) and K2 backward (one pass writing
    d logits, in place over the logits buffer when the caller no longer needs them)."""

    @staticmethod
    def forward(ctx, logits, labels, temperature, want_entropy, inplace_backward):
        logp, ent, lse = native.logprob_entropy_fwd(logits, labels, temperature, want_entropy=want_entropy)
        ctx.save_for_backward(logits, labels, lse, ent if ent is not None else lse.new_empty(0))
        ctx.temperature = temperature
        ctx.inplace = inplace_backward
        ctx.want_entropy = want_entropy
        shape = labels.shape
        if ent is None:
            ent = logp.new_zeros(0)
        else:
            ent = ent.view(shape)
        return logp.view(shape), ent

    @staticmethod
    def backward(ctx, dlogp, dent):
        logits, labels, lse, ent = ctx.saved_tensors
        if not ctx.want_entropy:
            dent = None
        out = logits if ctx.inplace and logits.is_contiguous() else None
        dlogits = native.logprob_entropy_bwd(logits, labels, ctx.temperature, dlogp, dent, lse,
                                             ent if dent is not None else None, out=out.view(-1, logits.shape[-1])
                                             if out is not None else None)
        return dlogits.view(logits.shape), None, None, None, None


def logprobs_and_entropy_from_logits(logits, labels, temperature=1.0, calculate_entropy=True, inplace_backward=True):
    """log p(label) and entropy of softmax(logits / T) — the pair _forward_micro_batch computes
    (dp_actor.py:195-211, 263-272), in one read of the logits. Returns (log_probs, entropy or None), fp32."""
    logp, ent = _LogprobEntropy.apply(logits, labels, float(temperature), bool(calculate_entropy), inplace_backward)
    return logp, (ent if calculate_entropy else None)


def logprobs_from_logits(logits, labels, inplace_backward=True):
    """torch_functional.py:64-92 (flash-attn CE semantics: fp32 result)."""
    return logprobs_and_entropy_from_logits(logits, labels, 1.0, False, inplace_backward)[0]


def entropy_from_logits(logits: torch.Tensor):
    """torch_functional.py:145-149."""
    labels = torch.zeros(logits.shape[:-1], dtype=torch.int64, device=logits.device)
    return logprobs_and_entropy_from_logits(logits, labels, 1.0, True, False)[1]


class _FusedLinearLogprobEntropy(torch.autograd.Function):
    """A21: lm_head + log-prob + entropy without materialising logits (FusedLinearForPPOFunction,
    utils/experimental/torch_functional.py:75-150; linear_cross_entropy.py:41-117 with reduction "none").
    Backward = the reference's BackwardEnum._Total_Separate: one kernel writes d_logits^T (V, N) bf16 from
    recomputed logits, then d_hidden = d_logits W and d_W += d_logits^T hidden on drl_gemm (csrc/gemm_sk.hip;
    d_W straight into the fp32 gradient buffer ``weight_grad`` when given)."""

    @staticmethod
    def forward(ctx, hidden, weight, weight_grad, labels, temperature, want_entropy):
        logp, ent, lse = native.linear_logprob_fwd(hidden, weight, labels, temperature, want_entropy=want_entropy)
        ctx.save_for_backward(hidden, weight, labels, lse, ent if ent is not None else lse.new_empty(0))
        ctx.weight_grad = weight_grad
        ctx.temperature = temperature
        ctx.want_entropy = want_entropy
        return logp, (ent if ent is not None else logp.new_zeros(0))

    @staticmethod
    def backward(ctx, dlogp, dent):
        hidden, weight, labels, lse, ent = ctx.saved_tensors
        if dlogp is None:
            dlogp = torch.zeros_like(lse)
        if not ctx.want_entropy:
            dent = None
        N = hidden.shape[0]
        n8 = (N + 7) // 8 * 8  # 16-B aligned rows of d_logits^T, so drl_gemm reads it in place for any N
        dlt = native.linear_logprob_dlogits(hidden, weight, labels, ctx.temperature, dlogp, dent, lse,
                                            ent if dent is not None else None,
                                            out=torch.empty(weight.shape[0], n8, dtype=torch.bfloat16,
                                                            device=hidden.device)[:, :N])
        V, N = dlt.shape
        H = weight.shape[1]
        hip = dlt.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
        if hip:  # dh (N, H) = dlt^T W on drl_gemm: both operands read in place (layout T), any V
            dh = native.gemm(dlt, native.LAYOUT_T, weight, native.LAYOUT_T, N, H, V,
                             torch.empty(N, H, dtype=torch.bfloat16, device=dlt.device))
        else:
            dh = dlt.t() @ weight
        dw = None
        if ctx.weight_grad is not None:
            if hip and N % 64 == 0 and hidden.is_contiguous():  # dW (V, H) += dlt hidden, fp32 in place
                # (layout-K dlt needs whole 64-token k-tiles; other N — A21 is opt-in — take torch's GEMM)
                native.gemm(dlt, native.LAYOUT_K, hidden, native.LAYOUT_T, V, H, N, ctx.weight_grad, beta=True)
            else:
                torch.addmm(ctx.weight_grad, dlt, hidden, out_dtype=torch.float32, out=ctx.weight_grad)
        elif ctx.needs_input_grad[1]:
            dw = dlt @ hidden
        return dh, dw, None, None, None, None


def fused_linear_logprob_entropy(hidden, weight, labels, temperature=1.0, calculate_entropy=True, weight_grad=None):
    """hidden (N, H) bf16, weight (V, H) bf16 -> (log_probs, entropy or None), (N,) fp32 (A21). With
    ``weight_grad`` (fp32, (V, H)) the weight gradient accumulates there instead of being returned."""
    logp, ent = _FusedLinearLogprobEntropy.apply(hidden, weight, weight_grad, labels, float(temperature),
                                                 bool(calculate_entropy))
    return logp, (ent if calculate_entropy else None)


def masked_sum(values, mask, axis=None):
    """torch_functional.py:163-168."""
    assert axis is None, "only the full reduction is on the hot path"
    return masked_mean(values, mask) * (mask.sum() + 1e-8)


def masked_mean(values, mask, axis=None):
    """torch_functional.py:171-185 — token-mean reduction of the agg kernel."""
    assert axis is None, "only the full reduction is on the hot path"
    return native.agg_loss(values, mask, "token-mean")


def get_response_mask(response_id: torch.Tensor, eos_token=2, dtype=torch.int64):
    """torch_functional.py:226-246 — 1 up to and including the first EOS."""
    eos = torch.tensor(eos_token if isinstance(eos_token, (list, tuple)) else [eos_token], dtype=torch.int64,
                       device=response_id.device)
    return native.response_mask(response_id.contiguous(), eos, dtype=dtype)


def compute_position_id_with_mask(mask):
    """utils/model.py:219."""
    return native.position_ids(mask)
