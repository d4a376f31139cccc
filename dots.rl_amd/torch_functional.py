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


_BUFFER_RANGE = 1 << 31  # drl_gemm's operands stay below one 2 GB buffer range


def fused_linear_vocab_block(V, n_cols):
    """Vocabulary rows per d_logits^T block of the fused lm_head backward: the (block, n_cols) bf16 block plus one
    tile of overhang stays below the 2 GB buffer range drl_gemm reads in place (256-row multiples)."""
    rows = (_BUFFER_RANGE // (2 * n_cols) - 320) // 256 * 256
    assert rows >= 256, f"{n_cols} tokens: a 256-row d_logits block exceeds the 2 GB operand range"
    return min(V, rows)


class _FusedLinearLogprobEntropy(torch.autograd.Function):
    """A21: lm_head + log-prob + entropy without materialising logits (FusedLinearForPPOFunction,
    utils/experimental/torch_functional.py:75-150; linear_cross_entropy.py:41-117 with reduction "none").

    Backward = the reference's BackwardEnum._Split_Dlogits_N (kernels.py:1519-1580) on this repo's kernels: the
    vocabulary in blocks whose d_logits^T (block, N) bf16 stays below the 2 GB operand range; per block
    ``drl_linear_logprob_dlogits`` recomputes z on MFMA and writes d_logits^T, then d_hidden (+)= d_logits W_blk and
    d_W[blk] (+)= d_logits^T hidden on drl_gemm (csrc/gemm_sk.hip, fp32 accumulation; d_W straight into the fp32
    gradient buffer ``weight_grad`` when given). d_hidden accumulates in fp32 across blocks and is rounded to bf16
    once, as the reference's single bf16 matmul over the whole vocabulary rounds its fp32 sum once."""

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
        assert hidden.dtype == weight.dtype == torch.bfloat16, "the fused lm_head runs on bf16 operands"
        N, H = hidden.shape
        V = weight.shape[0]
        dev = hidden.device
        weight = weight.contiguous()
        labels = labels.reshape(-1)
        # d_W's GEMM reads d_logits^T with the tokens along K (layout K): whole 64-token k-tiles, so the block has
        # 64-aligned rows whose columns past N stay zero, and hidden is read through a zero-padded copy when N is
        # ragged (zero rows x zero columns: the padding adds exact zeros)
        n64 = (N + 63) // 64 * 64
        hid = hidden.contiguous()
        if n64 != N:
            hid = torch.zeros(n64, H, dtype=hidden.dtype, device=dev)
            hid[:N] = hidden
        vb = fused_linear_vocab_block(V, n64)
        blk = torch.empty(vb, n64, dtype=torch.bfloat16, device=dev)
        if n64 != N:
            blk[:, N:].zero_()
        one_block = vb >= V
        dh = torch.empty(N, H, dtype=torch.bfloat16 if one_block else torch.float32, device=dev)
        wg = ctx.weight_grad
        dw = None
        if wg is None and ctx.needs_input_grad[1]:
            dw = torch.empty(V, H, dtype=torch.float32, device=dev)
        for v0 in range(0, V, vb):
            rows = min(vb, V - v0)
            w_blk = weight[v0:v0 + rows]
            dlt = native.linear_logprob_dlogits(hidden, w_blk, labels - v0 if v0 else labels, ctx.temperature, dlogp,
                                                dent, lse, ent if dent is not None else None, out=blk[:rows, :N])
            # d_hidden (N, H) (+)= d_logits (N, rows) W_blk: A = d_logits^T read as layout T, B = W_blk layout T
            native.gemm(dlt, native.LAYOUT_T, w_blk, native.LAYOUT_T, N, H, rows, dh, beta=v0 > 0)
            # d_W[blk] (rows, H) (+)= d_logits^T hidden: A = the block (layout K over n64 tokens), B = hidden layout T
            tgt = wg[v0:v0 + rows] if wg is not None else (dw[v0:v0 + rows] if dw is not None else None)
            if tgt is not None:
                native.gemm(blk[:rows], native.LAYOUT_K, hid, native.LAYOUT_T, rows, H, n64, tgt, beta=wg is not None)
        if not one_block:
            dh = dh.to(torch.bfloat16)
        return dh, (dw.to(weight.dtype) if dw is not None else None), None, None, None, None


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
