"""MFU accounting (mirror of verl/utils/flops_counter.py:26-167, 326-343).

``FlopsCounter.estimate_flops(batch_seqlens, delta_time)`` returns (achieved TFLOP/s, device peak TFLOP/s)
with the reference's convention for the Qwen2 / Llama family: 6 * N_dense * tokens (forward + backward,
embedding and lm_head counted once each) + 12 * sum(seqlen^2) * head_dim * heads * layers for attention.
The device table adds the MI355X dense bf16 MFMA peak (the reference's table has no MI355X entry and
reports inf for an unknown GPU, i.e. an MFU of 0).
"""

from __future__ import annotations

VALID_CONFIG_TYPE = {"llama", "qwen2", "qwen2_vl", "qwen2_5_vl", "qwen3", "mistral", "minicpmv", "minicpmo"}

# dense (no 2:1 sparsity) bf16 peaks, FLOP/s, matched on the device name
_DEVICE_FLOPS = [
    ("MI355X", 2.5e15), ("gfx950", 2.5e15), ("MI300X", 1336e12), ("GB200", 2.5e15), ("B200", 2.25e15),
    ("H100", 989e12), ("H800", 989e12), ("H200", 989e12), ("A100", 312e12), ("A800", 312e12),
    ("L40", 181.05e12), ("L20", 119.5e12), ("H20", 148e12),
]


def get_device_flops(unit: str = "T") -> float:
    """flops_counter.py:26-96: the current device's dense peak in ``unit`` (B K M G T P)."""
    import torch

    if torch.cuda.is_available():
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        name = f"{props.name} {getattr(props, 'gcnArchName', '')}"
        flops = next((f for k, f in _DEVICE_FLOPS if k in name), float("inf"))
    else:
        flops = 448e9  # the reference's CPU placeholder
    scale = {"B": 1e9, "K": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "P": 1e15}[unit]
    return flops / scale


class FlopsCounter:
    """flops_counter.py:99-167. ``config`` needs hidden_size, vocab_size, num_hidden_layers, num_attention_heads,
    num_key_value_heads, intermediate_size (head_dim optional) and model_type."""

    def __init__(self, config):
        self.config = config
        mt = getattr(config, "model_type", "qwen2")
        if mt not in VALID_CONFIG_TYPE:
            print(f"Only support config type of {VALID_CONFIG_TYPE}, but got {mt}. MFU will always be zero.")
        self._fn = self._estimate_qwen2_flops if mt in VALID_CONFIG_TYPE else (lambda *a: 0)

    def _estimate_qwen2_flops(self, tokens_sum, batch_seqlens, delta_time):
        c = self.config
        H, V, L = c.hidden_size, c.vocab_size, c.num_hidden_layers
        heads, kv_heads, inter = c.num_attention_heads, c.num_key_value_heads, c.intermediate_size
        head_dim = getattr(c, "head_dim", None) or H // heads
        q, k, v = heads * head_dim, kv_heads * head_dim, kv_heads * head_dim
        mlp_n = H * inter * 3
        attn_linear_n = H * (q + k + v + heads * head_dim)
        dense_n = (mlp_n + attn_linear_n) * L + V * H * 2
        dense_flops = 6 * dense_n * tokens_sum
        sq = sum(s * s for s in batch_seqlens)
        attn_flops = 12 * sq * head_dim * heads * L
        return (dense_flops + attn_flops) * (1.0 / delta_time) / 1e12

    def estimate_flops(self, batch_seqlens, delta_time):
        """(achieved TFLOP/s over ``delta_time`` seconds for these valid-token counts, device peak TFLOP/s)."""
        tokens_sum = sum(batch_seqlens)
        return self._fn(tokens_sum, batch_seqlens, delta_time), get_device_flops()

    def executed_flops(self, tokens=0, attn_pairs=0, lm_rows=0):
        """Forward + backward FLOPs (in TFLOP, the unit estimate_flops' rate and peak share) that the update passes
        actually executed, from the actor's exec_stats: ``tokens`` packed rows through the decoder layers (prefix
        sharing runs a prompt group's tokens once; remove-padding skips pads), ``attn_pairs`` causal (query, key) pairs
        per head the fused attention computed (the copies' skipped prompt queries excluded), ``lm_rows`` rows through
        the lm_head (the response-predicting positions only). Dense: 6 FLOP per weight and row (2 forward, 4
        backward); attention: 4 D FLOP per pair and head forward, 10 D backward (dS, dP, dQ, dK, dV and the
        recomputed S)."""
        c = self.config
        H, V, L = c.hidden_size, c.vocab_size, c.num_hidden_layers
        heads, kv_heads, inter = c.num_attention_heads, c.num_key_value_heads, c.intermediate_size
        D = getattr(c, "head_dim", None) or H // heads
        layer_n = H * inter * 3 + H * (heads * D + 2 * kv_heads * D + heads * D)
        dense = 6 * (layer_n * L * tokens + V * H * lm_rows)
        attn = 14 * D * heads * L * attn_pairs
        return (dense + attn) / 1e12
