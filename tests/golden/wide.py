"""Deterministic CPU-seeded weights for configs #4 / #5 at FULL WIDTH and reduced depth (2 decoder layers):
Llama-3-8B (H 4096, I 14336, 32 / 8 heads of 128, V 128256, untied lm_head, no qkv bias, RoPE theta 5e5) and
Qwen2.5-7B (H 3584, I 18944, 28 / 4 heads of 128, V 152064, untied, qkv bias). Shared by make_golden.py (which runs
the reference HF models on them) and tests/test_wide_gpu.py (which rebuilds the identical tensors on the GPU box);
the ~6 GB per model are never committed. Every tensor comes from its own seeded numpy PCG64 stream (bit-identical
across hosts, like full_depth.py); ``checksum`` pins that. Critic: the same backbone + a `score` head (num_labels=1).
"""

import hashlib

import numpy as np
import torch

LLAMA3_8B_W = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
                   num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0,
                   rms_norm_eps=1e-5, tie_word_embeddings=False, attention_bias=False, bos_token_id=128000,
                   eos_token_id=128001, pad_token_id=128001)
QWEN25_7B_W = dict(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=2,
                   num_attention_heads=28, num_key_value_heads=4, max_position_embeddings=32768, rope_theta=1000000.0,
                   rms_norm_eps=1e-6, tie_word_embeddings=False, bos_token_id=151643, eos_token_id=151643,
                   pad_token_id=151643)
SEED = {"llama": 20261017, "qwen7b": 20261018}


def hf_shapes(cfg, bias):
    H, I, L = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    hd = H // cfg["num_attention_heads"]
    q, kv = cfg["num_attention_heads"] * hd, cfg["num_key_value_heads"] * hd
    out = [("model.embed_tokens.weight", (cfg["vocab_size"], H))]
    for i in range(L):
        p = f"model.layers.{i}."
        out += [(p + "self_attn.q_proj.weight", (q, H)), (p + "self_attn.k_proj.weight", (kv, H)),
                (p + "self_attn.v_proj.weight", (kv, H))]
        if bias:
            out += [(p + "self_attn.q_proj.bias", (q,)), (p + "self_attn.k_proj.bias", (kv,)),
                    (p + "self_attn.v_proj.bias", (kv,))]
        out += [(p + "self_attn.o_proj.weight", (H, q)), (p + "mlp.gate_proj.weight", (I, H)),
                (p + "mlp.up_proj.weight", (I, H)), (p + "mlp.down_proj.weight", (H, I)),
                (p + "input_layernorm.weight", (H,)), (p + "post_attention_layernorm.weight", (H,))]
    out += [("model.norm.weight", (H,)), ("lm_head.weight", (cfg["vocab_size"], H))]
    return out


def make_state_dict(which):
    """HF state dict (fp32) of the 2-layer full-width model ``which`` ("llama" / "qwen7b"), plus the critic's
    `score.weight` / `score.bias`."""
    cfg = LLAMA3_8B_W if which == "llama" else QWEN25_7B_W
    seed = SEED[which]
    H = cfg["hidden_size"]
    sd = {}
    shapes = hf_shapes(cfg, which == "qwen7b") + [("score.weight", (1, H)), ("score.bias", (1,))]
    for i, (name, shape) in enumerate(shapes):
        g = np.random.Generator(np.random.PCG64(seed * 1000 + i))
        x = g.standard_normal(shape, dtype=np.float32)
        if name.endswith("norm.weight"):
            x = 1.0 + 0.05 * x
        elif name.endswith("bias"):
            x = 0.1 * x
        elif name.startswith("score"):
            x = 0.2 * x / np.sqrt(H, dtype=np.float32)
        else:  # N(0, 1/sqrt(fan_in)): unit-scale activations whatever the width
            x = x / np.sqrt(shape[1], dtype=np.float32)
        sd[name] = torch.from_numpy(x)
    return sd


def checksum(sd):
    return {k: hashlib.sha1(v.contiguous().numpy().tobytes()).hexdigest() for k, v in sd.items()}


def sequences(which, B=2, P=24, R=16):
    """B sequences of P prompt + R response tokens (ids below the special range), row 1 left-padded by 5 and its
    response ending after 11 tokens (EOS then pad), with the attention mask / position ids the rollout produces."""
    cfg = LLAMA3_8B_W if which == "llama" else QWEN25_7B_W
    g = np.random.Generator(np.random.PCG64(SEED[which] + 1))
    hi = 128000 if which == "llama" else 151643
    ids = torch.from_numpy(g.integers(0, hi, (B, P + R), dtype=np.int64))
    am = torch.ones(B, P + R, dtype=torch.int64)
    am[1, :5] = 0
    ids[1, :5] = cfg["pad_token_id"]
    ids[1, P + 10] = cfg["eos_token_id"]
    ids[1, P + 11:] = cfg["pad_token_id"]
    am[1, P + 11:] = 0
    pos = torch.clamp(torch.cumsum(am[:, :P], -1) - 1, min=0)
    pos = torch.cat([pos, pos[:, -1:] + torch.arange(1, R + 1).unsqueeze(0)], -1)
    return ids, am, pos, R
