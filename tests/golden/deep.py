"""Configs #4 / #5 at FULL DEPTH: Llama-3-8B (32 layers, H 4096, I 14336, 32 / 8 heads of 128, V 128256, untied
lm_head, no qkv bias, RoPE theta 5e5) and Qwen2.5-7B (28 layers, H 3584, I 18944, 28 / 4 heads of 128, V 152064,
untied, qkv bias), with weights from a counter hash that numpy (tests/golden/make_golden.py, CPU, which runs the
reference HF models on them) and torch on the GPU (tests/test_deep_gpu.py) evaluate bit-identically — 30 GB of fp32
per model are never committed, and regenerating them with a sequential RNG on the GPU box's CPU would take minutes.

Element e of tensor t: h = fmix(e * C1 + off(t)) over 32-bit words (multipliers below 2^31, so every product stays
inside int64 on the GPU), u = (h >> 8) * 2^-24 in [0, 1) (exact in float32), x = (2u - 1) * scale: uniform with
std scale / sqrt(3). Matrices: scale sqrt(3 / fan_in) (unit-scale activations at any width); norm gains 1 + 0.1 u;
qkv biases 0.2 (2u - 1); the embedding 0.05 (2u - 1) * sqrt(3).
"""

import hashlib

import numpy as np
import torch

LLAMA3_8B = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                 num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0,
                 rms_norm_eps=1e-5, tie_word_embeddings=False, attention_bias=False, bos_token_id=128000,
                 eos_token_id=128001, pad_token_id=128001)
QWEN25_7B = dict(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=28,
                 num_attention_heads=28, num_key_value_heads=4, max_position_embeddings=32768, rope_theta=1000000.0,
                 rms_norm_eps=1e-6, tie_word_embeddings=False, bos_token_id=151643, eos_token_id=151643,
                 pad_token_id=151643)
MODELS = {"llama": LLAMA3_8B, "qwen7b": QWEN25_7B}
SEED = {"llama": 20261020, "qwen7b": 20261021}
C1, C2, M32 = 0x27D4EB2D, 0x45D9F3B, 0xFFFFFFFF
B, P, R = 2, 32, 32


def hf_shapes(which):
    cfg = MODELS[which]
    H, I, L = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    hd = H // cfg["num_attention_heads"]
    q, kv = cfg["num_attention_heads"] * hd, cfg["num_key_value_heads"] * hd
    out = [("model.embed_tokens.weight", (cfg["vocab_size"], H))]
    for i in range(L):
        p = f"model.layers.{i}."
        out += [(p + "self_attn.q_proj.weight", (q, H)), (p + "self_attn.k_proj.weight", (kv, H)),
                (p + "self_attn.v_proj.weight", (kv, H))]
        if which == "qwen7b":
            out += [(p + "self_attn.q_proj.bias", (q,)), (p + "self_attn.k_proj.bias", (kv,)),
                    (p + "self_attn.v_proj.bias", (kv,))]
        out += [(p + "self_attn.o_proj.weight", (H, q)), (p + "mlp.gate_proj.weight", (I, H)),
                (p + "mlp.up_proj.weight", (I, H)), (p + "mlp.down_proj.weight", (H, I)),
                (p + "input_layernorm.weight", (H,)), (p + "post_attention_layernorm.weight", (H,))]
    out += [("model.norm.weight", (H,)), ("lm_head.weight", (cfg["vocab_size"], H))]
    return out


def _offset(which, t):
    return ((SEED[which] * 1000003 + t) * 2654435761) & M32


def _scale(name, shape):
    if name.endswith("norm.weight"):
        return None
    if name.endswith("bias"):
        return 0.2
    if "embed_tokens" in name:
        return 0.05 * 3 ** 0.5
    return (3.0 / shape[1]) ** 0.5


def _finish(u, name, scale):
    if scale is None:
        return 1.0 + 0.1 * u
    return (2.0 * u - 1.0) * scale


def tensor_np(which, t, name, shape):
    n = int(np.prod(shape))
    h = (np.arange(n, dtype=np.uint64) * np.uint64(C1) + np.uint64(_offset(which, t))) & np.uint64(M32)
    h = (((h >> np.uint64(16)) ^ h) * np.uint64(C2)) & np.uint64(M32)
    h = (((h >> np.uint64(16)) ^ h) * np.uint64(C2)) & np.uint64(M32)
    h = (h >> np.uint64(16)) ^ h
    u = (h >> np.uint64(8)).astype(np.float32) * np.float32(2.0 ** -24)
    sc = _scale(name, shape)
    x = np.float32(1.0) + np.float32(0.1) * u if sc is None else (np.float32(2.0) * u - np.float32(1.0)) * np.float32(sc)
    return torch.from_numpy(x.reshape(shape))


def tensor_torch(which, t, name, shape, device="cuda"):
    n = int(np.prod(shape))
    h = (torch.arange(n, dtype=torch.int64, device=device) * C1 + _offset(which, t)) & M32
    h = (((h >> 16) ^ h) * C2) & M32
    h = (((h >> 16) ^ h) * C2) & M32
    h = (h >> 16) ^ h
    u = (h >> 8).to(torch.float32) * (2.0 ** -24)
    sc = _scale(name, shape)
    one, pt1 = torch.tensor(1.0, dtype=torch.float32, device=device), torch.tensor(0.1, dtype=torch.float32, device=device)
    if sc is None:
        x = one + pt1 * u
    else:
        x = (torch.tensor(2.0, dtype=torch.float32, device=device) * u - one) * torch.tensor(sc, dtype=torch.float32,
                                                                                            device=device)
    return x.reshape(shape)


def state_dict(which, device=None):
    """HF state dict (fp32) of the full-depth model: numpy on the CPU (device None), torch on ``device``."""
    out = {}
    for t, (name, shape) in enumerate(hf_shapes(which)):
        out[name] = tensor_np(which, t, name, shape) if device is None else tensor_torch(which, t, name, shape, device)
    return out


def sample_digest(sd):
    """sha1 of a fixed strided sample of every tensor (pins bit-identical regeneration on either side)."""
    h = hashlib.sha1()
    for name in sorted(sd):
        v = sd[name].reshape(-1)
        idx = torch.linspace(0, v.numel() - 1, 4096, dtype=torch.float64).long().to(v.device)
        h.update(name.encode())
        h.update(v[idx].cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def sequences(which):
    """B sequences of P prompt + R response tokens (random ids below the special range), row 1 left-padded by 4,
    with the attention mask / position ids the rollout produces."""
    cfg = MODELS[which]
    g = np.random.Generator(np.random.PCG64(SEED[which] + 7))
    hi = 128000 if which == "llama" else 151643
    ids = torch.from_numpy(g.integers(0, hi, (B, P + R), dtype=np.int64))
    am = torch.ones(B, P + R, dtype=torch.int64)
    am[1, :4] = 0
    ids[1, :4] = cfg["pad_token_id"]
    pos = torch.clamp(torch.cumsum(am[:, :P], -1) - 1, min=0)
    pos = torch.cat([pos, pos[:, -1:] + torch.arange(1, R + 1).unsqueeze(0)], -1)
    return ids, am, pos
