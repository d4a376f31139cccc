"""Deterministic CPU-seeded Qwen2.5-0.5B-shaped weights (config #2 at full depth: 24 layers, H 896, I 4864,
14 / 2 heads, V 151 936, tied embeddings), shared by tests/golden/make_golden.py (which runs the reference
HF model on them) and tests/test_full_depth_gpu.py (which rebuilds the identical tensors on the GPU box).
The 2 GB of weights are never committed: every tensor is drawn from its own seeded numpy PCG64 generator
(numpy's streams are bit-identical across hosts; torch's CPU randn is not - its vectorised kernels depend on
the host's SIMD level), so any host with this numpy reproduces them bit for bit. ``checksum`` pins that.

Scales (SCALES): q/k/v/gate/up N(0, 0.04), o/down N(0, 0.06), the embedding N(0, 0.05) with every row scaled by
exp(0.8 N(0, 1)) (a log-normal spread of token-embedding norms, as trained vocabularies have), RMSNorm gains
1 + N(0, 0.05), q/k/v biases N(0, 0.5) (Qwen2.5's real biases are large). Chosen by measurement so that greedy
decoding neither collapses into one repeated token (HF initializer_range 0.02 everywhere does; 43 distinct tokens in
the 4 x 64 here) nor overflows, and most of the reference's top-2 logit margins clear twice the largest CPU bf16
margin error (80 % of the steps; equal-norm embedding rows left 29 %, too few to pin a bf16 decode step against).
"""

import numpy as np
import torch

QWEN25_05B = dict(vocab_size=151936, hidden_size=896, intermediate_size=4864, num_hidden_layers=24,
                  num_attention_heads=14, num_key_value_heads=2, max_position_embeddings=32768,
                  rope_theta=1000000.0, rms_norm_eps=1e-6, tie_word_embeddings=True, bos_token_id=151643,
                  eos_token_id=151645, pad_token_id=151643)
SEED = 20251016


def hf_shapes(cfg=QWEN25_05B):
    """HF Qwen2ForCausalLM state-dict names and shapes, in module order (tied lm_head omitted)."""
    H, I, L = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    hd = H // cfg["num_attention_heads"]
    q, kv = cfg["num_attention_heads"] * hd, cfg["num_key_value_heads"] * hd
    out = [("model.embed_tokens.weight", (cfg["vocab_size"], H))]
    for i in range(L):
        p = f"model.layers.{i}."
        out += [(p + "self_attn.q_proj.weight", (q, H)), (p + "self_attn.q_proj.bias", (q,)),
                (p + "self_attn.k_proj.weight", (kv, H)), (p + "self_attn.k_proj.bias", (kv,)),
                (p + "self_attn.v_proj.weight", (kv, H)), (p + "self_attn.v_proj.bias", (kv,)),
                (p + "self_attn.o_proj.weight", (H, q)), (p + "mlp.gate_proj.weight", (I, H)),
                (p + "mlp.up_proj.weight", (I, H)), (p + "mlp.down_proj.weight", (H, I)),
                (p + "input_layernorm.weight", (H,)), (p + "post_attention_layernorm.weight", (H,))]
    out.append(("model.norm.weight", (H,)))
    return out


SCALES = dict(norm=0.05, bias=0.5, embed=0.05, matrix=0.04, out=0.06, embed_row_sigma=0.8)


def make_state_dict(seed=SEED, scales=None):
    sc = dict(SCALES, **(scales or {}))
    sd = {}
    for i, (name, shape) in enumerate(hf_shapes()):
        g = np.random.Generator(np.random.PCG64(seed * 1000 + i))
        x = torch.from_numpy(g.standard_normal(shape, dtype=np.float32))
        if name.endswith("norm.weight"):
            x = 1.0 + sc["norm"] * x
        elif name.endswith("bias"):
            x = sc["bias"] * x
        elif "embed_tokens" in name:
            rows = np.random.Generator(np.random.PCG64(seed * 1000 + 999_999)).standard_normal((shape[0], 1),
                                                                                             dtype=np.float32)
            x = sc["embed"] * x * torch.from_numpy(np.exp(sc["embed_row_sigma"] * rows))
        elif name.endswith(("o_proj.weight", "down_proj.weight")):
            x = sc["out"] * x
        else:
            x = sc["matrix"] * x
        sd[name] = x
    return sd


def checksum(sd):
    """sha1 of every tensor's bytes."""
    import hashlib

    return {k: hashlib.sha1(v.contiguous().numpy().tobytes()).hexdigest() for k, v in sd.items()}


def prompts(n=4, P=64, seed=SEED):
    """4 x 64-token prompts (ids below the special-token range), rows 1 and 3 left-padded by 5 and 17."""
    g = np.random.Generator(np.random.PCG64(seed + 1))
    ids = torch.from_numpy(g.integers(0, 151643, (n, P), dtype=np.int64))
    am = torch.ones(n, P, dtype=torch.int64)
    for i, npad in enumerate([0, 5, 0, 17][:n]):
        am[i, :npad] = 0
        ids[i, :npad] = QWEN25_05B["pad_token_id"]
    pos = torch.clamp(torch.cumsum(am, -1) - 1, min=0)
    return ids, am, pos
