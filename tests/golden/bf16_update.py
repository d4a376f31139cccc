"""Deterministic CPU-seeded inputs for the bf16 production-path update fixture (``bf16_update.npz``).

A Qwen2.5-0.5B-width model (H 896, I 4864, 14 / 2 heads of 64, V 151936, tied lm_head, qkv bias) at reduced depth
(4 decoder layers), 16 sequences of 48 prompt + 48 response tokens with left padding and EOS-terminated responses.
Shared by make_golden.py (which runs the reference's DataParallelPPOActor on them in fp32 and under its own
torch.autocast(bf16)) and tests/test_bf16_update_gpu.py (which rebuilds the identical tensors on the GPU box); the
~0.9 GB of weights are never committed. Every tensor comes from its own seeded numpy PCG64 stream (bit-identical
across hosts); ``checksum`` pins that. ``sample_index`` gives the fixed element sample of each parameter whose
gradient / update the fixture stores.
"""

import hashlib

import numpy as np
import torch

CFG = dict(vocab_size=151936, hidden_size=896, intermediate_size=4864, num_hidden_layers=4, num_attention_heads=14,
           num_key_value_heads=2, max_position_embeddings=32768, rope_theta=1000000.0, rms_norm_eps=1e-6,
           tie_word_embeddings=True, bos_token_id=151643, eos_token_id=151645, pad_token_id=151643)
SEED = 20261019
B, P, R = 16, 48, 48
N_SAMPLE = 4096


def hf_shapes():
    H, I, L = CFG["hidden_size"], CFG["intermediate_size"], CFG["num_hidden_layers"]
    hd = H // CFG["num_attention_heads"]
    q, kv = CFG["num_attention_heads"] * hd, CFG["num_key_value_heads"] * hd
    out = [("model.embed_tokens.weight", (CFG["vocab_size"], H))]
    for i in range(L):
        p = f"model.layers.{i}."
        out += [(p + "self_attn.q_proj.weight", (q, H)), (p + "self_attn.k_proj.weight", (kv, H)),
                (p + "self_attn.v_proj.weight", (kv, H)), (p + "self_attn.q_proj.bias", (q,)),
                (p + "self_attn.k_proj.bias", (kv,)), (p + "self_attn.v_proj.bias", (kv,)),
                (p + "self_attn.o_proj.weight", (H, q)), (p + "mlp.gate_proj.weight", (I, H)),
                (p + "mlp.up_proj.weight", (I, H)), (p + "mlp.down_proj.weight", (H, I)),
                (p + "input_layernorm.weight", (H,)), (p + "post_attention_layernorm.weight", (H,))]
    out += [("model.norm.weight", (H,))]
    return out


def make_state_dict():
    """HF Qwen2ForCausalLM state dict (fp32; lm_head tied to the embedding)."""
    sd = {}
    for i, (name, shape) in enumerate(hf_shapes()):
        g = np.random.Generator(np.random.PCG64(SEED * 1000 + i))
        x = g.standard_normal(shape, dtype=np.float32)
        if name.endswith("norm.weight"):
            x = 1.0 + 0.05 * x
        elif name.endswith("bias"):
            x = 0.1 * x
        else:  # N(0, 1/sqrt(fan_in)): unit-scale activations and logits
            x = x / np.sqrt(shape[1], dtype=np.float32)
        sd[name] = torch.from_numpy(x)
    return sd


def checksum(sd):
    return {k: hashlib.sha1(v.contiguous().numpy().tobytes()).hexdigest() for k, v in sd.items()}


def sample_index(name, numel):
    """Fixed sample of N_SAMPLE flat element indices of parameter ``name`` (all of them when smaller)."""
    if numel <= N_SAMPLE:
        return np.arange(numel, dtype=np.int64)
    h = int(hashlib.sha1(name.encode()).hexdigest()[:8], 16)
    g = np.random.Generator(np.random.PCG64(SEED + h))
    return np.sort(g.choice(numel, N_SAMPLE, replace=False)).astype(np.int64)


def embed_rows_index(input_ids):
    """Sample of the tied embedding: every row the batch touches (those carry the lookup gradient) plus the fixed
    element sample (lm_head-only rows)."""
    H = CFG["hidden_size"]
    rows = np.unique(input_ids.reshape(-1))
    touched = (rows[:, None] * H + np.arange(0, H, 7)[None, :]).reshape(-1)
    return np.unique(np.concatenate([touched, sample_index("model.embed_tokens.weight", CFG["vocab_size"] * H)]))


GROUPS, N_PER = 4, 4  # the grouped batch: 4 prompts x n = 4 samples


def batch(grouped=False):
    """input_ids, attention_mask, position_ids, responses, response_mask, old_log_probs noise, ref noise and
    advantages: left-padded prompts (0..11 pads), responses of 6..48 tokens ending in EOS then pad.

    ``grouped``: the GRPO layout the trainer hands the actor (ray_trainer.py:1119 ``repeat(n, interleave=True)``):
    GROUPS distinct prompts, each repeated N_PER times in consecutive rows (identical prompt tokens, pads and
    positions), every row with its own response; its own seeded stream (the ungrouped batch is unchanged)."""
    g = np.random.Generator(np.random.PCG64(SEED + (2 if grouped else 1)))
    V, pad, eos = CFG["vocab_size"], CFG["pad_token_id"], CFG["eos_token_id"]
    ids = torch.from_numpy(g.integers(0, 151643, (B, P + R), dtype=np.int64))
    am = torch.ones(B, P + R, dtype=torch.int64)
    npad = g.integers(0, 12, B)
    rlen = g.integers(6, R + 1, B)
    rlen[0] = R  # one full-length response (no EOS inside)
    if grouped:
        assert GROUPS * N_PER == B
        lead = np.repeat(np.arange(GROUPS) * N_PER, N_PER)  # row -> its group's first row
        ids[:, :P] = ids[torch.from_numpy(lead), :P]
        npad = npad[lead]
    for b in range(B):
        am[b, :npad[b]] = 0
        ids[b, :npad[b]] = pad
        if rlen[b] < R:
            ids[b, P + rlen[b] - 1] = eos
            ids[b, P + rlen[b]:] = pad
            am[b, P + rlen[b]:] = 0
    pos = torch.clamp(torch.cumsum(am[:, :P], -1) - 1, min=0)
    pos = torch.cat([pos, pos[:, -1:] + torch.arange(1, R + 1).unsqueeze(0)], -1)
    rmask = am[:, P:].clone()
    noise_old = torch.from_numpy(g.standard_normal((B, R), dtype=np.float32))
    noise_ref = torch.from_numpy(g.standard_normal((B, R), dtype=np.float32))
    adv = torch.from_numpy(g.standard_normal((B, 1), dtype=np.float32)).expand(B, R) * rmask
    assert V > 151643
    return dict(input_ids=ids, attention_mask=am, position_ids=pos, responses=ids[:, P:].clone(), response_mask=rmask,
                noise_old=noise_old, noise_ref=noise_ref, advantages=adv.contiguous())
