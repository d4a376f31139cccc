"""Plain-PyTorch restatement of HF ``Qwen2ForCausalLM`` as the reference runs it — TEST INFRASTRUCTURE ONLY.

The reference's actor / reference / rollout model is HF transformers' Qwen2 (``dp_actor.py:90-280`` calls
``self.actor_module(input_ids, attention_mask, position_ids)``; ``hf_rollout.py:112-124`` calls
``generate``). Transformers is installed here but the checks must not depend on its internals, so this
module restates the math in eager torch ops on any device (CPU by default):

* RMSNorm with fp32 variance, rotate_half RoPE from ``position_ids``, grouped-query attention with the
  causal + key-padding mask applied additively as ``finfo.min`` (a query row with no allowed key is
  therefore uniform over all keys, exactly as HF), SiLU-gated MLP, tied lm_head;
* ``logp_entropy`` = ``logprobs_from_logits`` / ``entropy_from_logits`` on ``logits[:, -R-1:-1] / T``
  (``dp_actor.py:187-230``);
* ``generate_greedy`` = HF greedy ``generate`` with a KV cache and the attention mask grown by one valid
  key per step, EOS -> pad for finished rows (``hf_rollout.py:112-160``).

Pinned by ``tests/test_oracle_golden.py`` against ``tests/golden/tiny_qwen2_rollout.npz`` (outputs of the
reference's HF model, ``tests/golden/make_golden.py::gen_tiny_qwen2``). Parameter names follow the fused
layout of ``dots.rl_amd.qwen2.param_specs`` (qkv and gate_up concatenated) so GPU tests can compare
gradients name by name. Also the model of ``oracle.cpu_baseline``.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def load_hf_state_dict(cfg, sd, device="cpu"):
    """HF state dict -> fused-name fp32 parameter dict."""
    P = {"embed_tokens": sd["model.embed_tokens.weight"]}
    for i in range(cfg.num_hidden_layers):
        p, q = f"model.layers.{i}.", f"layers.{i}."
        P[q + "input_layernorm"] = sd[p + "input_layernorm.weight"]
        P[q + "qkv_proj.weight"] = torch.cat([sd[p + f"self_attn.{x}_proj.weight"] for x in "qkv"], 0)
        if getattr(cfg, "attention_bias", True):  # Llama (LlamaForCausalLM): no q/k/v bias
            P[q + "qkv_proj.bias"] = torch.cat([sd[p + f"self_attn.{x}_proj.bias"] for x in "qkv"], 0)
        P[q + "o_proj"] = sd[p + "self_attn.o_proj.weight"]
        P[q + "post_attention_layernorm"] = sd[p + "post_attention_layernorm.weight"]
        P[q + "gate_up_proj"] = torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0)
        P[q + "down_proj"] = sd[p + "mlp.down_proj.weight"]
    P["norm"] = sd["model.norm.weight"]
    if not cfg.tie_word_embeddings:
        P["lm_head"] = sd["lm_head.weight"]
    return {k: v.to(device=device, dtype=torch.float32) for k, v in P.items()}


def init_params(cfg, seed=0, device="cpu"):
    """HF Qwen2 init: N(0, initializer_range) matrices, unit norms, zero biases (fp32)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * D

    def n(*shape):
        return (torch.randn(*shape, generator=g) * cfg.initializer_range).to(device)

    P = {"embed_tokens": n(cfg.vocab_size, H)}
    for i in range(cfg.num_hidden_layers):
        q = f"layers.{i}."
        P[q + "input_layernorm"] = torch.ones(H, device=device)
        P[q + "qkv_proj.weight"] = n(qkv, H)
        if getattr(cfg, "attention_bias", True):
            P[q + "qkv_proj.bias"] = torch.zeros(qkv, device=device)
        P[q + "o_proj"] = n(H, cfg.num_attention_heads * D)
        P[q + "post_attention_layernorm"] = torch.ones(H, device=device)
        P[q + "gate_up_proj"] = n(2 * I, H)
        P[q + "down_proj"] = n(H, I)
    P["norm"] = torch.ones(H, device=device)
    if not cfg.tie_word_embeddings:
        P["lm_head"] = n(cfg.vocab_size, H)
    return P


def _rms(cfg, x, w):
    return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + cfg.rms_norm_eps))


def _rope_tables(cfg, pos):
    D = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, device=pos.device).float() / D))
    fr = pos.float()[..., None] * inv
    emb = torch.cat([fr, fr], -1)
    return emb.cos()[:, None], emb.sin()[:, None]  # (B, 1, T, D)


def _rope(x, cos, sin):
    d = x.shape[-1] // 2
    return x * cos + torch.cat([-x[..., d:], x[..., :d]], -1) * sin


def _layers(cfg, P, x, pos, allowed, cache=None, koff=0):
    """Decoder stack. allowed (B, Tq, Tk) bool; cache: list of (K, V) (B, Hkv, Tmax, D) written at koff."""
    B, T, _ = x.shape
    Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    cos, sin = _rope_tables(cfg, pos)
    add = (~allowed[:, None]).float() * torch.finfo(torch.float32).min
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}."
        h = _rms(cfg, x, P[p + "input_layernorm"])
        qkv = h @ P[p + "qkv_proj.weight"].t()
        if p + "qkv_proj.bias" in P:
            qkv = qkv + P[p + "qkv_proj.bias"]
        q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], -1)
        q = _rope(q.view(B, T, Hq, D).transpose(1, 2), cos, sin)
        k = _rope(k.view(B, T, Hkv, D).transpose(1, 2), cos, sin)
        v = v.view(B, T, Hkv, D).transpose(1, 2)
        if cache is not None:
            cache[i][0][:, :, koff:koff + T] = k
            cache[i][1][:, :, koff:koff + T] = v
            k = cache[i][0][:, :, :koff + T]
            v = cache[i][1][:, :, :koff + T]
        k = k.repeat_interleave(Hq // Hkv, 1)
        v = v.repeat_interleave(Hq // Hkv, 1)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(D) + add
        o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, T, Hq * D)
        x = x + o @ P[p + "o_proj"].t()
        h2 = _rms(cfg, x, P[p + "post_attention_layernorm"])
        g, u = (h2 @ P[p + "gate_up_proj"].t()).chunk(2, -1)
        x = x + (F.silu(g) * u) @ P[p + "down_proj"].t()
    return _rms(cfg, x, P["norm"])


def _lm_head(cfg, P):
    return P["embed_tokens"] if cfg.tie_word_embeddings else P["lm_head"]


def hidden_states(cfg, P, ids, am, pos):
    """Full-sequence forward -> final-norm hidden (B, T, H) fp32."""
    T = ids.shape[1]
    causal = torch.ones(T, T, dtype=torch.bool, device=ids.device).tril()
    allowed = causal[None] & am.bool()[:, None, :]
    return _layers(cfg, P, P["embed_tokens"][ids], pos, allowed)


def logp_entropy(cfg, P, ids, am, pos, resp, temperature=1.0):
    """log pi(response token) and entropy over the response positions (dp_actor.py:187-230)."""
    R = resp.shape[1]
    h = hidden_states(cfg, P, ids, am, pos)
    logits = (h[:, -R - 1:-1] @ _lm_head(cfg, P).t()) / temperature
    lsm = torch.log_softmax(logits, -1)
    logp = lsm.gather(-1, resp[..., None])[..., 0]
    ent = -(lsm.exp() * lsm).sum(-1)
    return logp, ent


@torch.no_grad()
def generate_greedy(cfg, P, ids, am, pos, R, eos_ids, pad_id, max_steps=None):
    """HF greedy generate with a KV cache (hf_rollout.py:112-160): returns responses (B, R) int64.

    ``max_steps`` < R stops early (bounded CPU samples) and leaves the rest of ``responses`` as pad."""
    B, Pl = ids.shape
    Hkv, D = cfg.num_key_value_heads, cfg.head_dim
    steps = R if max_steps is None else min(R, max_steps)
    cache = [(torch.zeros(B, Hkv, Pl + steps, D, device=ids.device), torch.zeros(B, Hkv, Pl + steps, D, device=ids.device))
             for _ in range(cfg.num_hidden_layers)]
    valid = torch.zeros(B, Pl + steps, dtype=torch.bool, device=ids.device)
    valid[:, :Pl] = am.bool()
    causal = torch.ones(Pl, Pl, dtype=torch.bool, device=ids.device).tril()
    h = _layers(cfg, P, P["embed_tokens"][ids], pos, causal[None] & valid[:, None, :Pl], cache, 0)[:, -1]
    W = _lm_head(cfg, P)
    eos = torch.tensor(list(eos_ids), device=ids.device)
    responses = torch.full((B, R), pad_id, dtype=torch.int64, device=ids.device)
    alive = torch.ones(B, dtype=torch.bool, device=ids.device)
    last = pos[:, -1]
    for t in range(steps):
        tok = torch.argmax(h @ W.t(), -1)
        tok = torch.where(alive, tok, torch.full_like(tok, pad_id))
        responses[:, t] = tok
        alive &= ~torch.isin(tok, eos)
        if t + 1 == steps:
            break
        valid[:, Pl + t] = True
        x = P["embed_tokens"][tok][:, None]
        h = _layers(cfg, P, x, (last + 1 + t)[:, None], valid[:, None, :Pl + t + 1], cache, Pl + t)[:, 0]
    return responses
