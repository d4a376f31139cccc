"""Qwen2 decoder (Qwen2.5-0.5B architecture) laid out for MI355X training + decode.

Parameters live in three flat device buffers (``ParamStore``): fp32 master weights, a compute copy (bf16)
that the GEMMs read, and fp32 gradients. The optimizer (HIP AdamW kernel) updates the master buffer and
rewrites the bf16 copy in the same pass; data-parallel gradient averaging is a single RCCL all-reduce of
the flat gradient; GEMM weight gradients accumulate straight into fp32 (drl_gemm bf16 x bf16 -> fp32 with
beta = 1), so micro-batch accumulation never rounds through bf16.

Per decoder layer every bf16 GEMM (forward, input gradient, weight gradient, lm_head) runs on the hand-written
stream-K GEMM ``drl_gemm`` (``csrc/gemm_sk.hip``) and everything else on hand-written HIP kernels:
``csrc/layers.hip`` (residual-add + RMSNorm, QKV split + RoPE + grouped-query re-layout so the 7 query
heads of a KV head share one K/V stream, SwiGLU), ``csrc/flash_attn.hip`` (fused MFMA attention forward
and backward for bf16 full sequences; the fp32 parity model uses fp32-score GEMMs + masked softmax) and
``csrc/attention.hip`` (decode attention over the preallocated KV cache). The backward of a whole layer
is hand-written (``_DecoderLayer``).

Semantics follow HF ``Qwen2ForCausalLM`` as the reference runs it (dp_actor.py:110 autocast bf16 over
fp32 master weights): bf16 GEMM inputs with fp32 accumulation, fp32 RMSNorm and residual stream, fp32
attention scores, bf16 probabilities into the PV GEMM. ``compute_dtype=float32`` runs the same kernels
in fp32 end to end (the parity model checked against HF / golden greedy tokens).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import native
from .torch_functional import fused_linear_logprob_entropy


@dataclass
class Qwen2Config:
    vocab_size: int = 151936
    hidden_size: int = 896
    intermediate_size: int = 4864
    num_hidden_layers: int = 24
    num_attention_heads: int = 14
    num_key_value_heads: int = 2
    rope_theta: float = 1000000.0
    rms_norm_eps: float = 1e-6
    tie_word_embeddings: bool = True
    initializer_range: float = 0.02
    max_position_embeddings: int = 32768
    bos_token_id: int = 151643
    eos_token_id: int = 151645
    pad_token_id: int = 151643
    # > 0: token-classification head `score` Linear(H, num_labels, bias=True) instead of the lm_head (the
    # critic the reference loads with AutoModelForTokenClassification, num_labels=1, fsdp_workers.py:1045)
    num_labels: int = 0
    # False: Llama-family attention (no q/k/v bias; LlamaForCausalLM, config #4's Llama-3-8B). The kernels are
    # shared: the qkv GEMM epilogues read a constant zero bias instead of a parameter.
    attention_bias: bool = True
    rope_scaling: dict | None = None
    # HF's attention switch: "eager" = the unfused bf16 attention (fp32 score GEMM on torch bmm + the HIP masked softmax
    # + PV bmm), an explicit opt-in for head dims the fused kernels do not take (the tiny test models' 16); anything
    # else ("sdpa", "flash_attention_2", None) = the fused kernels (csrc/flash_attn.hip), which raise when they cannot
    attn_implementation: str | None = None
    model_type: str = "qwen2"
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @classmethod
    def from_dict(cls, d):
        known = {k: v for k, v in d.items() if k in cls.__dataclass_fields__}
        return cls(**known)


def param_specs(cfg: Qwen2Config):
    """(name, shape, kind) in buffer order; kind: 'gemm' (read through the compute copy) or 'small' (fp32)."""
    H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd
    specs = [("embed_tokens", (cfg.vocab_size, H), "gemm")]
    for i in range(cfg.num_hidden_layers):
        p = f"layers.{i}."
        specs += [
            (p + "input_layernorm", (H,), "small"),
            (p + "qkv_proj.weight", (qkv, H), "gemm"),
        ]
        if cfg.attention_bias:
            specs.append((p + "qkv_proj.bias", (qkv,), "gemm"))  # GEMM epilogue operand: read in the compute dtype
        specs += [
            (p + "o_proj", (H, cfg.num_attention_heads * hd), "gemm"),
            (p + "post_attention_layernorm", (H,), "small"),
            (p + "gate_up_proj", (2 * I, H), "gemm"),
            (p + "down_proj", (H, I), "gemm"),
        ]
    specs.append(("norm", (H,), "small"))
    if cfg.num_labels > 0:  # critic value head, read in the compute dtype like the autocast Linear
        specs += [("score.weight", (cfg.num_labels, H), "gemm"), ("score.bias", (cfg.num_labels,), "gemm")]
    elif not cfg.tie_word_embeddings:
        specs.append(("lm_head", (cfg.vocab_size, H), "gemm"))
    return specs


class ParamStore:
    """Flat parameter/gradient buffers with named views (64-element = 256-B aligned offsets).

    Layout: the fp32 'small' parameters (norm weights, read by the kernels straight from the fp32 master) come
    first, then the GEMM parameters (read through the compute-dtype copy), each group in param_specs order.
    Buffers by mode:
      * trainable, replicated   : fp32 master (numel), compute copy (numel; the master itself in fp32 mode),
                                  fp32 grad (numel);
      * trainable, ``shard=(rank, world)`` (ZeRO-style, what FSDP FULL_SHARD gives the reference,
        fsdp_workers.py:397-418): the GEMM region's fp32 master and the optimizer moments are split into
        `world` equal contiguous shards; master = [small region | this rank's shard], the compute copy and
        the fp32 gradient stay full (all-gathered after every optimizer step / reduce-scattered before it);
      * frozen (trainable=False) bf16: fp32 master of the small region only + the bf16 compute copy.
    ``small`` is always master[:n_small]."""

    ALIGN = 64

    def __init__(self, cfg: Qwen2Config, device, compute_dtype=torch.bfloat16, trainable=True, shard=None,
                 group=None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.trainable = trainable
        self.specs = param_specs(cfg)
        self.rank, self.world = (int(shard[0]), int(shard[1])) if shard is not None else (0, 1)
        self.sharded = trainable and self.world > 1
        self.group = group
        A = self.ALIGN

        def padded(n):
            return (n + A - 1) // A * A

        pos, off = {}, 0
        for name, shape, kind in self.specs:
            if kind == "small":
                pos[name] = off
                off += padded(math.prod(shape))
        self.n_small = off
        for name, shape, kind in self.specs:
            if kind != "small":
                pos[name] = off
                off += padded(math.prod(shape))
        gemm_len = off - self.n_small
        gemm_len = (gemm_len + A * self.world - 1) // (A * self.world) * (A * self.world)
        self.numel = self.n_small + gemm_len
        self.shard_len = gemm_len // self.world
        self.offsets = {name: (pos[name], shape, kind) for name, shape, kind in self.specs}  # spec order
        self.n_params = sum(math.prod(s) for _, s, _ in self.specs)
        f32 = torch.float32
        if self.sharded:
            self.master = torch.zeros(self.n_small + self.shard_len, dtype=f32, device=self.device)
            self.compute = torch.zeros(self.numel, dtype=compute_dtype, device=self.device)
        elif not trainable and compute_dtype != f32:
            self.master = torch.zeros(self.n_small, dtype=f32, device=self.device)
            self.compute = torch.zeros(self.numel, dtype=compute_dtype, device=self.device)
        else:
            self.master = torch.zeros(self.numel, dtype=f32, device=self.device)
            self.compute = self.master if compute_dtype == f32 else torch.zeros(self.numel, dtype=compute_dtype,
                                                                               device=self.device)
        self.small = self.master[:self.n_small]
        self.grad = torch.zeros(self.numel, dtype=f32, device=self.device) if trainable else None
        self.version = 0  # bumped whenever the compute copy changes (derived copies, e.g. Qwen2Model.wt, refresh)
        self._views = {}
        for name, (o, shape, kind) in self.offsets.items():
            n = math.prod(shape)
            w = (self.small if kind == "small" else self.compute)[o:o + n].view(shape)
            g = self.grad[o:o + n].view(shape) if trainable else None
            self._views[name] = (w, g)

    def w(self, name):
        return self._views[name][0]

    def g(self, name):
        return self._views[name][1]

    def master_range(self):
        """[lo, hi) of the flat layout held by master[n_small:] (the GEMM region, or this rank's shard of it)."""
        if self.master.numel() == self.n_small:
            return self.n_small, self.n_small
        if self.sharded:
            lo = self.n_small + self.rank * self.shard_len
            return lo, lo + self.shard_len
        return self.n_small, self.numel

    def _put(self, name, vals):
        """Write one parameter's fp32 values (flat) into the master (the part this rank holds) and the
        compute copy."""
        self.version += 1
        o, shape, kind = self.offsets[name]
        n = math.prod(shape)
        if kind == "small":
            self.small[o:o + n].copy_(vals)
            return
        lo, hi = self.master_range()
        a, b = max(o, lo), min(o + n, hi)
        if a < b:
            self.master[self.n_small + a - lo:self.n_small + b - lo].copy_(vals[a - o:b - o])
        if self.compute is not self.master:
            self.compute[o:o + n].copy_(vals)

    @torch.no_grad()
    def init_random(self, seed: int):
        """HF Qwen2 init: N(0, initializer_range) for matrices, ones for norms, zeros for biases. Values are
        drawn per parameter in param_specs order (the same numbers in every layout / sharding)."""
        gen = torch.Generator(device=self.device).manual_seed(seed)
        for name, (o, shape, kind) in self.offsets.items():
            vals = torch.empty(math.prod(shape), dtype=torch.float32, device=self.device)
            if name.endswith("layernorm") or name == "norm":
                vals.fill_(1.0)
            elif name.endswith("bias"):
                vals.zero_()
            else:
                vals.normal_(0.0, self.cfg.initializer_range, generator=gen)
            self._put(name, vals)
        self.refresh_compute()

    @torch.no_grad()
    def refresh_compute(self):
        """compute copy <- master (GEMM region); sharded: this rank's shard, then an all-gather."""
        self.version += 1
        if self.compute is self.master:
            return
        lo, hi = self.master_range()
        if hi > lo:
            self.compute[lo:hi].copy_(self.master[self.n_small:])
        if self.sharded:
            self.all_gather_compute()

    def all_gather_compute(self):
        """Every rank's shard of the compute copy's GEMM region -> the full region on every rank (RCCL
        all-gather, in place)."""
        lo, hi = self.master_range()
        full = self.compute[self.n_small:]
        if dist.get_backend(self.group) == "nccl" or full.device.type == "cpu":
            dist.all_gather_into_tensor(full, self.compute[lo:hi], group=self.group)
        else:  # gloo on device tensors (ranks sharing one GPU in a test): zero the other shards + SUM, exact
            mine = self.compute[lo:hi].clone()
            full.zero_()
            self.compute[lo:hi].copy_(mine)
            dist.all_reduce(full, op=dist.ReduceOp.SUM, group=self.group)

    @torch.no_grad()
    def copy_from(self, other: "ParamStore"):
        """This store's weights := other's (same config): the small fp32 region and the compute copy; a
        replicated fp32 master gets the full values (sharded other: gathered through its compute copy)."""
        self.version += 1
        self.small.copy_(other.small)
        if self.compute is not self.master:
            self.compute.copy_(other.compute.to(self.compute.dtype))
        lo, hi = self.master_range()
        if hi > lo:
            olo, ohi = other.master_range()
            if (olo, ohi) == (lo, hi):
                self.master[self.n_small:].copy_(other.master[other.n_small:])
            else:
                self.master[self.n_small:].copy_(other.compute[lo:hi].to(torch.float32))

    @torch.no_grad()
    def load_state_dict_hf(self, sd: dict):
        """Load HF Qwen2ForCausalLM weights (q/k/v and gate/up are concatenated into the fused layouts)."""
        cfg = self.cfg

        def put(name, t):
            self._put(name, t.reshape(-1).to(device=self.device, dtype=torch.float32))

        put("embed_tokens", sd["model.embed_tokens.weight"])
        for i in range(cfg.num_hidden_layers):
            p, q = f"model.layers.{i}.", f"layers.{i}."
            put(q + "input_layernorm", sd[p + "input_layernorm.weight"])
            put(q + "qkv_proj.weight", torch.cat([sd[p + f"self_attn.{x}_proj.weight"] for x in "qkv"], 0))
            if cfg.attention_bias:
                put(q + "qkv_proj.bias", torch.cat([sd[p + f"self_attn.{x}_proj.bias"] for x in "qkv"], 0))
            put(q + "o_proj", sd[p + "self_attn.o_proj.weight"])
            put(q + "post_attention_layernorm", sd[p + "post_attention_layernorm.weight"])
            put(q + "gate_up_proj", torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0))
            put(q + "down_proj", sd[p + "mlp.down_proj.weight"])
        put("norm", sd["model.norm.weight"])
        if cfg.num_labels > 0:
            put("score.weight", sd["score.weight"])
            put("score.bias", sd["score.bias"] if "score.bias" in sd else torch.zeros(cfg.num_labels))
        elif not cfg.tie_word_embeddings:
            put("lm_head", sd["lm_head.weight"])

    def zero_grad(self):
        if self.grad is not None:
            self.grad.zero_()

    def memory_bytes(self):
        """Bytes of device memory held by this store's buffers."""
        bufs = {id(t): t for t in (self.master, self.compute, self.grad) if t is not None}
        return sum(t.numel() * t.element_size() for t in bufs.values())

    def layer_range(self, i):
        """[start, end) of decoder layer i's GEMM parameters in the flat buffers (contiguous; its two norm
        weights live in the small region at the front)."""
        names = [n for n, _, k in self.specs if n.startswith(f"layers.{i}.") and k != "small"]
        start = self.offsets[names[0]][0]
        last = self.offsets[names[-1]]
        return start, last[0] + math.prod(last[1])


# --------------------------------------------------------------------------------------------- GEMM helpers
# Every bf16 GEMM of the full-sequence passes — forward, dgrad and wgrad of each projection and of the lm_head — runs
# on csrc/gemm_sk.hip (drl_gemm: 256 x 256 ping-pong tiles, weights read in their stored layout for the dgrad, fp32
# accumulation into the gradient buffer for the wgrad); a reduction dimension that is not a multiple of 64 is
# zero-padded on the device (native._pad_to_64) — there is no library fallback. The fp32 parity model
# (compute_dtype=float32) uses torch's fp32 GEMMs.


def _sk(*ts):
    """bf16 device operands: the drl_gemm path (every bf16 GEMM of the model)."""
    return all(t.dtype == torch.bfloat16 and t.is_cuda for t in ts)


def _fp32_only(t):
    if t.dtype != torch.float32:
        raise NotImplementedError(f"dtype {t.dtype}: bf16 GEMMs run on drl_gemm (device tensors); torch GEMMs serve "
                                  "only the fp32 parity model")


def linear(x, w, bias=None):
    """y = x W^T (+ bias) for x (N, in), w (out, in) in the compute dtype (bias added before the single rounding)."""
    if _sk(x, w):
        return native.linear_fwd(x, w, bias=bias)
    _fp32_only(x)
    return torch.addmm(bias, x, w.t()) if bias is not None else x @ w.t()


def dgrad(dy, w):
    """dx = dy W (F.linear's grad_input) for dy (N, out), w (out, in)."""
    if _sk(dy, w):
        return native.linear_dgrad(dy, w)
    _fp32_only(dy)
    return dy @ w


def acc_wgrad(gw, dy, x):
    """gw (out, in) fp32 += dy^T x  with dy (N, out), x (N, in) in the compute dtype (fp32 accumulation in place)."""
    if _sk(dy, x):
        native.linear_wgrad(gw, dy, x)
    else:
        _fp32_only(dy)
        gw.addmm_(dy.t(), x)


# The weight gradient of a projection runs on a side stream while its input gradient runs on the current one: the
# pair's workgroups share the CUs (gate_up's weight gradient is 152 tiles of 256 x 256 at any row count, the other
# 104 CUs otherwise idle for its ~2 ms). It pays since whole-tile drl_gemm launches one workgroup per tile (the
# hardware deals tiles to CUs as they free up; a persistent grid's static rounds could not take the idle CUs):
# update 1.44 -> 1.38 s (round 3). DRL_CONCURRENT_WGRAD=0 turns it off. Round 5: only where the weight gradient runs
# as whole tiles that leave CUs idle (gate_up: 152 tiles of 256 x 256 over 642 k-pairs); the small projections'
# weight gradients (qkv 20, o 16 tiles) now split K over every CU (csrc/gemm_sk.hip), and beside their input
# gradients the pair took longer than the two in sequence (qkv 468 vs 190 + 242 us, o 392 vs 151 + 184 us per call,
# profiles/r05_gemm_launches_splitk_concurrent.txt).
CONCURRENT_WGRAD = os.environ.get("DRL_CONCURRENT_WGRAD", "1") != "0"
CONCURRENT_DOWN = os.environ.get("DRL_CONCURRENT_DOWN", "0") == "1"  # measurement switch: down_proj's pair concurrent
_SIDE_STREAMS = {}
_CU_COUNT = {}


def _cus(device):
    dev = device.index
    if dev not in _CU_COUNT:
        _CU_COUNT[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CU_COUNT[dev]


def _concurrent_pair(gw):
    """The weight gradient gw (out, in) runs beside its input gradient when drl_gemm deals it as whole 256 x 256 tiles
    that fill more than half of the CUs but not all of them (gemm_sk.hip's automatic decomposition)."""
    cus = _cus(gw.device)
    tiles = -(-gw.shape[0] // 256) * -(-gw.shape[1] // 256)
    return cus < 2 * tiles and tiles < cus


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev.index)
    if s is None:
        s = _SIDE_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return s


def dgrad_wgrad(dy, w, gw, x):
    """dx = dy W and gw (fp32) += dy^T x for one projection (dy (N, out), w (out, in), x (N, in)); returns dx. On
    drl_gemm the weight gradient is launched first on the side stream (its own workspace slot) and joined before
    returning, so callers see plain stream order."""
    if not (CONCURRENT_WGRAD and _sk(dy, w, x) and _concurrent_pair(gw)):
        dx = dgrad(dy, w)
        acc_wgrad(gw, dy, x)
        return dx
    # co-residency rule (c) of csrc/gemm_sk.hip: at most one of two concurrent launches may spin-wait
    cus = _cus(dy.device)
    assert not (native.gemm_spins(gw.shape[0], gw.shape[1], dy.shape[0], cus=cus) and
                native.gemm_spins(dy.shape[0], w.shape[1], dy.shape[1], cus=cus)), "two spinning drl_gemm plans side by side"
    main = torch.cuda.current_stream()
    side = _side_stream(dy.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        native.linear_wgrad(gw, dy, x, ws_slot=1)
    dx = native.linear_dgrad(dy, w)
    main.wait_stream(side)
    return dx


def bmm_f32(a, b):
    """Batched a @ b (bf16 or fp32 inputs) with an fp32 result: the fp32 parity model's attention scores (torch
    bmm); the bf16 model runs the fused attention kernels instead (csrc/flash_attn.hip)."""
    if a.dtype == torch.float32:
        return torch.bmm(a, b)
    return torch.bmm(a, b, out_dtype=torch.float32)


class _Linear(torch.autograd.Function):
    """y = x W^T; backward dx = dy W, dW += dy^T x in fp32 (lm_head over the response rows)."""

    @staticmethod
    def forward(ctx, x, w, gw, dummy):
        ctx.save_for_backward(x, w)
        ctx.gw = gw
        return linear(x.reshape(-1, x.shape[-1]), w).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous().reshape(-1, dy.shape[-1])
        if ctx.gw is not None:
            acc_wgrad(ctx.gw, dy, x.reshape(-1, x.shape[-1]))
        return dgrad(dy, w).view(*x.shape), None, None, None


class _Embedding(torch.autograd.Function):
    """fp32 residual stream input; backward accumulates into the fp32 embedding gradient through aten's
    embedding_dense_backward (sorted ids, segment sums: deterministic — the nn.Embedding backward the reference runs).
    An index_add_ scatter is atomic on the GPU: its summation order changed run to run (tools/probes/det_probe2.py:
    ~1500 of the 131072 tiny-model embedding-gradient entries differed between identical steps)."""

    @staticmethod
    def forward(ctx, ids, w, gw, dummy):
        ctx.save_for_backward(ids)
        ctx.gw = gw
        return F.embedding(ids, w).to(torch.float32)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        if ctx.gw is not None:
            g = torch.ops.aten.embedding_dense_backward(dy.reshape(-1, dy.shape[-1]).to(torch.float32),
                                                        ids.reshape(-1), ctx.gw.shape[0], -1, False)
            ctx.gw.add_(g)
        return None, None, None, None


# --------------------------------------------------------------------------------------------- decoder layer
# Full-sequence projections (bias / SwiGLU fused in the epilogue) on drl_gemm (above) for every row count; torch GEMMs
# only for the fp32 parity model.
def _hip_gemm(x):
    if _sk(x):
        return True
    _fp32_only(x)
    return False


def _layer_forward(m, i, x_prev, delta, pos, key_valid, save, cache=None, koff=0, koff_dev=None, rm=None):
    """x = x_prev (+ delta); returns (x2 = x + attn(x), mlp_out) — the next consumer adds them.

    ``save`` (dict or None) receives the activations the hand-written backward needs. ``koff_dev`` (device
    int64 (1,)) is the cache position of a single decode token kept on the device (graph capture). With ``rm``
    (RmPad) x_prev / delta hold only the attended tokens (1, nnz, H): norms and GEMMs run on the nnz rows, q / k / v
    are scattered into the padded (B, T) layout for RoPE + attention and the attention output is gathered back."""
    cfg, s, dt = m.cfg, m.store, m.dtype
    B, T, H = x_prev.shape
    Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    G = Hq // Hkv
    p = f"layers.{i}."
    dev = x_prev.device
    x = torch.empty_like(x_prev) if delta is not None else x_prev
    h1 = torch.empty(B, T, H, dtype=dt, device=dev)
    rstd1 = torch.empty(B * T, dtype=torch.float32, device=dev) if save is not None else None
    native.add_rmsnorm_fwd(x_prev, delta, x if delta is not None else None, s.w(p + "input_layernorm"), h1, rstd1,
                           cfg.rms_norm_eps)
    if _hip_gemm(h1):
        qkv = native.linear_fwd(h1.view(B * T, H), s.w(p + "qkv_proj.weight"), bias=m.qkv_bias(i))
    else:
        qkv = torch.addmm(m.qkv_bias(i), h1.view(B * T, H), s.w(p + "qkv_proj.weight").t())
    src_rows = None
    if rm is not None:  # RoPE reads the packed qkv through the inverse map: no padded copy of it
        src_rows = rm.inv
        B, T = rm.B, rm.T
    else:
        qkv = qkv.view(B, T, -1)
    q = torch.empty(B, Hkv, G, T, D, dtype=dt, device=dev)
    # bf16 full-sequence passes run the fused MFMA attention (csrc/flash_attn.hip): log-probs and prefill
    # forward-only, the training forward with the LSE its fused backward needs; the unfused path (fp32 scores
    # GEMM + masked softmax + PV GEMM, probabilities kept for the backward) serves the fp32 parity model
    flash_ok = T > 1 and dt == torch.bfloat16 and D in (64, 128) and G <= 8 and key_valid.stride(0) % 4 == 0
    flash = save is None and flash_ok
    if dt == torch.bfloat16 and not (cache is not None and T == 1):
        # bf16 full-sequence attention is the fused kernel pair unless the config asks for eager attention: no silent
        # torch bmm / softmax fallback
        if cfg.attn_implementation == "eager":
            flash_ok = flash = False
        elif not flash_ok:
            raise NotImplementedError(f"bf16 attention: the fused kernels (csrc/flash_attn.hip) need head_dim 64 / 128 "
                                      f"and <= 8 query heads per KV head (head_dim {D}, {G} per KV head, T {T}); "
                                      "attn_implementation='eager' selects the unfused path")
        elif save is not None and cache is None and T % 8 != 0:
            raise NotImplementedError(f"bf16 training pass over T = {T} positions: the fused attention backward needs "
                                      "T % 8 == 0 (pad prompt_length + response_length to a multiple of 8)")
    if save is not None and flash_ok and cache is None and T % 8 == 0:
        # training forward: fused attention that saves only the LSE; the backward (flash_attn_bwd)
        # recomputes P and needs a head-dim-major copy of k besides row-major k and v
        kbuf = torch.empty(B, Hkv, T, D, dtype=dt, device=dev)
        vbuf = torch.empty_like(kbuf)
        kt = torch.empty(B, Hkv, D, T, dtype=dt, device=dev)
        vt = torch.empty(B, Hkv, D, T, dtype=dt, device=dev)
        qs = getattr(rm, "q_start", None)  # prefix sharing: q rows the fused kernels never read are not written
        native.rope_qkv_fwd(qkv, pos, m.cos, m.sin, Hq, Hkv, D, q, kbuf, vbuf, kt=kt, vt=vt, src_rows=src_rows,
                            q_skip=qs)
        lse = torch.empty(B, Hkv, G, T, dtype=torch.float32, device=dev)
        if rm is not None:
            # packed rows written by the attention itself; the backward reads O through the same map
            rows = getattr(rm, "inv_own", rm.inv)
            attn = torch.empty(rm.nnz, Hq * D, dtype=dt, device=dev)
            native.flash_attn_fwd(q, kbuf, vt, key_valid, attn, lse=lse, q_start=qs, out_rows=rows)
            attn = attn.view(1, rm.nnz, -1)
            save["o_rows"] = rows
        else:
            attn = torch.empty(B, T, Hq * D, dtype=dt, device=dev)
            native.flash_attn_fwd(q, kbuf, vt, key_valid, attn, lse=lse, q_start=qs)
        del vt
        save.update(kt=kt, lse=lse, key_valid=key_valid, q_start=qs)
        P = "flash"
        return _layer_mlp(m, i, x, attn, save, kbuf, vbuf, P, q, h1, rstd1)
    vt = None
    if cache is None:
        kbuf = torch.empty(B, Hkv, T, D, dtype=dt, device=dev)
        if flash:
            vt = torch.empty(B, Hkv, D, (T + 7) // 8 * 8, dtype=dt, device=dev)
            vbuf = None
        else:
            vbuf = torch.empty_like(kbuf)
        koff = 0
    else:  # bf16 caches keep V head-dim-major (cache.vt), the layout of the MFMA prefill / decode kernels
        kbuf, vbuf = cache.k[i], cache.v[i]
        vt = cache.vt[i]
    qs = getattr(rm, "q_start", None) if flash and cache is None else None
    native.rope_qkv_fwd(qkv, pos, m.cos, m.sin, Hq, Hkv, D, q, kbuf, vbuf, koff, koff_dev, vt=vt, src_rows=src_rows,
                        q_skip=qs)
    L = koff + T
    if flash and rm is not None and cache is None:
        # forward-only pass over packed rows: the attention writes the packed rows itself (each padded query to its
        # own packed row; pads without one and the shared copies are not written) — no padded output, no row copy
        attn = torch.empty(rm.nnz, Hq * D, dtype=dt, device=dev)
        native.flash_attn_fwd(q, kbuf, vt, key_valid, attn, Tk=L, qoff=L - T, q_start=getattr(rm, "q_start", None),
                              out_rows=getattr(rm, "inv_own", rm.inv))
        return _layer_mlp(m, i, x, attn.view(1, rm.nnz, -1), save, kbuf, vbuf, None, q, h1, rstd1)
    if flash:
        attn = torch.empty(B, T, Hq * D, dtype=dt, device=dev)
        native.flash_attn_fwd(q, kbuf, vt, key_valid, attn, Tk=L, qoff=L - T, q_start=getattr(rm, "q_start", None))
        P = None
    elif cache is not None and T == 1:
        # one new token: decode attention streams the cache once (MFMA kernel over V^T for bf16 caches,
        # csrc/flash_attn.hip; VALU kernel over row-major V for the fp32 parity model, csrc/attention.hip)
        attn = torch.empty(B, 1, Hq * D, dtype=dt, device=dev)
        Lk = L if koff_dev is None else kbuf.shape[2]  # device position: the kernel stops at koff_dev
        if vt is not None:
            native.decode_attention_vt(q.view(B, Hkv, G, D), kbuf, vt, key_valid, Lk, attn, qpos_dev=koff_dev,
                                       group=cache.group, shared_keys=cache.shared)
        else:
            native.decode_attention(q.view(B, Hkv, G, D), kbuf, vbuf, key_valid, Lk, attn, qpos_dev=koff_dev)
        P = None
    else:
        k3 = kbuf[:, :, :L].reshape(B * Hkv, L, D)
        v3 = vbuf[:, :, :L].reshape(B * Hkv, L, D)
        q3 = q.view(B * Hkv, G * T, D)
        S = bmm_f32(q3, k3.transpose(1, 2))  # (B*Hkv, G*T, L) fp32 scores
        P = torch.empty(B * Hkv, G * T, L, dtype=dt, device=dev)
        native.masked_softmax_fwd(S, P, key_valid, B, Hkv * G, T, L, L - T, 1.0 / math.sqrt(D))
        del S
        O = torch.bmm(P, v3)  # (B*Hkv, G*T, D)
    if P is None:
        pass
    elif T == 1:
        attn = O.view(B, 1, Hq * D)
    else:
        attn = O.view(B, Hkv, G, T, D).permute(0, 3, 1, 2, 4).reshape(B, T, Hq * D)
    return _layer_mlp(m, i, x, _repack(rm, attn, save), save, kbuf, vbuf, P, q, h1, rstd1)


def _repack(rm, attn, save):
    """Padded attention output (B, T, Hq*D) -> the packed rows (1, nnz, Hq*D) under remove-padding (the padded
    copy is kept for the fused attention backward)."""
    if rm is None:
        return attn
    if save is not None:
        save["attn_pad"] = attn
    return rm.pack(attn.view(rm.B * rm.T, -1)).view(1, rm.nnz, -1)


def _layer_mlp(m, i, x, attn, save, kbuf, vbuf, P, q, h1, rstd1):
    """o_proj + residual + post-attention RMSNorm + SwiGLU MLP of layer i (shared by both attention paths)."""
    cfg, s, dt = m.cfg, m.store, m.dtype
    B, T, H = x.shape
    Hq = cfg.num_attention_heads
    D = cfg.head_dim
    p = f"layers.{i}."
    dev = x.device
    if _hip_gemm(attn):
        o = native.linear_fwd(attn.reshape(B * T, Hq * D), s.w(p + "o_proj"))
    else:
        o = attn.view(B * T, Hq * D) @ s.w(p + "o_proj").t()
    x2 = torch.empty_like(x)
    h2 = torch.empty(B, T, H, dtype=dt, device=dev)
    rstd2 = torch.empty(B * T, dtype=torch.float32, device=dev) if save is not None else None
    native.add_rmsnorm_fwd(x, o, x2, s.w(p + "post_attention_layernorm"), h2, rstd2, cfg.rms_norm_eps)
    if _hip_gemm(h2):
        # SwiGLU fused into the gate_up GEMM's epilogue; gu = [g | u] written only when the backward needs it
        gu = torch.empty(B * T, 2 * cfg.intermediate_size, dtype=dt, device=dev) if save is not None else None
        a = native.linear_fwd(h2.view(B * T, H), s.w(p + "gate_up_proj"), swiglu=True, out_gu=gu)
    else:
        gu = h2.view(B * T, H) @ s.w(p + "gate_up_proj").t()
        a = torch.empty(B * T, cfg.intermediate_size, dtype=dt, device=dev)
        native.swiglu_fwd(gu, a)
    mlp = linear(a, s.w(p + "down_proj")).view(B, T, H)
    if save is not None:
        save.update(x=x, rstd1=rstd1, h1=h1, q=q, k=kbuf, v=vbuf, P=P, attn=attn, x2=x2, rstd2=rstd2, h2=h2,
                    gu=gu, a=a)
    return x2, mlp


class _DecoderLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_prev, delta, m, i, pos, key_valid, rm=None):
        save = {}
        x2, mlp = _layer_forward(m, i, x_prev, delta, pos, key_valid, save, rm=rm)
        ctx.m, ctx.i, ctx.save, ctx.pos, ctx.rm = m, i, save, pos, rm
        ctx.has_delta = delta is not None
        return x2, mlp

    @staticmethod
    def backward(ctx, g_x2, g_mlp):
        m, i, sv = ctx.m, ctx.i, ctx.save
        cfg, s, dt = m.cfg, m.store, m.dtype
        p = f"layers.{i}."
        B, T, H = sv["x"].shape
        Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        G = Hq // Hkv
        N = B * T
        # the residual gradient passes through the first RMSNorm backward into a fresh buffer (no clone pass)
        g_res = g_x2.to(torch.float32).contiguous()
        dx2 = torch.empty_like(g_res)
        lowp = dt == torch.bfloat16  # the bf16 operand of the next dgrad comes out of the norm backward's pass
        dm = g_mlp.to(dt).contiguous().view(N, H)
        # MLP
        if _sk(dm, sv["gu"]):
            # down_proj dgrad with the SwiGLU backward in its epilogue (d a never written)
            if CONCURRENT_DOWN:
                H_, I_ = s.w(p + "down_proj").shape
                cus = _cus(dm.device)
                assert not (native.gemm_spins(H_, I_, N, cus=cus) and
                            native.gemm_spins(N, I_, H_, native.GEMM_SWIGLU_BWD, cus=cus)), \
                    "two spinning drl_gemm plans side by side"
                main = torch.cuda.current_stream()
                side = _side_stream(dm.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    native.linear_wgrad(s.g(p + "down_proj"), dm, sv["a"], ws_slot=1)
                dgu = native.linear_dgrad_swiglu_bwd(dm, s.w(p + "down_proj"), sv["gu"])
                main.wait_stream(side)
            else:
                acc_wgrad(s.g(p + "down_proj"), dm, sv["a"])
                dgu = native.linear_dgrad_swiglu_bwd(dm, s.w(p + "down_proj"), sv["gu"])
        else:
            da = dgrad_wgrad(dm, s.w(p + "down_proj"), s.g(p + "down_proj"), sv["a"])
            dgu = torch.empty_like(sv["gu"])
            native.swiglu_bwd(sv["gu"], da, dgu)
        dh2 = dgrad_wgrad(dgu, s.w(p + "gate_up_proj"), s.g(p + "gate_up_proj"), sv["h2"].view(N, H))
        do = torch.empty(dx2.shape, dtype=dt, device=dx2.device) if lowp else None
        native.rmsnorm_bwd(sv["x2"], s.w(p + "post_attention_layernorm"), sv["rstd2"], dh2, dx2,
                           s.g(p + "post_attention_layernorm"), dx_in=g_res, dx_bf16=do)
        del g_res
        # attention output projection
        do = (do if lowp else dx2.to(dt)).view(N, H)
        dattn = dgrad_wgrad(do, s.w(p + "o_proj"), s.g(p + "o_proj"), sv["attn"].reshape(N, Hq * D))
        rm = ctx.rm
        attn = sv["attn"]
        if rm is not None:  # attention backward in the padded layout (zero gradient at the pad rows)
            dattn = rm.unpack_grad(dattn)
            attn = sv.get("attn_pad", attn)  # the fused path keeps the packed O (read through sv["o_rows"])
            B, T = rm.B, rm.T
        if isinstance(sv["P"], str):  # "flash": fused forward, fused backward
            # fused attention backward (P recomputed from the saved LSE)
            dq = torch.empty_like(sv["q"])
            dk = torch.empty_like(sv["k"])
            dv = torch.empty_like(sv["v"])
            native.flash_attn_bwd(sv["q"], sv["k"], sv["kt"], sv["v"], attn, dattn.view(B, T, Hq * D),
                                  sv["lse"], sv["key_valid"], dq, dk, dv, q_start=sv["q_start"],
                                  o_rows=sv.get("o_rows"))
        else:
            dO = dattn.view(B, T, Hkv, G, D).permute(0, 2, 3, 1, 4).reshape(B * Hkv, G * T, D)
            q3 = sv["q"].view(B * Hkv, G * T, D)
            k3 = sv["k"].view(B * Hkv, T, D)
            v3 = sv["v"].view(B * Hkv, T, D)
            P = sv["P"]
            dP = bmm_f32(dO, v3.transpose(1, 2))  # fp32 (B*Hkv, G*T, T)
            dv = torch.bmm(P.transpose(1, 2), dO)  # (B*Hkv, T, D): sums the 7 query heads of the group
            dS = torch.empty_like(P)
            native.masked_softmax_bwd(P, dP, dS, B * Hkv * G * T, T, 1.0 / math.sqrt(D))
            del dP
            dq = torch.bmm(dS, k3)
            dk = torch.bmm(dS.transpose(1, 2), q3)
        dqkv = torch.empty(B, T, (Hq + 2 * Hkv) * D, dtype=dt, device=dx2.device)
        native.rope_qkv_bwd(dq, dk, dv, ctx.pos, m.cos, m.sin, Hq, Hkv, D, dqkv)
        dqkv2 = dqkv.view(B * T, -1) if rm is None else rm.pack_grad(dqkv.view(B * T, -1))
        dh1 = dgrad_wgrad(dqkv2, s.w(p + "qkv_proj.weight"), s.g(p + "qkv_proj.weight"), sv["h1"].view(N, H))
        if m.cfg.attention_bias:
            if dqkv2.dtype == torch.bfloat16:
                native.colsum_bf16_acc(dqkv2, s.g(p + "qkv_proj.bias"))
            else:
                s.g(p + "qkv_proj.bias").add_(dqkv2.sum(0, dtype=torch.float32))
        dx = dx2  # residual: x2 = x + o
        # the previous layer's bf16 delta gets bf16(dx): written by the same pass
        ddelta = torch.empty(dx.shape, dtype=torch.bfloat16, device=dx.device) \
            if ctx.has_delta and g_mlp.dtype == torch.bfloat16 else None
        native.rmsnorm_bwd(sv["x"], s.w(p + "input_layernorm"), sv["rstd1"], dh1, dx, s.g(p + "input_layernorm"),
                           dx_bf16=ddelta)
        ctx.save = None
        if m.grad_ready_hook is not None:  # layer i's gradient is complete for this micro-batch
            m.grad_ready_hook(i)
        if ctx.has_delta and ddelta is None:
            ddelta = dx.to(g_mlp.dtype)
        return dx, ddelta, None, None, None, None, None


class _FinalNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_prev, delta, m):
        x = torch.empty_like(x_prev)
        h = torch.empty(x_prev.shape, dtype=m.dtype, device=x_prev.device)
        rstd = torch.empty(x_prev.numel() // x_prev.shape[-1], dtype=torch.float32, device=x_prev.device)
        native.add_rmsnorm_fwd(x_prev, delta, x, m.store.w("norm"), h, rstd, m.cfg.rms_norm_eps)
        ctx.save_for_backward(x, rstd)
        ctx.m = m
        ctx.delta_dtype = delta.dtype
        return h

    @staticmethod
    def backward(ctx, dh):
        x, rstd = ctx.saved_tensors
        m = ctx.m
        dx = torch.empty_like(x)
        ddelta = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) \
            if ctx.delta_dtype == torch.bfloat16 else None
        native.rmsnorm_bwd(x, m.store.w("norm"), rstd, dh.contiguous(), dx, m.store.g("norm"), dx_in=None,
                           dx_bf16=ddelta)
        return dx, (ddelta if ddelta is not None else dx.to(ctx.delta_dtype)), None


class RmPad:
    """Remove-padding index maps of one (B, T) micro-batch — the reference's unpad_input / pad_input
    (flash_attn.bert_padding, dp_actor.py:119-247, dp_critic.py:69-107 under use_remove_padding=True): ``idx``
    (nnz,) the flat positions b*T+t of the attended tokens in order, ``inv`` (B*T,) the packed row of each padded
    position (-1 at pads). Building it reads nnz back to the host once (the packed tensors' size)."""

    def __init__(self, attention_mask):
        B, T = attention_mask.shape
        dev = attention_mask.device
        self.B, self.T = B, T
        self.idx = torch.nonzero(attention_mask.reshape(-1)).reshape(-1).contiguous()
        self.nnz = int(self.idx.numel())
        self.inv = torch.full((B * T,), -1, dtype=torch.int64, device=dev)
        self.inv[self.idx] = torch.arange(self.nnz, dtype=torch.int64, device=dev)

    def pack(self, x):
        """(B*T, C) padded rows -> (nnz, C) (index_first_axis)."""
        out = torch.empty(self.nnz, x.shape[1], dtype=x.dtype, device=x.device)
        return native.copy_rows(x, out, src_idx=self.idx)

    def unpack(self, x):
        """(nnz, C) packed rows -> (B*T, C) with zero rows at the pads (pad_input): a gather through ``inv`` that
        writes the pad rows' zeros itself (no memset of the padded buffer)."""
        out = torch.empty(self.B * self.T, x.shape[1], dtype=x.dtype, device=x.device)
        return native.gather_rows_zero(x, out, self.inv)

    def tokens(self, t):
        """(B, T) per-token tensor (ids, positions) -> (1, nnz)."""
        return t.reshape(-1).index_select(0, self.idx).view(1, -1)

    # adjoints used by the layer backward: pack's is the scatter unpack, unpack's the gather pack (each padded
    # position holds at most one packed row and vice versa)
    def unpack_grad(self, x):
        return self.unpack(x)

    def pack_grad(self, x):
        return self.pack(x)


def pad_seq_columns(m, input_ids, attention_mask, position_ids, multiple=8):
    """Right-pads a micro-batch's (B, T) columns to a multiple of 8 for the bf16 model: the fused attention backward
    needs T % 8 == 0 and its forward a key-valid row stride % 4 == 0 (csrc/flash_attn.hip). The added columns are pads
    (attention_mask 0, token 0, positions continuing): no real query attends to them (masked, and causally after every
    real token), so every real position's values are unchanged and the caller slices its [T - R - 1, T - 1) rows at
    the ORIGINAL T. The reference actor takes any T (dp_actor.py:90-280). Returns (ids, mask, positions, added)."""
    T = input_ids.shape[1]
    pad = (-T) % multiple
    if pad == 0 or m.dtype != torch.bfloat16:
        return input_ids, attention_mask, position_ids, 0
    ids = F.pad(input_ids, (0, pad))
    am = F.pad(attention_mask, (0, pad))
    extra = position_ids[..., -1:] + torch.arange(1, pad + 1, device=position_ids.device, dtype=position_ids.dtype)
    return ids, am, torch.cat([position_ids, extra], -1), pad


class PrefixShare(RmPad):
    """Prefix sharing of one pass's rows: the samples of one prompt (rows with identical input ids and attention mask
    over the prompt) run the prompt's tokens once. The reference computes every sample's copy
    (dp_actor.py:119-247); each copy's hidden states are the same function of the same tokens, so the per-token
    work (embedding, norms, projections, MLP) runs on one of them and the copies only exist in the padded (B, T)
    layout the attention reads. An RmPad whose packed rows are the distinct tokens:

    * ``idx`` / ``nnz``: the packed tokens — every position except the shared copies (the group's first row, the
      leader, holds the prompt; the other rows contribute their responses), and except the pads unless
      ``keep_pads`` (the padded forward's values at pad positions, use_remove_padding False);
    * ``inv`` (B*T,): the packed row each padded position reads — a shared copy reads its leader's token;
    * shared positions are the prompt's first P - 1: the last prompt position predicts the first response token
      and stays each row's own (its gradient is then the row's own, and the predicting rows are distinct).

    unpack (packed -> padded) is the gather through ``inv``; its adjoint, pack_grad, adds the K copies' gradients
    into the shared row (drl_sum_rows, fp32 in row order: deterministic). pack and its adjoint are RmPad's."""

    @classmethod
    def build(cls, input_ids, attention_mask, R, keep_pads=False):
        """The pass's prompt groups, or None when no two rows share a prompt (P - 1 < 1 or all prompts distinct).
        Two host reads: the rows' prompt hashes and one check that every row equals its leader over the prompt."""
        B, T = attention_mask.shape
        S = T - R - 1
        if B < 2 or S < 1:
            return None
        dev = attention_mask.device
        ids, am = input_ids[:, :S], attention_mask[:, :S]
        g = torch.Generator(device="cpu").manual_seed(0x5EED)
        w = torch.randint(1, 1 << 20, (2, S), generator=g, dtype=torch.int64).to(dev)
        key = torch.stack([(ids.to(torch.int64) * w[0]).sum(-1), (am.to(torch.int64) * w[1]).sum(-1)], 1).cpu()
        groups = {}
        for b, k in enumerate(map(tuple, key.tolist())):
            groups.setdefault(k, []).append(b)
        members = list(groups.values())
        if max(len(mm) for mm in members) < 2:
            return None
        leader = torch.empty(B, dtype=torch.int64)
        for mm in members:
            leader[mm] = mm[0]
        leader = leader.to(dev)
        if not bool(((ids == ids[leader]) & (am == am[leader])).all()):  # a hash collision: no sharing
            return None
        return cls(attention_mask, S, leader, members, keep_pads)

    def __init__(self, attention_mask, S, leader, members, keep_pads):
        B, T = attention_mask.shape
        dev = attention_mask.device
        self.B, self.T, self.S = B, T, S
        rows = torch.arange(B, device=dev)
        copy = (leader != rows)[:, None] & (torch.arange(T, device=dev) < S)[None, :]
        own = ~copy if keep_pads else (attention_mask.bool() & ~copy)
        self.idx = torch.nonzero(own.reshape(-1)).reshape(-1).contiguous()
        self.nnz = int(self.idx.numel())
        inv_own = torch.full((B * T,), -1, dtype=torch.int64, device=dev)
        inv_own[self.idx] = torch.arange(self.nnz, dtype=torch.int64, device=dev)
        self.inv_own = inv_own  # each packed row at its own padded position only (unpack_grad)
        inv_own = inv_own.view(B, T)
        self.inv = torch.where(copy, inv_own[leader], inv_own).reshape(-1).contiguous()
        self.groups = len(members)
        # the fused attention skips the copies' query tiles (their outputs are never packed, their gradient is 0)
        self.q_start = torch.where(leader != rows, S, 0).to(torch.int32).contiguous()
        # pack_grad: the shared packed rows (leader positions t < S that are packed tokens) and, per group member
        # slot k, the padded position of member k's copy (-1 past the group's size)
        shared = [mm for mm in members if len(mm) > 1]
        K = max(len(mm) for mm in shared)
        mem = torch.full((len(shared), K), -1, dtype=torch.int64)
        for gi, mm in enumerate(shared):
            mem[gi, :len(mm)] = torch.tensor(mm)
        mem = mem.to(dev)
        gi, t = torch.nonzero(own[mem[:, 0], :S], as_tuple=True)
        self.sum_dst = inv_own[mem[gi, 0], t].contiguous()
        m = mem[gi].t()  # (K, m)
        self.sum_src = torch.where(m >= 0, m * T + t[None, :], torch.full_like(m, -1)).contiguous()

    def unpack(self, x):
        """(nnz, C) packed -> (B*T, C): every padded position reads its packed row (shared copies their leader's),
        zero rows at the pads that hold no packed row."""
        out = torch.empty(self.B * self.T, x.shape[1], dtype=x.dtype, device=x.device)
        return native.gather_rows_zero(x, out, self.inv)

    def unpack_grad(self, x):
        """RmPad's unpack (the adjoint of pack): each packed row to its own padded position, zeros elsewhere —
        including the shared copies' positions."""
        out = torch.empty(self.B * self.T, x.shape[1], dtype=x.dtype, device=x.device)
        return native.gather_rows_zero(x, out, self.inv_own)

    def pack_grad(self, x):
        """Adjoint of unpack: each packed row gets the sum of the gradients of the padded positions that read it."""
        out = self.pack(x)
        if self.sum_dst.numel():
            native.sum_rows(x, self.sum_src, out, self.sum_dst)
        return out


class _GatherRows(torch.autograd.Function):
    """out[j] = x[idx[j]] for x (n, C) and idx (m,) with -1 -> a zero row; every source row is selected at most once,
    so the backward is the inverse scatter (no accumulation)."""

    @staticmethod
    def forward(ctx, x, idx):
        ctx.idx, ctx.n = idx, x.shape[0]
        out = torch.empty(idx.shape[0], x.shape[1], dtype=x.dtype, device=x.device)
        return native.gather_rows_zero(x.contiguous(), out, idx)

    @staticmethod
    def backward(ctx, dy):
        dx = torch.zeros(ctx.n, dy.shape[1], dtype=dy.dtype, device=dy.device)
        return native.copy_rows(dy.contiguous(), dx, dst_idx=ctx.idx), None


def gather_rows(x, idx):
    return _GatherRows.apply(x, idx)


def _key_valid(attention_mask):
    """u8 key-valid rows padded to a multiple of 4 bytes (the fused attention reads them as 32-bit words)."""
    B, T = attention_mask.shape
    buf = torch.zeros(B, (T + 3) // 4 * 4, dtype=torch.uint8, device=attention_mask.device)
    buf[:, :T] = attention_mask
    return buf[:, :T]


class KVCacheRows:
    """Rows [r0, r1) of a KVCache as a KVCache-shaped view (dim-0 slices: contiguous, the same strides), for one
    row lane of the graphed decode step."""

    def __init__(self, cache, r0, r1):
        self.k = [t[r0:r1] for t in cache.k]
        self.vt = [None if t is None else t[r0:r1] for t in cache.vt]
        self.v = [None if t is None else t[r0:r1] for t in cache.v]
        self.valid = cache.valid[r0:r1]
        self.len = cache.len
        self.Tmax = cache.Tmax
        self.group, self.shared = 1, 0


class KVCache:
    """Per-layer K (B, Hkv, Tmax, D) and V (bf16: head-dim-major in 32-key blocks (B, Hkv, ceil(Tmax / 32), D, 32);
    fp32: row-major) in the compute dtype, plus the key-valid mask (u8)."""

    def __init__(self, cfg: Qwen2Config, B, Tmax, device, dtype):
        Hkv, D, L = cfg.num_key_value_heads, cfg.head_dim, cfg.num_hidden_layers
        self.k = [torch.empty(B, Hkv, Tmax, D, device=device, dtype=dtype) for _ in range(L)]
        if dtype == torch.bfloat16 and D in (64, 128):
            # V^T key-blocked (native.DRL_VT_BLOCKED): a 32-key block of V^T is one contiguous 32 * D run, the unit
            # the MFMA prefill and decode kernels fetch (the K block is one contiguous run already)
            self.vt = [torch.zeros(B, Hkv, (Tmax + 31) // 32, D, 32, device=device, dtype=dtype) for _ in range(L)]
            self.v = [None] * L
        else:
            self.vt = [None] * L
            self.v = [torch.empty_like(t) for t in self.k]
        self.valid = torch.zeros(B, (Tmax + 3) // 4 * 4, dtype=torch.uint8, device=device)[:, :Tmax]
        self.len = 0
        self.Tmax = Tmax
        # prompt groups (share_prompts): row p * group + r reads keys < shared from row p
        self.group, self.shared = 1, 0

    def share_prompts(self, group, P):
        """After rows [0, B / group) were prefilled with the distinct prompts (keys [0, P)): rows p * group + r (the
        group's samples of prompt p) read the whole 32-key blocks below P from row p in the MFMA decode attention
        (drl_decode_attention_vt prompt groups); every row gets its own copy of the rest — the keys of the block
        holding P - 1 when P % 32 != 0, all of them for the fp32 cache (row-major V, no grouped kernel) — and of
        the prompt's key-valid bytes."""
        B = self.valid.shape[0]
        src = torch.arange(B, device=self.valid.device) // group
        shared = P // 32 * 32 if self.vt[0] is not None else 0
        for i in range(len(self.k)):
            if shared < P:
                self.k[i][:, :, shared:P] = self.k[i][src, :, shared:P]
                if self.vt[i] is not None:
                    b0, b1 = shared // 32, (P + 31) // 32
                    self.vt[i][:, :, b0:b1] = self.vt[i][src, :, b0:b1]
                else:
                    self.v[i][:, :, :P] = self.v[i][src, :, :P]
        self.valid[:, :P] = self.valid[src, :P]
        self.len = P
        self.group, self.shared = (group, shared) if shared > 0 else (1, 0)

    def vt_plain(self, i):
        """Layer i's V^T as a head-dim-major (B, Hkv, D, Tmax) copy (tests / inspection)."""
        from . import native
        return native.vt_blocked_to_plain(self.vt[i])[..., :self.Tmax]


class Qwen2Model:
    """Functional Qwen2 over a ParamStore (no nn.Module: the parameters are views into flat buffers)."""

    def __init__(self, cfg: Qwen2Config, store: ParamStore):
        self.cfg = cfg
        self.store = store
        self.dtype = store.compute_dtype
        self.training = False
        dev = store.device
        half = cfg.head_dim // 2
        inv_freq = 1.0 / (cfg.rope_theta ** (torch.arange(0, cfg.head_dim, 2, dtype=torch.int64, device=dev).float()
                                             / cfg.head_dim))
        t = torch.arange(cfg.max_position_embeddings, device=dev, dtype=torch.float32)
        freqs = t[:, None] * inv_freq[None, :half]
        self.cos = freqs.cos().contiguous()
        self.sin = freqs.sin().contiguous()
        self._dummy = torch.empty(0, device=dev, requires_grad=True)
        # called with layer index i at the end of layer i's backward (FlatAdamW's overlapped all-reduce)
        self.grad_ready_hook = None
        if cfg.rope_scaling:
            raise NotImplementedError(f"rope_scaling {cfg.rope_scaling} (plain RoPE only: Qwen2 / Llama-3-8B)")
        self._zero_bias = None
        if not cfg.attention_bias:  # Llama: the shared qkv epilogues add a constant zero bias
            nq = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * cfg.head_dim
            self._zero_bias = torch.zeros(nq, dtype=self.dtype, device=dev)

    def qkv_bias(self, i):
        return self.store.w(f"layers.{i}.qkv_proj.bias") if self.cfg.attention_bias else self._zero_bias

    def _gw(self, name):
        return self.store.g(name) if (self.training and self.store.trainable) else None

    def lm_head_weight(self):
        return "embed_tokens" if self.cfg.tie_word_embeddings else "lm_head"

    def logits(self, h):
        """h (N, H) in the compute dtype -> (N, V) logits in the compute dtype."""
        name = self.lm_head_weight()
        if self.training and self.store.trainable:
            return _Linear.apply(h, self.store.w(name), self.store.g(name), self._dummy)
        return linear(h.reshape(-1, h.shape[-1]), self.store.w(name)).view(*h.shape[:-1], -1)

    def select_tokens(self, h, out_tokens, fused=True, logprob_out=None, logprob_temperature=1.0, logits_fn=None,
                      **sel):
        """Token selection from the final-norm hidden h (N, H): K4 fused with the lm_head on bf16 (the (N, V)
        logits are never written, csrc/fused_linear.hip), else lm_head logits + K4 (fp32 parity model, and
        sampling: the slice race and the top-k / top-p cut read the logits row). With ``logprob_out`` (the
        rollout's calculate_log_probs) the selected token's log p under logits / ``logprob_temperature`` is written
        to the same column of it (native.token_logprob, one more pass over the logits rows). ``logits_fn``: the
        decode step's own lm_head (PackedDecode.logits) in place of self.logits."""
        w = self.store.w(self.lm_head_weight())
        if logprob_out is None and fused and not sel.get("do_sample") and self.dtype == torch.bfloat16 and \
                h.shape[-1] % 64 == 0 and logits_fn is None:
            return native.linear_select_tokens(h.contiguous(), w, out_tokens, **sel)
        logits = logits_fn(h) if logits_fn is not None else self.logits(h)
        native.select_tokens(logits, out_tokens, **sel)
        if logprob_out is not None:
            native.token_logprob(logits, out_tokens, logprob_out, logprob_temperature, dev_step=sel.get("dev_step"))
        return out_tokens

    def fused_logprob(self, h, labels, temperature, calculate_entropy):
        """A21: h (N, H) in bf16 -> (log_probs, entropy or None) over the lm_head without materialising logits
        (csrc/fused_linear.hip); in training the weight gradient accumulates into the fp32 gradient buffer."""
        name = self.lm_head_weight()
        gw = self.store.g(name) if (self.training and self.store.trainable) else None
        return fused_linear_logprob_entropy(h, self.store.w(name), labels, temperature, calculate_entropy,
                                            weight_grad=gw)

    def hidden_states(self, input_ids, attention_mask, position_ids, rm=None):
        """Full-sequence forward -> final-norm hidden states (B, T, H) in the compute dtype; with ``rm`` (RmPad of
        attention_mask) only the attended tokens run through the norms / GEMMs / MLP and the result is the packed
        (1, nnz, H) (the reference's use_remove_padding forward)."""
        cfg = self.cfg
        key_valid = _key_valid(attention_mask)
        pos = position_ids.contiguous()
        ids = input_ids if rm is None else rm.tokens(input_ids)
        if self.training and self.store.trainable:
            x = _Embedding.apply(ids, self.store.w("embed_tokens"), self.store.g("embed_tokens"), self._dummy)
            delta = None
            for i in range(cfg.num_hidden_layers):
                x, delta = _DecoderLayer.apply(x, delta, self, i, pos, key_valid, rm)
            return _FinalNorm.apply(x, delta, self)
        with torch.no_grad():
            x = F.embedding(ids, self.store.w("embed_tokens")).to(torch.float32)
            delta = None
            for i in range(cfg.num_hidden_layers):
                x, delta = _layer_forward(self, i, x, delta, pos, key_valid, None, rm=rm)
            return self._final_norm(x, delta)

    def _final_norm(self, x, delta):
        h = torch.empty(x.shape, dtype=self.dtype, device=x.device)
        native.add_rmsnorm_fwd(x, delta, None, self.store.w("norm"), h, None, self.cfg.rms_norm_eps)
        return h

    # ----------------------------------------------------------------------------------- decode
    @torch.no_grad()
    def prefill(self, cache: KVCache, input_ids, attention_mask, position_ids):
        """Prompt pass writing the KV cache; returns the last position's hidden state (B, H)."""
        cfg = self.cfg
        B, T = input_ids.shape
        cache.valid[:, :T] = attention_mask.to(torch.uint8)
        pos = position_ids.contiguous()
        x = F.embedding(input_ids, self.store.w("embed_tokens")).to(torch.float32)
        delta = None
        for i in range(cfg.num_hidden_layers):
            x, delta = _layer_forward(self, i, x, delta, pos, cache.valid, None, cache, 0)
        cache.len = T
        return self._final_norm(x[:, -1:].contiguous(), delta[:, -1:].contiguous())[:, 0]

    @torch.no_grad()
    def decode_step(self, cache: KVCache, tokens, positions):
        """One token per sequence at cache position cache.len; returns (B, H) hidden."""
        cfg = self.cfg
        t = cache.len
        x = F.embedding(tokens[:, None], self.store.w("embed_tokens")).to(torch.float32)
        cache.valid[:, t] = 1
        pos = positions[:, None].contiguous()
        delta = None
        for i in range(cfg.num_hidden_layers):
            x, delta = _layer_forward(self, i, x, delta, pos, cache.valid, None, cache, t)
        cache.len = t + 1
        return self._final_norm(x, delta)[:, 0]

    @torch.no_grad()
    def decode_step_dev(self, cache: KVCache, tokens, positions, kpos_dev):
        """decode_step with the cache position in device memory (int64 (1,)): every shape and address is
        static, so the step can be captured once into a HIP graph and replayed for each response token."""
        x = F.embedding(tokens.view(-1, 1), self.store.w("embed_tokens")).to(torch.float32)
        cache.valid.index_fill_(1, kpos_dev, 1)
        pos = positions.view(-1, 1)
        delta = None
        for i in range(self.cfg.num_hidden_layers):
            x, delta = _layer_forward(self, i, x, delta, pos, cache.valid, None, cache, 0, koff_dev=kpos_dev)
        return self._final_norm(x, delta)[:, 0]


class PackedDecode:
    """Decode step on fragment-packed operands (csrc/decode_gemm.hip) for one rollout of B <= 512 sequences:
    per layer decode RMSNorm (packed out) -> qkv GEMM with bias + RoPE + cache writes in its epilogue (weights
    packed in rotation pairs) -> MFMA decode attention (packed out) -> o_proj GEMM (fp32 K-slice partials) ->
    decode RMSNorm (adds the o_proj partials) -> gate_up GEMM with the SwiGLU epilogue (packed out) ->
    down_proj GEMM, whose partials the next layer's RMSNorm adds. Seven launches per layer instead of nine,
    every projection a one-round-trip weight stream. The weights are packed once per rollout from the bf16
    compute copy (they change at every optimizer step); every buffer is preallocated so the step is
    graph-capturable. Module math is the unpacked decode path's (bf16 module outputs, fp32 residual)."""

    @staticmethod
    def supported(model, B, max_rows=512):
        cfg = model.cfg
        H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        NQ = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * D
        # 1..512 rows (rollout at B=64: 0.66 -> 0.38 s; at B=512 1.20 -> 1.18 s, tools/kernel_bench.py
        # --only decode_gemm for the per-projection times)
        return (B <= max_rows and model.dtype == torch.bfloat16 and D in (64, 128) and H % 64 == 0 and I % 64 == 0
                and (cfg.num_attention_heads * D) % 64 == 0 and I % 16 == 0
                and all(native.decode_gemm_plan(B, n, k, sw) is not None
                        for n, k, sw in ((NQ, H, False), (H, cfg.num_attention_heads * D, False), (2 * I, H, True),
                                         (H, I, False))))

    def __init__(self, model, B, weights=None, fused_norm=False, lm_head=True):
        """``weights``: another PackedDecode's packed weights (the layout does not depend on B), shared by the
        row lanes of one rollout instead of packed again. ``fused_norm``: the five-launch layer (the RMSNorms in the
        consumer GEMMs' prologue, the residual adds in the o_proj / down_proj epilogues) where the fused kernels take
        the shape (1..128 rows at Qwen2.5-0.5B width); otherwise the seven-launch layer. Off by default: measured
        slower (64 rows: 47.7 against 41.7 us per layer graph-replayed, profiles/r06_decode_fused_norm_sweep_rejected
        .jsonl) — the gate_up consumer's workgroups each re-read the fp32 residual panel (twice the bytes of the packed
        bf16 norm output they read otherwise), and the K-split down_proj's last-arriver combine costs more than the
        norm launch it replaces."""
        cfg, s, dev = model.cfg, model.store, model.store.device
        self.model = model
        self.B = B
        H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        Hq, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads
        self.NQ = (Hq + 2 * Hkv) * D
        self.HD = Hq * D
        self.plans = {"o": native.decode_gemm_plan(B, H, self.HD),
                      "gu": native.decode_gemm_plan(B, 2 * I, H, True), "d": native.decode_gemm_plan(B, H, I)}
        self.mbt = self.plans["o"][1]
        assert all(p[1] == self.mbt for p in self.plans.values())
        fplans = None
        if fused_norm:
            fplans = {"o": native.decode_norm_plan(B, H, self.HD, native.DECODE_RESID),
                      "d": native.decode_norm_plan(B, H, I, native.DECODE_RESID),
                      "gu": native.decode_norm_plan(B, 2 * I, H, native.DECODE_SWIGLU),
                      "qkv": native.decode_norm_plan(B, self.NQ, H, native.DECODE_ROPE)}
            if any(v is None or v[1] != self.mbt for v in fplans.values()):
                fplans = None
        self.fused = fplans is not None
        self.fplans = fplans
        bf = torch.bfloat16
        self.w = weights if weights is not None else []
        for i in range(0 if weights is not None else cfg.num_hidden_layers):
            p = f"layers.{i}."
            self.w.append(dict(qkv=native.decode_pack_weight_rope(s.w(p + "qkv_proj.weight"), D),
                               o=native.decode_pack_weight(s.w(p + "o_proj")),
                               gu=native.decode_pack_weight(s.w(p + "gate_up_proj"), swiglu=True),
                               d=native.decode_pack_weight(s.w(p + "down_proj"))))
        rows = self.mbt * 32
        self.h_p = torch.zeros(rows * H, dtype=bf, device=dev)        # RMSNorm out (packed; pad rows stay 0)
        self.attn_p = torch.zeros(rows * self.HD, dtype=bf, device=dev)
        self.a_p = torch.zeros(rows * I, dtype=bf, device=dev)        # SwiGLU out
        if self.fused:
            # the packed fp32 residual stream (pad rows stay 0), K-slice scratch and arrival counters (left zeroed by
            # every launch; the two producers run one after the other on the stream, so they share them)
            self.xr = torch.zeros(rows * H, device=dev)
            self.part_o = torch.empty(max(1, self.fplans["o"][0]), B, H, device=dev)
            self.part_d = torch.empty(max(1, self.fplans["d"][0]), B, H, device=dev)
            nb = max(native.lib().drl_decode_resid_counter_bytes(B, H, self.HD),
                     native.lib().drl_decode_resid_counter_bytes(B, H, I))
            self.cnt = torch.zeros((nb + 3) // 4, dtype=torch.int32, device=dev)
            self.x = None
        else:
            self.part_o = torch.empty(self.plans["o"][0], B, H, device=dev)
            self.part_d = torch.empty(self.plans["d"][0], B, H, device=dev)
            self.x = torch.empty(B, H, device=dev)                         # fp32 residual stream
        self.q = torch.empty(B, Hkv, Hq // Hkv, D, dtype=bf, device=dev)
        self.h_out = torch.empty(B, H, dtype=bf, device=dev)
        # the decode lm_head at <= 64 rows (csrc/decode_gemm.hip decode_lm_head_kernel: the packed h panel in LDS, the
        # packed weight streamed once per token); the final norm also writes h packed for it
        V = cfg.vocab_size
        self.lm_mbt = native.decode_lm_head_plan(B, V, H) if lm_head else None
        self.lm_w = None
        if self.lm_mbt is not None:
            self.lm_w = native.decode_pack_weight(s.w(model.lm_head_weight()))
            self.h_pk = torch.zeros(self.lm_mbt * 32 * H, dtype=bf, device=dev)
            self.logits_buf = torch.empty(B, V, dtype=bf, device=dev)
        self.pos = torch.empty(B, dtype=torch.int64, device=dev)   # step_from: rotary positions of the new token
        self.kpos = torch.empty(1, dtype=torch.int64, device=dev)  # step_from: its cache slot
        self.t_cur = torch.empty(1, dtype=torch.int64, device=dev)  # step_from: the step's t (Philox offset / column)

    @torch.no_grad()
    def step_from(self, cache, responses, t_dev, last_pos, P):
        """One graphed decode step driven by the device counter t_dev: the previous token of every row is
        responses[:, t - 1]; one prologue launch embeds it, sets positions / the cache slot / key_valid, publishes
        t (self.t_cur, the selection's step) and advances t_dev. Returns the final-norm hidden (B, H)."""
        if self.fused:
            native.decode_step_prologue(responses, t_dev, self.t_cur, last_pos.reshape(-1).contiguous(), P,
                                        self.model.store.w("embed_tokens"), self.xr, self.pos, self.kpos, cache.valid,
                                        x_mbt=self.mbt)
        else:
            native.decode_step_prologue(responses, t_dev, self.t_cur, last_pos.reshape(-1).contiguous(), P,
                                        self.model.store.w("embed_tokens"), self.x, self.pos, self.kpos, cache.valid)
        return self._layers(cache, self.pos, self.kpos)

    @torch.no_grad()
    def step(self, cache, tokens, positions, kpos_dev):
        """One token per sequence at device cache position kpos_dev; returns the final-norm hidden (B, H)."""
        s = self.model.store
        x = F.embedding(tokens.view(-1), s.w("embed_tokens")).to(torch.float32)
        if self.fused:
            native.pack_residual(x, self.mbt, out=self.xr)
        else:
            self.x.copy_(x)
        cache.valid.index_fill_(1, kpos_dev, 1)
        return self._layers(cache, positions.view(-1), kpos_dev)

    def _layers(self, cache, pos, kpos_dev):
        m = self.model
        cfg, s = m.cfg, m.store
        B, H, I = self.B, cfg.hidden_size, cfg.intermediate_size
        Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        eps, mbt = cfg.rms_norm_eps, self.mbt
        Lk = cache.k[0].shape[2]
        if self.fused:
            # five launches per layer: the RMSNorms run in the consumers' prologues (qkv + RoPE, gate_up + SwiGLU),
            # the residual adds in the producers' epilogues (o_proj, down_proj) on the packed fp32 residual xr
            for i in range(cfg.num_hidden_layers):
                p, w = f"layers.{i}.", self.w[i]
                native.decode_qkv_rope_norm(self.xr, s.w(p + "input_layernorm"), eps, w["qkv"], m.qkv_bias(i), pos,
                                            m.cos, m.sin, B, H, Hq, Hkv, D, self.q, cache.k[i], cache.vt[i], kpos_dev)
                native.decode_attention_vt(self.q, cache.k[i], cache.vt[i], cache.valid, Lk, self.attn_p,
                                           qpos_dev=kpos_dev, out_mbt=mbt, group=cache.group, shared_keys=cache.shared)
                native.decode_gemm_resid(self.attn_p, w["o"], B, H, self.HD, self.xr, mbt, self.part_o, self.cnt)
                native.decode_gemm_norm(self.xr, s.w(p + "post_attention_layernorm"), eps, w["gu"], B, 2 * I, H,
                                        self.a_p)
                native.decode_gemm_resid(self.a_p, w["d"], B, H, I, self.xr, mbt, self.part_d, self.cnt)
            native.decode_final_norm(self.xr, mbt, s.w("norm"), self.h_out, B, H, eps,
                                     y_packed=self.h_pk if self.lm_w is not None else None,
                                     packed_mbt=self.lm_mbt or 0)
            return self.h_out
        prev = None
        for i in range(cfg.num_hidden_layers):
            p, w = f"layers.{i}.", self.w[i]
            native.decode_rmsnorm(self.x, prev, self.x, s.w(p + "input_layernorm"), self.h_p, eps, mbt=mbt)
            native.decode_qkv_rope(self.h_p, w["qkv"], m.qkv_bias(i), pos, m.cos, m.sin, B, H, Hq, Hkv, D,
                                   self.q, cache.k[i], cache.vt[i], kpos_dev)
            native.decode_attention_vt(self.q, cache.k[i], cache.vt[i], cache.valid, Lk, self.attn_p,
                                       qpos_dev=kpos_dev, out_mbt=mbt, group=cache.group, shared_keys=cache.shared)
            native.decode_gemm(self.attn_p, w["o"], B, H, self.HD, partials=self.part_o)
            native.decode_rmsnorm(self.x, self.part_o, self.x, s.w(p + "post_attention_layernorm"), self.h_p, eps,
                                  mbt=mbt)
            native.decode_gemm(self.h_p, w["gu"], B, 2 * I, H, swiglu=True, out_packed=self.a_p)
            native.decode_gemm(self.a_p, w["d"], B, H, I, partials=self.part_d)
            prev = self.part_d
        native.decode_rmsnorm(self.x, prev, None, s.w("norm"), self.h_out, eps, mbt=0,
                              y_packed=self.h_pk if self.lm_w is not None else None, packed_mbt=self.lm_mbt or 0)
        return self.h_out

    def logits(self, h):
        """lm_head logits (B, V) bf16 of this step's final-norm output (h is self.h_out): the decode lm_head kernel
        at <= 64 rows, the model's drl_gemm lm_head otherwise."""
        if self.lm_w is not None and h is self.h_out:
            cfg = self.model.cfg
            return native.decode_lm_head(self.h_pk, self.lm_mbt, self.lm_w, self.B, cfg.vocab_size, cfg.hidden_size,
                                         self.logits_buf)
        return self.model.logits(h)


def flops_per_token(cfg: Qwen2Config, seqlen: int) -> float:
    """flops_counter.py:135-167 convention: 2 * N_dense per token forward (embedding + lm_head counted)
    plus attention 2 * 2 * s * d * h * L."""
    H, I, L, V = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers, cfg.vocab_size
    hd = cfg.head_dim
    q, kv = cfg.num_attention_heads * hd, cfg.num_key_value_heads * hd
    dense = L * (H * (q + 2 * kv) + q * H + 3 * H * I) + 2 * V * H
    return 2 * dense + 4 * seqlen * hd * cfg.num_attention_heads * L
