"""Key-blocked V^T cache layout (include/dotsrl_amd.h DRL_VT_BLOCKED; KVCache's layout): every producer and
consumer gives bit-identical results on the blocked tensor and on the head-dim-major (B, Hkv, D, ld) one, which
the rest of the suite pins to the references:

* writers: drl_rope_qkv_fwd (element-wise form below 16 positions, tiled form above, any key offset),
  drl_decode_rope and drl_decode_qkv_rope (device key offset);
* readers: the prefill flash attention (query offset into a cache) and the MFMA decode attention (host and
  device query position, ragged key-valid, split plans).
"""

import pytest
import torch

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def blocked(vt_plain, cap):
    """(B, Hkv, D, >= cap) head-dim-major -> (B, Hkv, ceil(cap / 32), D, 32) key-blocked (zero past cap)."""
    B, Hkv, D = vt_plain.shape[:3]
    nb = (cap + 31) // 32
    out = torch.zeros(B, Hkv, D, nb * 32, dtype=vt_plain.dtype, device=vt_plain.device)
    out[..., :cap] = vt_plain[..., :cap]
    return out.view(B, Hkv, D, nb, 32).permute(0, 1, 3, 2, 4).contiguous()


def rope_tables(D, n=2048):
    half = D // 2
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    fr = torch.arange(n, device=DEV).float()[:, None] * inv[None, :half]
    return fr.cos().contiguous(), fr.sin().contiguous()


def test_blocked_round_trip():
    x = torch.randn(2, 3, 64, 70, device=DEV).to(BF)
    assert torch.equal(native.vt_blocked_to_plain(blocked(x, 70))[..., :70], x)


@pytest.mark.parametrize("T,koff,cap", [(8, 5, 40), (1, 37, 64), (100, 0, 100), (48, 17, 96), (64, 32, 130)])
def test_rope_writes_blocked(T, koff, cap):
    B, Hq, Hkv, D = 3, 14, 2, 64
    G = Hq // Hkv
    g = torch.Generator(device=DEV).manual_seed(T + koff)
    qkv = torch.randn(B, T, (Hq + 2 * Hkv) * D, device=DEV, generator=g).to(BF)
    pos = torch.arange(T, device=DEV).repeat(B, 1) + koff
    cos_t, sin_t = rope_tables(D)
    outs = []
    for blk in (False, True):
        q = torch.empty(B, Hkv, G, T, D, dtype=BF, device=DEV)
        k = torch.zeros(B, Hkv, cap, D, dtype=BF, device=DEV)
        ld = (cap + 7) // 8 * 8
        vt = torch.zeros(B, Hkv, (cap + 31) // 32, D, 32, dtype=BF, device=DEV) if blk else \
            torch.zeros(B, Hkv, D, ld, dtype=BF, device=DEV)
        native.rope_qkv_fwd(qkv, pos, cos_t, sin_t, Hq, Hkv, D, q, k, None, koff=koff, vt=vt)
        outs.append((q, k, native.vt_blocked_to_plain(vt)[..., :cap] if blk else vt[..., :cap]))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_decode_rope_writes_blocked():
    B, Hq, Hkv, D, Tk, koff = 64, 14, 2, 64, 72, 45
    G = Hq // Hkv
    NQ = (Hq + 2 * Hkv) * D
    part = torch.randn(2, B, NQ, device=DEV)
    bias = torch.randn(NQ, device=DEV).to(BF)
    pos = torch.randint(0, 1000, (B,), device=DEV)
    cos_t, sin_t = rope_tables(D)
    kd = torch.tensor([koff], device=DEV)
    outs = []
    for blk in (False, True):
        q = torch.empty(B, Hkv, G, D, dtype=BF, device=DEV)
        k = torch.zeros(B, Hkv, Tk, D, dtype=BF, device=DEV)
        vt = torch.zeros(B, Hkv, (Tk + 31) // 32, D, 32, dtype=BF, device=DEV) if blk else \
            torch.zeros(B, Hkv, D, Tk, dtype=BF, device=DEV)
        native.decode_rope(part, bias, pos, cos_t, sin_t, Hq, Hkv, D, q, k, vt_cache=vt, koff_dev=kd)
        outs.append((q, k, native.vt_blocked_to_plain(vt)[..., :Tk] if blk else vt))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,K,Hq,Hkv,D", [(64, 896, 14, 2, 64), (100, 256, 4, 2, 128)])
def test_decode_qkv_rope_writes_blocked(M, K, Hq, Hkv, D):
    NQ = (Hq + 2 * Hkv) * D
    G, Tk, koff = Hq // Hkv, 64, 41
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, K, device=DEV, generator=g).to(BF)
    w = (torch.randn(NQ, K, device=DEV, generator=g) * 0.05).to(BF)
    bias = torch.randn(NQ, device=DEV, generator=g).to(BF)
    pos = torch.randint(0, 500, (M,), device=DEV)
    cos_t, sin_t = rope_tables(D, 1024)
    kd = torch.tensor([koff], device=DEV)
    xp = native.pack_activations(x, native.decode_gemm_plan(M, NQ, K)[1])
    wp = native.decode_pack_weight_rope(w, D)
    outs = []
    for blk in (False, True):
        q = torch.zeros(M, Hkv, G, D, dtype=BF, device=DEV)
        kc = torch.zeros(M, Hkv, Tk, D, dtype=BF, device=DEV)
        vt = torch.zeros(M, Hkv, Tk // 32, D, 32, dtype=BF, device=DEV) if blk else \
            torch.zeros(M, Hkv, D, Tk, dtype=BF, device=DEV)
        native.decode_qkv_rope(xp, wp, bias, pos, cos_t, sin_t, M, K, Hq, Hkv, D, q, kc, vt, kd)
        outs.append((q, kc, native.vt_blocked_to_plain(vt) if blk else vt))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,Hkv,G,D,Tq,cap,qoff", [(2, 2, 7, 64, 96, 160, 40), (3, 2, 7, 64, 33, 100, 0),
                                                    (1, 2, 4, 128, 64, 200, 77)])
def test_flash_prefill_reads_blocked(B, Hkv, G, D, Tq, cap, qoff):
    Tk = Tq + qoff
    g = torch.Generator(device=DEV).manual_seed(Tq + cap)
    q = torch.randn(B, Hkv, G, Tq, D, device=DEV, generator=g).to(BF)
    k = torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF)
    v = torch.randn(B, Hkv, D, cap, device=DEV, generator=g).to(BF)
    valid = torch.zeros(B, (cap + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    valid[:, :Tk] = 1
    for b in range(B):
        valid[b, : 5 * b] = 0
    ld = (cap + 7) // 8 * 8
    vt = torch.zeros(B, Hkv, D, ld, dtype=BF, device=DEV)
    vt[..., :cap] = v
    outs = []
    for t in (vt, blocked(vt, cap)):
        o = torch.empty(B, Tq, Hkv * G * D, dtype=BF, device=DEV)
        lse = torch.empty(B, Hkv, G, Tq, device=DEV)
        native.flash_attn_fwd(q, k, t, valid[:, :cap], o, Tk=Tk, qoff=qoff, lse=lse)
        outs.append((o, lse))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("B,Hkv,G,D,cap,L", [(64, 2, 7, 64, 768, 700), (512, 2, 7, 64, 768, 640),
                                              (5, 2, 4, 128, 300, 257), (9, 1, 8, 64, 4096, 4000)])
def test_decode_attention_reads_blocked(B, Hkv, G, D, cap, L):
    g = torch.Generator(device=DEV).manual_seed(L)
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
    k = torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF)
    vt = torch.randn(B, Hkv, D, (cap + 7) // 8 * 8, device=DEV, generator=g).to(BF)
    valid = torch.zeros(B, (cap + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    valid[:, :L] = 1
    for b in range(B):
        valid[b, : min(3 * b, L - 1)] = 0
    vb = blocked(vt, cap)
    qp = torch.tensor([L - 3], device=DEV)
    for kw in ({}, {"qpos_dev": qp}):
        a = native.decode_attention_vt(q, k, vt, valid[:, :cap], L, torch.empty_like(q), **kw)
        b = native.decode_attention_vt(q, k, vb, valid[:, :cap], L, torch.empty_like(q), **kw)
        assert torch.equal(a, b)
