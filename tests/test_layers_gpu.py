"""Transformer-layer HIP kernels (csrc/layers.hip, csrc/attention.hip) against plain PyTorch fp32 references.

The model-level tests (test_model_gpu.py) check these kernels composed into Qwen2 against HF; this file
pins each kernel on its own, including ragged masks (left padding, masked-out rows) and sizes that cross
the kernels' chunk boundaries. fp32 runs must agree to ~1e-5 relative; bf16 runs to bf16 rounding.
"""

import math

import pytest
import torch
import torch.nn.functional as F

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tol(dt):
    return dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)


def _rope_tables(D, maxpos=4096, theta=1e4):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, device=DEV).float() / D))
    f = torch.arange(maxpos, device=DEV).float()[:, None] * inv[None]
    return f.cos().contiguous(), f.sin().contiguous()


def _rot(x, c, s):  # HF rotate_half RoPE; x (..., D), c/s (..., D/2)
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_rope_qkv_forward_backward(dt):
    B, T, Hq, Hkv, D, Tk, koff = 3, 37, 14, 2, 64, 50, 9
    G = Hq // Hkv
    g = torch.Generator(device=DEV).manual_seed(0)
    qkv = torch.randn(B, T, (Hq + 2 * Hkv) * D, device=DEV, generator=g).to(dt)
    pos = torch.randint(0, 4000, (B, T), device=DEV, generator=g)
    cos, sin = _rope_tables(D)
    q = torch.empty(B, Hkv, G, T, D, device=DEV, dtype=dt)
    k = torch.zeros(B, Hkv, Tk, D, device=DEV, dtype=dt)
    v = torch.zeros_like(k)
    native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q, k, v, koff)
    if dt == torch.float32:  # device-side key offset (graph-captured decode) writes the same slots
        k2 = torch.zeros_like(k)
        v2 = torch.zeros_like(v)
        native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, torch.empty_like(q), k2, v2, 0, torch.tensor([koff], device=DEV))
        assert torch.equal(k2, k) and torch.equal(v2, v)
    x = qkv.float().view(B, T, Hq + 2 * Hkv, D)
    c, s = cos[pos][:, :, None], sin[pos][:, :, None]
    rq = _rot(x[:, :, :Hq], c, s)  # (B,T,Hq,D)
    rk = _rot(x[:, :, Hq:Hq + Hkv], c, s)
    torch.testing.assert_close(q.float(), rq.view(B, T, Hkv, G, D).permute(0, 2, 3, 1, 4), **_tol(dt))
    torch.testing.assert_close(k[:, :, koff:koff + T].float(), rk.permute(0, 2, 1, 3), **_tol(dt))
    assert torch.equal(v[:, :, koff:koff + T], qkv.view(B, T, -1, D)[:, :, Hq + Hkv:].permute(0, 2, 1, 3))
    assert not k[:, :, :koff].any() and not k[:, :, koff + T:].any()
    # backward = transpose rotation; check against autograd of the fp32 reference
    dq = torch.randn(B, Hkv, G, T, D, device=DEV, generator=g).to(dt)
    dk = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(dt)
    dv = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(dt)
    dqkv = torch.empty(B, T, (Hq + 2 * Hkv) * D, device=DEV, dtype=dt)
    native.rope_qkv_bwd(dq, dk, dv, pos, cos, sin, Hq, Hkv, D, dqkv)
    xr = qkv.float().requires_grad_(True)
    xv = xr.view(B, T, Hq + 2 * Hkv, D)
    oq = _rot(xv[:, :, :Hq], c, s).view(B, T, Hkv, G, D).permute(0, 2, 3, 1, 4)
    ok = _rot(xv[:, :, Hq:Hq + Hkv], c, s).permute(0, 2, 1, 3)
    ov = xv[:, :, Hq + Hkv:].permute(0, 2, 1, 3)
    torch.autograd.backward([oq, ok, ov], [dq.float(), dk.float(), dv.float()])
    torch.testing.assert_close(dqkv.float(), xr.grad, **_tol(dt))


def _ref_masked_softmax(S, valid, Tq, qoff, scale):
    """HF semantics: allowed = valid[b, j] & (j <= q + qoff); a fully-masked row is uniform over all keys."""
    B, HG, _, Tk = S.shape
    j = torch.arange(Tk, device=DEV)
    qi = torch.arange(Tq, device=DEV)[:, None]
    allowed = (valid[:, None, None, :].bool()) & (j[None, None, None, :] <= qi[None, None] + qoff)
    z = torch.where(allowed, S * scale, torch.full_like(S, torch.finfo(torch.float32).min))
    return torch.softmax(z, -1)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Tq,Tk,qoff", [(1, 700, 699), (33, 33, 0), (64, 300, 236), (5, 5000, 4995)])
def test_masked_softmax_forward_backward(dt, Tq, Tk, qoff):
    B, HG, scale = 3, 4, 0.125
    g = torch.Generator(device=DEV).manual_seed(Tk)
    S = torch.randn(B, HG, Tq, Tk, device=DEV, generator=g) * 4
    valid = torch.ones(B, Tk, dtype=torch.uint8, device=DEV)
    valid[0, :7] = 0  # left padding
    valid[1, : Tk // 2] = 0
    valid[2, :] = 0  # every row of batch 2 fully masked -> uniform
    P = torch.empty(B, HG, Tq, Tk, device=DEV, dtype=dt)
    native.masked_softmax_fwd(S, P, valid, B, HG, Tq, Tk, qoff, scale)
    ref = _ref_masked_softmax(S, valid, Tq, qoff, scale)
    torch.testing.assert_close(P.float(), ref, rtol=1e-5 if dt == torch.float32 else 1e-2, atol=1e-6 if dt == torch.float32 else 4e-3)
    dP = torch.randn(B, HG, Tq, Tk, device=DEV, generator=g)
    dS = torch.empty_like(P)
    native.masked_softmax_bwd(P, dP, dS, B * HG * Tq, Tk, scale)
    Pf = P.float()
    ref_dS = Pf * (dP - (Pf * dP).sum(-1, keepdim=True)) * scale
    torch.testing.assert_close(dS.float(), ref_dS, **_tol(dt))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("with_delta", [False, True])
@pytest.mark.parametrize("N,H", [(77, 896), (3000, 896), (77, 320)])  # 896: vectorised backward; 320: generic
def test_add_rmsnorm_forward_backward(dt, with_delta, N, H):
    eps = 1e-6
    g = torch.Generator(device=DEV).manual_seed(1)
    x_in = torch.randn(N, H, device=DEV, generator=g)
    delta = torch.randn(N, H, device=DEV, generator=g).to(dt) if with_delta else None
    w = torch.rand(H, device=DEV, generator=g) + 0.5
    x_out = torch.empty_like(x_in) if with_delta else None
    y = torch.empty(N, H, device=DEV, dtype=dt)
    rstd = torch.empty(N, device=DEV)
    native.add_rmsnorm_fwd(x_in, delta, x_out, w, y, rstd, eps)
    x = x_in + (delta.float() if with_delta else 0)
    r = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)
    torch.testing.assert_close(rstd, r[:, 0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(y.float(), (w * (x * r)), **_tol(dt))
    if with_delta:
        torch.testing.assert_close(x_out, x, rtol=0, atol=0)
    # backward accumulates into dx / dw
    dy = torch.randn(N, H, device=DEV, generator=g).to(dt)
    dx = torch.ones(N, H, device=DEV)
    dw = torch.ones(H, device=DEV)
    native.rmsnorm_bwd(x, w, rstd, dy, dx, dw)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    out = wr * (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + eps))
    out.backward(dy.float())
    torch.testing.assert_close(dx, 1 + xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw, 1 + wr.grad, rtol=1e-4, atol=1e-3)
    # pass-through form (drl_rmsnorm_bwd_ex): dx_in read, dx written, bf16 copy from the same pass — bit-identical
    # to the in-place form and to torch's bf16 rounding of it
    res = torch.randn(N, H, device=DEV, generator=g)
    ref = res.clone()
    native.rmsnorm_bwd(x, w, rstd, dy, ref, torch.zeros(H, device=DEV))
    out, lp, dw2 = torch.empty_like(res), torch.empty(N, H, device=DEV, dtype=torch.bfloat16), torch.zeros(H, device=DEV)
    native.rmsnorm_bwd(x, w, rstd, dy, out, dw2, dx_in=res, dx_bf16=lp)
    assert torch.equal(out, ref) and torch.equal(lp, ref.to(torch.bfloat16))
    zero = torch.zeros_like(res)
    native.rmsnorm_bwd(x, w, rstd, dy, zero, torch.zeros(H, device=DEV))
    native.rmsnorm_bwd(x, w, rstd, dy, out, dw2, dx_in=None)
    assert torch.equal(out, zero)


@pytest.mark.parametrize("I", [4864, 36])  # bf16: 16-B-per-lane path (I % 8 == 0) and the generic one
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_swiglu_forward_backward(dt, I):
    N = 131
    g = torch.Generator(device=DEV).manual_seed(2)
    gu = (torch.randn(N, 2 * I, device=DEV, generator=g) * 3).to(dt)
    a = torch.empty(N, I, device=DEV, dtype=dt)
    native.swiglu_fwd(gu, a)
    gr = gu.float().requires_grad_(True)
    ref = torch.nn.functional.silu(gr[:, :I]) * gr[:, I:]
    torch.testing.assert_close(a.float(), ref.detach(), **_tol(dt))
    da = torch.randn(N, I, device=DEV, generator=g).to(dt)
    dgu = torch.empty_like(gu)
    native.swiglu_bwd(gu, da, dgu)
    ref.backward(da.float())
    torch.testing.assert_close(dgu.float(), gr.grad, **_tol(dt))


def _ref_decode(q, k, v, valid, L, qpos):
    B, Hkv, G, D = q.shape
    S = torch.einsum("bhgd,bhtd->bhgt", q.float(), k[:, :, :L].float()) / math.sqrt(D)
    j = torch.arange(L, device=DEV)
    allowed = valid[:, None, None, :L].bool() & (j <= qpos)
    S = S.masked_fill(~allowed, float("-inf"))
    P = torch.softmax(S, -1).nan_to_num(0.0)  # a row with no allowed key: the kernel writes zeros
    return torch.einsum("bhgt,bhtd->bhgd", P, v[:, :, :L].float())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,Hkv,G,D,Tk,L", [(4, 2, 7, 64, 768, 513), (3, 2, 7, 64, 300, 1), (2, 4, 4, 128, 1100, 1100),
                                            (300, 2, 7, 64, 768, 700), (520, 2, 7, 64, 768, 700),
                                            (5, 1, 8, 32, 256, 256)])
def test_decode_attention(dt, B, Hkv, G, D, Tk, L):
    g = torch.Generator(device=DEV).manual_seed(L)
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(dt)
    k = torch.randn(B, Hkv, Tk, D, device=DEV, generator=g).to(dt)
    v = torch.randn(B, Hkv, Tk, D, device=DEV, generator=g).to(dt)
    valid = torch.zeros(B, Tk, dtype=torch.uint8, device=DEV)
    valid[:, :L] = 1
    for b in range(B):  # ragged left padding; the newest key (L-1) is always valid
        valid[b, : min(3 * b, L - 1)] = 0
    out = torch.empty(B, Hkv, G, D, device=DEV, dtype=dt)
    ref = _ref_decode(q, k, v, valid, L, L - 1)
    for split in (True, False):  # split-K + merge (small grids), and the single-pass form
        native.decode_attention(q, k, v, valid, L, out, split=split)
        torch.testing.assert_close(out.float(), ref, **_tol(dt))
    # device-side query position (graph-capturable form) and a position short of L
    if L > 4:
        qp = torch.tensor([L - 4], device=DEV)
        native.decode_attention(q, k, v, valid, L, out, qpos_dev=qp)
        torch.testing.assert_close(out.float(), _ref_decode(q, k, v, valid, L, L - 4), **_tol(dt))
    if dt == torch.bfloat16 and D in (64, 128):
        # MFMA kernel over the head-dim-major V cache (the bf16 rollout layout)
        ldv = (Tk + 7) // 8 * 8
        vt = torch.full((B, Hkv, D, ldv), float("nan"), device=DEV, dtype=dt)
        vt[..., :Tk] = v.transpose(-1, -2)
        ldk = (Tk + 3) // 4 * 4
        valid4 = torch.zeros(B, ldk, dtype=torch.uint8, device=DEV)
        valid4[:, :Tk] = valid
        out2 = torch.empty_like(out)
        native.decode_attention_vt(q, k, vt, valid4[:, :Tk], L, out2)
        torch.testing.assert_close(out2.float(), ref, **_tol(dt))
        if L > 4:
            native.decode_attention_vt(q, k, vt, valid4[:, :Tk], L, out2, qpos_dev=qp)
            torch.testing.assert_close(out2.float(), _ref_decode(q, k, v, valid, L, L - 4), **_tol(dt))


def _ref_attn(q, k, v, valid, qoff):
    """fp32 causal + key-padding attention, grouped layout; rows with no allowed key -> zeros."""
    B, Hkv, G, Tq, D = q.shape
    Tk = k.shape[2]
    S = torch.einsum("bhgtd,bhkd->bhgtk", q.float(), k.float()) / math.sqrt(D)
    j = torch.arange(Tk, device=DEV)
    t = torch.arange(Tq, device=DEV)[:, None] + qoff
    allowed = valid[:, None, None, None, :].bool() & (j <= t)[None, None, None]
    S = S.masked_fill(~allowed, float("-inf"))
    lse = torch.logsumexp(S, -1)
    P = torch.softmax(S, -1).nan_to_num(0.0)
    O = torch.einsum("bhgtk,bhkd->bhgtd", P, v.float())
    return O.permute(0, 3, 1, 2, 4).reshape(B, Tq, Hkv * G * D), lse


@pytest.mark.parametrize("B,Hkv,G,D,Tq,Tk,qoff", [(2, 2, 7, 64, 768, 768, 0), (3, 2, 7, 64, 100, 100, 0),
                                                  (2, 1, 4, 128, 40, 100, 60), (1, 2, 7, 64, 17, 17, 0),
                                                  (2, 2, 8, 64, 64, 64, 0)])
def test_flash_attn_forward(B, Hkv, G, D, Tq, Tk, qoff):
    g = torch.Generator(device=DEV).manual_seed(Tq * 7 + Tk)
    q = torch.randn(B, Hkv, G, Tq, D, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, Tk, D, device=DEV, generator=g).to(torch.bfloat16)
    v = torch.randn(B, Hkv, Tk, D, device=DEV, generator=g).to(torch.bfloat16)
    ld = (Tk + 7) // 8 * 8
    vt = torch.full((B, Hkv, D, ld), float("nan"), device=DEV, dtype=torch.bfloat16)  # pad columns must not leak
    vt[..., :Tk] = v.transpose(-1, -2)
    ldv = (Tk + 3) // 4 * 4
    valid = torch.zeros(B, ldv, dtype=torch.uint8, device=DEV)
    valid[:, :Tk] = 1
    for b in range(B):
        valid[b, : min(5 * b, Tk - 1)] = 0  # left padding: early query rows of b > 0 have no allowed key
    out = torch.empty(B, Tq, Hkv * G * D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, Hkv, G, Tq, device=DEV)
    native.flash_attn_fwd(q, k, vt, valid, out, Tk=Tk, qoff=qoff, lse=lse)
    ref, ref_lse = _ref_attn(q, k, v, valid[:, :Tk], qoff)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    fin = torch.isfinite(ref_lse)
    assert torch.equal(torch.isfinite(lse), fin)
    torch.testing.assert_close(lse[fin], ref_lse[fin], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("T,D", [(45, 64), (130, 64), (8, 64), (77, 128)])
def test_rope_writes_head_dim_major_copies(T, D):
    """The tiled kernel (head-dim-major copies through LDS) matches the per-element kernel bit for bit."""
    B, Hq, Hkv = 2, 14, 2
    G = Hq // Hkv
    g = torch.Generator(device=DEV).manual_seed(T)
    qkv = torch.randn(B, T, (Hq + 2 * Hkv) * D, device=DEV, generator=g).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (B, T), device=DEV, generator=g)
    cos, sin = _rope_tables(D)
    q = torch.empty(B, Hkv, G, T, D, device=DEV, dtype=torch.bfloat16)
    k = torch.empty(B, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    v = torch.empty_like(k)
    native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q, k, v)
    ld = (T + 7) // 8 * 8
    q2, k2, v2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    qt = torch.zeros(B, Hkv, G, D, ld, device=DEV, dtype=torch.bfloat16)
    kt = torch.zeros(B, Hkv, D, ld, device=DEV, dtype=torch.bfloat16)
    vt = torch.zeros_like(kt)
    native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q2, k2, v2, qt=qt, kt=kt, vt=vt)
    assert torch.equal(q2, q) and torch.equal(k2, k) and torch.equal(v2, v)
    assert torch.equal(qt[..., :T], q.transpose(-1, -2))
    assert torch.equal(kt[..., :T], k.transpose(-1, -2))
    assert torch.equal(vt[..., :T], v.transpose(-1, -2))
    vt2 = torch.zeros_like(vt)  # V only transposed (v = None)
    native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q2, k2, None, vt=vt2)
    assert torch.equal(vt2, vt)


def _ref_attn_autograd(q, k, v, valid, dout):
    """fp32 attention (causal + key padding, rows with no allowed key -> 0) and its autograd grads."""
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    B, Hkv, G, T, D = q.shape
    S = torch.einsum("bhgtd,bhkd->bhgtk", qf, kf) / math.sqrt(D)
    j = torch.arange(T, device=DEV)
    allowed = valid[:, None, None, None, :T].bool() & (j <= torch.arange(T, device=DEV)[:, None])[None, None, None]
    S = S.masked_fill(~allowed, -1e30)
    P = torch.softmax(S, -1) * allowed.any(-1, keepdim=True)
    O = torch.einsum("bhgtk,bhkd->bhgtd", P, vf)
    Ob = O.permute(0, 3, 1, 2, 4).reshape(B, T, Hkv * G * D)
    Ob.backward(dout.float())
    return Ob.detach(), qf.grad, kf.grad, vf.grad


@pytest.mark.parametrize("B,Hkv,G,D,T", [(2, 2, 7, 64, 256), (1, 2, 7, 64, 104), (2, 1, 4, 64, 64), (3, 2, 8, 64, 96),
                                         # head_dim 128: Llama-3-8B (G 4), Qwen2.5-7B (G 7), G > 4 heads per wave
                                         (2, 2, 4, 128, 128), (1, 2, 7, 128, 104), (2, 1, 8, 128, 64),
                                         (1, 1, 1, 128, 40)])
def test_flash_attn_backward(B, Hkv, G, D, T):
    g = torch.Generator(device=DEV).manual_seed(T + G)
    q = torch.randn(B, Hkv, G, T, D, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(torch.bfloat16)
    v = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(torch.bfloat16)
    dout = torch.randn(B, T, Hkv * G * D, device=DEV, generator=g).to(torch.bfloat16)
    valid = torch.zeros(B, (T + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    valid[:, :T] = 1
    for b in range(B):
        valid[b, : 7 * b] = 0
    ld = (T + 7) // 8 * 8
    kt = torch.zeros(B, Hkv, D, ld, device=DEV, dtype=torch.bfloat16)
    kt[..., :T] = k.transpose(-1, -2)
    vt = torch.zeros_like(kt)
    vt[..., :T] = v.transpose(-1, -2)
    o = torch.empty(B, T, Hkv * G * D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, Hkv, G, T, device=DEV)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv)
    _, rq, rk, rv = _ref_attn_autograd(q, k, v, valid, dout)
    for name, got, ref in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        err = (got.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert err < 3e-2, f"{name}: max err {err:.3e} relative to max |grad|"
    # deterministic: a second run is bitwise identical
    dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq2, dk2, dv2)
    assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)


@pytest.mark.parametrize("waves,splits", [(4, 2), (8, 4), (2, 8), (16, 1)])
def test_decode_attention_vt_split_plans(waves, splits):
    """Every forced (waves, key-split) plan of the MFMA decode kernel gives the same result as the default
    plan up to fp32 merge rounding (split partial states merged by the last arriving workgroup)."""
    B, Hkv, G, D, Tk = 6, 2, 7, 64, 640
    g = torch.Generator(device=DEV).manual_seed(waves * 10 + splits)
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, Tk, D, device=DEV, generator=g).to(torch.bfloat16)
    vt = torch.randn(B, Hkv, D, Tk, device=DEV, generator=g).to(torch.bfloat16)
    valid = (torch.rand(B, Tk, device=DEV, generator=g) > 0.2).to(torch.uint8)
    valid[0] = 0  # a row with no allowed key
    ref = native.decode_attention_vt(q, k, vt, valid, 600, torch.empty_like(q))
    lib = native.lib()
    lib.drl_decode_attention_set_plan(waves, splits)
    try:
        for _ in range(2):  # the arrival tickets reset themselves between calls
            out = native.decode_attention_vt(q, k, vt, valid, 600, torch.empty_like(q))
            torch.testing.assert_close(out.float(), ref.float(), rtol=2e-2, atol=2e-3)
        assert (out[0] == 0).all()
    finally:
        lib.drl_decode_attention_set_plan(0, 0)


@pytest.mark.parametrize("B,group,shared,cap,L", [(64, 8, 512, 768, 520), (64, 8, 512, 768, 767), (64, 8, 512, 768, 544),
                                                 (6, 1, 0, 640, 600), (16, 2, 96, 300, 290), (8, 1, 0, 100, 40)])
def test_decode_attention_lean_ring_bit_identical(B, group, shared, cap, L):
    """The register-lean loop with two key blocks in flight per wave (on request: measured slower than one at the
    N = 8 rank's 64 rows) == the one-in-flight loop bit for bit (same blocks, same order; a block past a wave's end
    consumed with no valid key), at 8 waves without key splits: prompt groups, a tail block, a wave with one block,
    left padding, a short cache; and the planner's own choice equals both."""
    Hkv, G, D = 2, 7, 64
    g = torch.Generator(device=DEV).manual_seed(B + L)
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(torch.bfloat16)
    vt = torch.randn(B, Hkv, (cap + 31) // 32, D, 32, device=DEV, generator=g).to(torch.bfloat16)
    valid = torch.ones(B, (cap + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    for b in range(B):
        valid[b, : 3 * (b % 5)] = 0
    qp = torch.tensor([L - 1], device=DEV)
    lib = native.lib()
    kw = dict(group=group, shared_keys=shared) if group > 1 else {}
    outs = []
    try:
        for variant in (1, 5):  # one / two blocks in flight
            lib.drl_decode_attention_set_plan(8, 1)
            lib.drl_decode_attention_set_variant(variant)
            outs.append(native.decode_attention_vt(q, k, vt, valid, cap, torch.empty_like(q), qpos_dev=qp, **kw))
    finally:
        lib.drl_decode_attention_set_plan(0, 0)
        lib.drl_decode_attention_set_variant(0)
    assert torch.equal(outs[0], outs[1])
    if B * Hkv <= 256:  # the planner's own plan at this grid: 8 waves, no key split
        auto = native.decode_attention_vt(q, k, vt, valid, cap, torch.empty_like(q), qpos_dev=qp, **kw)
        assert torch.equal(auto, outs[1])


@pytest.mark.parametrize("N,C", [(6144, 1152), (100, 200), (1, 64), (12288, 1152)])
def test_colsum_bf16_acc(N, C):
    """qkv bias gradient: column sums of bf16 dqkv accumulated into the fp32 gradient, deterministic."""
    g = torch.Generator(device=DEV).manual_seed(N + C)
    x = torch.randn(N, C, device=DEV, generator=g).to(torch.bfloat16)
    out = torch.randn(C, device=DEV, generator=g)
    want = out.double() + x.double().sum(0)
    got = native.colsum_bf16_acc(x, out.clone())
    assert (got.double() - want).abs().max().item() <= 1e-5 * (x.double().abs().sum(0).max().item() + 1)
    assert torch.equal(got, native.colsum_bf16_acc(x, out.clone()))


@pytest.mark.parametrize("B,Hkv,G,T,qs", [(2, 2, 7, 256, None), (1, 2, 7, 104, None), (2, 1, 4, 64, None),
                                          (3, 2, 8, 96, None), (2, 2, 7, 200, [0, 70]), (2, 2, 7, 256, [0, 128]),
                                          (1, 2, 7, 32, None), (2, 2, 7, 768, [0, 511])])
def test_flash_dq_two_tiles_bit_identical(B, Hkv, G, T, qs):
    """The dQ kernel over two query tiles per workgroup (csrc/flash_attn.hip flash_dq2_kernel, K / V fragments held
    in registers or re-read per tile) == the one-tile kernel bit for bit: odd and even tile counts, a ragged last tile,
    key-valid holes, and q_start skipping whole lower tiles of a pair (prefix sharing's copies)."""
    D = 64
    g = torch.Generator(device=DEV).manual_seed(T + G + B)
    q = torch.randn(B, Hkv, G, T, D, device=DEV, generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(torch.bfloat16)
    v = torch.randn(B, Hkv, T, D, device=DEV, generator=g).to(torch.bfloat16)
    dout = torch.randn(B, T, Hkv * G * D, device=DEV, generator=g).to(torch.bfloat16)
    valid = torch.zeros(B, (T + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    valid[:, :T] = 1
    for b in range(B):
        valid[b, : 5 * b] = 0
    q_start = torch.tensor(qs, dtype=torch.int32, device=DEV) if qs is not None else None
    if q_start is not None:  # dO is zero on the skipped query rows (the forward never produced them)
        for b, s in enumerate(qs):
            dout[b, : s // 32 * 32] = 0
    ld = (T + 7) // 8 * 8
    kt = torch.zeros(B, Hkv, D, ld, device=DEV, dtype=torch.bfloat16)
    kt[..., :T] = k.transpose(-1, -2)
    vt = torch.zeros_like(kt)
    vt[..., :T] = v.transpose(-1, -2)
    o = torch.zeros(B, T, Hkv * G * D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, Hkv, G, T, device=DEV)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse, q_start=q_start)
    outs = {}
    lib = native.lib()
    try:
        for var in (0, 1, 2):
            lib.drl_flash_attn_bwd_set_variant(var)
            dq = torch.full_like(q, float("nan"))
            dk, dv = torch.empty_like(k), torch.empty_like(v)
            native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv, q_start=q_start)
            outs[var] = (dq, dk, dv)
    finally:
        lib.drl_flash_attn_bwd_set_variant(0)
    for var in (1, 2):
        for a_, b_ in zip(outs[var], outs[0]):
            assert torch.equal(a_, b_), var
