"""Decode-step projections on fragment-packed operands (csrc/decode_gemm.hip) and their producers /
consumers, each against a plain PyTorch fp32 reference of the same bf16 module math:

* pack / unpack of the activation panel is a bijection (host helper == device layout, via the GEMM);
* drl_decode_gemm PARTIAL: sum of the fp32 partial slices == x W^T in fp32 (bf16 operands): 1e-5 relative
  (fp32 accumulation, different order);
* SWIGLU: bf16(bf16(silu(bf16 g)) * bf16 u) — within 1 bf16 ulp of the reference on 99.9 % of entries and
  2^-6 of the panel's largest entry everywhere (the fp32 sums differ in order before the three roundings);
* drl_decode_rmsnorm == drl_add_rmsnorm_fwd fed the bf16-rounded delta (bit-exact when the delta is the same);
* drl_decode_rope == drl_rope_qkv_fwd on the same bf16 qkv (bit-exact);
* decode attention with a packed output == its row-major output, packed (bit-exact).
"""

import math

import pytest
import torch

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0, dtype=BF):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(dtype)


@pytest.mark.parametrize("M", [1, 7, 32, 33, 64, 100, 128, 257, 512])  # >= 192 rows: the MFMA-tiled form
@pytest.mark.parametrize("N,K", [(1152, 896), (896, 896), (896, 4864), (96, 64), (200, 128)])
def test_decode_gemm_partials(M, N, K):
    plan = native.decode_gemm_plan(M, N, K)
    assert plan is not None
    ks, mbt = plan
    x = rnd(M, K, seed=M)
    w = rnd(N, K, scale=0.05, seed=N + K)
    xp = native.pack_activations(x, mbt)
    assert torch.equal(native.unpack_activations(xp, M, K, mbt), x)
    wp = native.decode_pack_weight(w)
    part = native.decode_gemm(xp, wp, M, N, K)
    assert part.shape == (ks, M, N)
    ref = x.float() @ w.float().t()
    got = part.sum(0)
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err
    assert torch.equal(part, native.decode_gemm(xp, wp, M, N, K))  # deterministic


@pytest.mark.parametrize("M", [200, 512])
@pytest.mark.parametrize("N,K", [(896, 4864), (896, 896)])
def test_decode_gemm_every_tiled_configuration(M, N, K):
    """Every MFMA-tiled configuration (csrc/decode_gemm.hip kTiled, forced) gives the planner's K-slice sums within
    fp32 rounding of the fp32 product, deterministically."""
    x = rnd(M, K, seed=M + 1)
    w = rnd(N, K, scale=0.05, seed=N + K + 1)
    ref = x.float() @ w.float().t()
    wp = native.decode_pack_weight(w)
    lib = native.lib()
    try:
        for ci in range(N_TILED):
            lib.drl_decode_gemm_force_tiled(ci, 1)
            ks, mbt = native.decode_gemm_plan(M, N, K)
            xp = native.pack_activations(x, mbt)
            part = native.decode_gemm(xp, wp, M, N, K)
            err = (part.sum(0) - ref).abs().max().item() / ref.abs().max().item()
            assert err < 1e-5, (ci, err)
            assert torch.equal(part, native.decode_gemm(xp, wp, M, N, K)), ci
    finally:
        lib.drl_decode_gemm_force_tiled(-1, 0)


N_TILED = 23  # csrc/decode_gemm.hip kTiled entries


@pytest.mark.parametrize("M", [64, 128, 300, 512])
def test_decode_gemm_swiglu_every_tiled_configuration(M):
    """The SwiGLU epilogue (whole K per workgroup) under every forced tiled configuration: every tiled configuration
    accumulates each output block's k-steps in the same order, so all are bit-identical to one another, deterministic,
    and within bf16 rounding of the one-round-trip kernel (4 waves on K quarters, another summation order)."""
    I, K = 4864, 896
    x = rnd(M, K, seed=M + 7)
    w = rnd(2 * I, K, scale=0.05, seed=11)
    wp = native.decode_pack_weight(w, swiglu=True)
    lib = native.lib()
    try:
        lib.drl_decode_gemm_set_tiled(0)
        ks, mbt = native.decode_gemm_plan(M, 2 * I, K, swiglu=True)
        xp = native.pack_activations(x, mbt)
        rt = native.unpack_activations(native.decode_gemm(xp, wp, M, 2 * I, K, swiglu=True), M, I, mbt).float()
        lib.drl_decode_gemm_set_tiled(1)
        want = None
        for ci in range(N_TILED):
            lib.drl_decode_gemm_force_tiled(ci, 1)
            assert native.decode_gemm_plan(M, 2 * I, K, swiglu=True)[1] == mbt
            got = native.decode_gemm(xp, wp, M, 2 * I, K, swiglu=True)
            if want is None:
                want = got.clone()
                a = native.unpack_activations(got, M, I, mbt).float()
                assert (a - rt).abs().max() <= 0.02 * rt.abs().max()
            assert torch.equal(got[:mbt * 32 * I], want[:mbt * 32 * I]), ci
            assert torch.equal(got, native.decode_gemm(xp, wp, M, 2 * I, K, swiglu=True)), ci
    finally:
        lib.drl_decode_gemm_force_tiled(-1, 0)
        lib.drl_decode_gemm_set_tiled(1)


@pytest.mark.parametrize("M", [5, 64, 128, 300, 512])
@pytest.mark.parametrize("I,K", [(4864, 896), (128, 64)])
def test_decode_gemm_swiglu_packed(M, I, K):
    ks, mbt = native.decode_gemm_plan(M, 2 * I, K, swiglu=True)
    assert ks == 1
    x = rnd(M, K, seed=3)
    w = rnd(2 * I, K, scale=0.05, seed=4)
    out = native.decode_gemm(native.pack_activations(x, mbt), native.decode_pack_weight(w, swiglu=True), M, 2 * I, K,
                             swiglu=True)
    a = native.unpack_activations(out, M, I, mbt).float()
    gu = (x.float() @ w.float().t()).to(BF).float()
    g, u = gu[:, :I], gu[:, I:]
    ref = ((g / (1 + torch.exp(-g))).to(BF).float() * u).to(BF).float()
    ulp = ref.abs().clamp_min(1e-30) * 2.0 ** -7
    bad = (a - ref).abs() > ulp * 1.01
    assert bad.float().mean().item() < 1e-3
    # where a differently-ordered fp32 sum rounds g or u to the neighbouring bf16 value the output moves by that
    # input ulp scaled through silu / the product: bounded relative to the panel's scale
    assert (a - ref).abs().max().item() <= 2.0 ** -6 * ref.abs().max().item()
    # rows past M of the packed panel stay zero (the next GEMM reads them)
    assert torch.count_nonzero(native.unpack_activations(out, mbt * 32, I, mbt)[M:]) == 0


@pytest.mark.parametrize("M,H,ns", [(64, 896, 4), (3, 64, 1), (128, 896, 19)])
def test_decode_rmsnorm_matches_add_rmsnorm(M, H, ns):
    x = torch.randn(M, H, device=DEV)
    part = torch.randn(ns, M, H, device=DEV) * 0.3
    w = torch.rand(H, device=DEV) + 0.5
    mbt = (M + 31) // 32
    yp = torch.zeros(mbt * 32 * H, dtype=BF, device=DEV)
    x_out = torch.empty_like(x)
    native.decode_rmsnorm(x, part, x_out, w, yp, 1e-6, mbt=mbt)
    delta = part.sum(0).to(BF)  # same fixed order: k = 0, 1, ...
    s = part[0].clone()
    for k in range(1, ns):
        s += part[k]
    delta = s.to(BF)
    x2, y2 = torch.empty_like(x), torch.empty(M, H, dtype=BF, device=DEV)
    native.add_rmsnorm_fwd(x.view(M, 1, H), delta.view(M, 1, H), x2.view(M, 1, H), w, y2.view(M, 1, H), None, 1e-6)
    assert torch.equal(x_out, x2)
    y = native.unpack_activations(yp, M, H, mbt)
    assert (y.float() - y2.float()).abs().max().item() <= 2.0 ** -7 * y2.float().abs().max().item()
    # row-major output form, no delta
    yr = torch.empty(M, H, dtype=BF, device=DEV)
    native.decode_rmsnorm(x, None, None, w, yr, 1e-6, mbt=0)
    y3 = torch.empty(M, H, dtype=BF, device=DEV)
    native.add_rmsnorm_fwd(x.view(M, 1, H), None, None, w, y3.view(M, 1, H), None, 1e-6)
    assert (yr.float() - y3.float()).abs().max().item() <= 2.0 ** -7 * y3.float().abs().max().item()


def test_decode_rope_matches_rope_qkv():
    B, Hq, Hkv, D, Tk, koff = 64, 14, 2, 64, 40, 17
    G = Hq // Hkv
    NQ = (Hq + 2 * Hkv) * D
    ns = 3
    part = torch.randn(ns, B, NQ, device=DEV)
    bias = rnd(NQ, seed=5)
    pos = torch.randint(0, 1000, (B,), device=DEV)
    half = D // 2
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    fr = torch.arange(2048, device=DEV).float()[:, None] * inv[None, :half]
    cos_t, sin_t = fr.cos().contiguous(), fr.sin().contiguous()
    s = part[0].clone()
    for k in range(1, ns):
        s += part[k]
    qkv = (s + bias.float()).to(BF).view(B, 1, NQ)
    q1 = torch.empty(B, Hkv, G, 1, D, dtype=BF, device=DEV)
    k1 = torch.zeros(B, Hkv, Tk, D, dtype=BF, device=DEV)
    vt1 = torch.zeros(B, Hkv, D, 48, dtype=BF, device=DEV)[..., :Tk]
    native.rope_qkv_fwd(qkv, pos.view(B, 1), cos_t, sin_t, Hq, Hkv, D, q1, k1, None, koff=koff, vt=vt1)
    q2 = torch.empty_like(q1)
    k2 = torch.zeros_like(k1)
    vt2 = torch.zeros(B, Hkv, D, 48, dtype=BF, device=DEV)[..., :Tk]
    kd = torch.tensor([koff], device=DEV)
    native.decode_rope(part, bias, pos, cos_t, sin_t, Hq, Hkv, D, q2, k2, vt_cache=vt2, koff_dev=kd)
    assert torch.equal(q1, q2) and torch.equal(k1, k2) and torch.equal(vt1, vt2)


def test_decode_attention_packed_output():
    B, Hkv, G, D, Tk, L = 70, 2, 7, 64, 96, 81
    q = rnd(B, Hkv, G, D, seed=1)
    k = rnd(B, Hkv, Tk, D, seed=2)
    vt = rnd(B, Hkv, D, Tk, seed=3)
    valid = torch.ones(B, Tk, dtype=torch.uint8, device=DEV)
    valid[:5, :9] = 0
    out = torch.empty(B, Hkv * G * D, dtype=BF, device=DEV)
    native.decode_attention_vt(q, k, vt, valid, L, out)
    mbt = 4
    outp = torch.zeros(mbt * 32 * Hkv * G * D, dtype=BF, device=DEV)
    native.decode_attention_vt(q, k, vt, valid, L, outp, out_mbt=mbt)
    assert torch.equal(native.unpack_activations(outp, B, Hkv * G * D, mbt), out)
    assert math.isfinite(out.float().sum().item())


def _small_model(seed=0, B=48):
    from dots.rl_amd.qwen2 import KVCache, ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                     num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=512,
                                     rope_theta=10000.0, rms_norm_eps=1e-6, tie_word_embeddings=True))
    store = ParamStore(cfg, DEV, compute_dtype=BF, trainable=False)
    store.init_random(seed)
    return cfg, Qwen2Model(cfg, store)


@pytest.mark.parametrize("B", [5, 48, 130, 512])
def test_packed_decode_step_tracks_unpacked(B):
    """PackedDecode.step (8 launches per layer on packed operands) against the unpacked decode step on the same
    prefilled cache and the same teacher-forced tokens: final hidden states and the written K/V agree at bf16
    level (the projections sum in a different order), step after step."""
    from dots.rl_amd.qwen2 import KVCache, PackedDecode

    cfg, m = _small_model(B=B)
    assert PackedDecode.supported(m, B)
    P, R = 24, 6
    g = torch.Generator(device=DEV).manual_seed(1)
    ids = torch.randint(0, 512, (B, P), device=DEV, generator=g)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    am[:3, :5] = 0
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    caches = []
    for _ in range(2):
        c = KVCache(cfg, B, P + R, DEV, BF)
        m.prefill(c, ids, am, pos)
        caches.append(c)
    pk = PackedDecode(m, B)
    toks = torch.randint(0, 512, (B, R), device=DEV, generator=g)
    for t in range(1, R):
        kd = torch.tensor([P + t - 1], device=DEV)
        h0 = m.decode_step_dev(caches[0], toks[:, t - 1:t], pos[:, -1] + t, kd).float()
        h1 = pk.step(caches[1], toks[:, t - 1:t], pos[:, -1] + t, kd).float()
        err = (h0 - h1).abs().max().item() / h0.abs().max().item()
        assert err < 3e-2, (t, err)
    n = P + R - 1  # positions written (the last cache slot is never filled here)
    for i in range(cfg.num_hidden_layers):
        for a, b in ((caches[0].k[i][:, :, :n], caches[1].k[i][:, :, :n]),
                     (caches[0].vt_plain(i)[..., :n], caches[1].vt_plain(i)[..., :n])):
            assert (a.float() - b.float()).abs().max().item() <= 3e-2 * a.float().abs().max().item()
    assert torch.equal(caches[0].valid, caches[1].valid)


def test_packed_rollout_graph_equals_eager():
    """The rollout's HIP-graph decode loop on the packed path replays exactly what eager packed steps produce
    (greedy), and the rollout outputs keep HFRollout's structure."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.qwen2 import KVCache, PackedDecode
    from dots.rl_amd.rollout import MI355XRollout

    B, P, R = 40, 16, 12
    cfg, m = _small_model(seed=3)
    g = torch.Generator(device=DEV).manual_seed(2)
    ids = torch.randint(0, 512, (B, P), device=DEV, generator=g)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    rcfg = to_attr(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0, response_length=R, ignore_eos=True,
                        seed=0, val_kwargs={}, use_hip_graph=True, packed_decode=True))
    ro = MI355XRollout(m, rcfg)
    out = ro.generate_sequences(DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos},
                                                    meta_info={"eos_token_id": 2, "pad_token_id": 0}))
    assert ro.last_packed_decode
    resp = out.batch["responses"]
    # eager packed greedy loop
    cache = KVCache(cfg, B, P + R, DEV, BF)
    h = m.prefill(cache, ids, am, pos)
    pk = PackedDecode(m, B)
    def pick(h):
        out = torch.empty(B, dtype=torch.int64, device=DEV)
        return m.select_tokens(h, out, fused=True)

    toks = [pick(h)]
    for t in range(1, R):
        kd = torch.tensor([P + t - 1], device=DEV)
        h = pk.step(cache, toks[-1].view(B, 1), pos[:, -1] + t, kd)
        toks.append(pick(h))
    assert torch.equal(resp, torch.stack(toks, 1))
    assert out.batch["input_ids"].shape == (B, P + R)


@pytest.mark.parametrize("do_sample", [False, True])
def test_decode_prologue_equals_torch_bookkeeping(do_sample):
    """The graphed step's one-launch prologue (embedding, rotary positions, cache slot, key_valid, step counter)
    replays exactly what the torch bookkeeping does: identical responses, sampled or greedy, on left-padded prompts
    (per-row positions) with EOS stops; the device step counter ends at R."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    B, P, R = 24, 16, 14
    cfg, m = _small_model(seed=5)
    g = torch.Generator(device=DEV).manual_seed(9)
    ids = torch.randint(3, 512, (B, P), device=DEV, generator=g)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    for b in range(0, B, 3):
        am[b, : (b % 7)] = 0  # left padding
    ids = torch.where(am == 0, torch.zeros_like(ids), ids)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    outs = []
    for prologue in (True, False):
        rcfg = to_attr(dict(do_sample=do_sample, temperature=0.9, top_k=-1, top_p=1.0, response_length=R,
                            ignore_eos=False, seed=11, val_kwargs={}, use_hip_graph=True, packed_decode=True,
                            decode_prologue=prologue))
        ro = MI355XRollout(m, rcfg)
        out = ro.generate_sequences(DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos},
                                                        meta_info={"eos_token_id": 2, "pad_token_id": 0}))
        assert ro.last_packed_decode
        outs.append(out.batch)
    for k in ("responses", "attention_mask", "position_ids"):
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("M,K,Hq,Hkv,D", [(64, 896, 14, 2, 64), (5, 128, 2, 1, 64), (100, 256, 4, 2, 128),
                                           (512, 896, 14, 2, 64), (200, 256, 4, 2, 128)])
def test_decode_qkv_rope_matches_gemm_then_rope(M, K, Hq, Hkv, D):
    """One-launch qkv_proj + bias + RoPE (rotation-pair packing) == the two-launch form (decode GEMM with the
    same single K slice, then decode RoPE) bit for bit: the same fp32 sums in the same order, the same roundings."""
    NQ = (Hq + 2 * Hkv) * D
    G, Tk, koff = Hq // Hkv, 32, 9
    x = rnd(M, K, seed=7)
    w = rnd(NQ, K, scale=0.05, seed=8)
    bias = rnd(NQ, seed=9)
    pos = torch.randint(0, 500, (M,), device=DEV)
    half = D // 2
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    fr = torch.arange(1024, device=DEV).float()[:, None] * inv[None, :half]
    cos_t, sin_t = fr.cos().contiguous(), fr.sin().contiguous()
    kd = torch.tensor([koff], device=DEV)
    mbt = native.decode_gemm_plan(M, NQ, K)[1]
    xp = native.pack_activations(x, mbt)
    outs = []
    for fused in (True, False):
        q = torch.zeros(M, Hkv, G, D, dtype=BF, device=DEV)
        kc = torch.zeros(M, Hkv, Tk, D, dtype=BF, device=DEV)
        vt = torch.zeros(M, Hkv, D, Tk, dtype=BF, device=DEV)
        if fused:
            native.decode_qkv_rope(xp, native.decode_pack_weight_rope(w, D), bias, pos, cos_t, sin_t, M, K, Hq, Hkv, D,
                                   q, kc, vt, kd)
        else:
            # the fused launch's shape at every row count: the one-round-trip kernel, one-block workgroups, whole
            # K per workgroup (K / 64 k16-steps per wave)
            native.lib().drl_decode_gemm_set_plan(1, K // 64)
            native.lib().drl_decode_gemm_set_tiled(0)
            part = native.decode_gemm(xp, native.decode_pack_weight(w), M, NQ, K)
            native.lib().drl_decode_gemm_set_tiled(1)
            native.lib().drl_decode_gemm_set_plan(0, 0)
            assert part.shape[0] == 1
            native.decode_rope(part, bias, pos, cos_t, sin_t, Hq, Hkv, D, q, kc, vt_cache=vt, koff_dev=kd)
        outs.append((q, kc, vt))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,H,V", [(64, 896, 151936), (300, 128, 5003), (1, 64, 257)])
def test_linear_select_matches_unfused(N, H, V):
    """lm_head fused with greedy K4 (no logits written) against K4 on the bf16 logits of the same GEMM: the same
    token wherever the fp32 sums round to the same bf16 logits (>= 99 % of rows; a differing row must be a
    near-tie: its pick is within one bf16 ulp of the unfused pick's logit). Sampling is refused (the two-level
    race reads one slice of the logits row)."""
    h = rnd(N, H, seed=N)
    w = rnd(V, H, scale=0.05, seed=V)
    with pytest.raises(RuntimeError, match="drl_select_tokens"):
        native.linear_select_tokens(h, w, torch.empty(N, dtype=torch.int64, device=DEV), do_sample=True,
                                    temperature=0.8)
    sample = False
    kw = dict(do_sample=sample, temperature=1.0, seed=1234, step=3, row_base=5)
    a = native.linear_select_tokens(h, w, torch.empty(N, dtype=torch.int64, device=DEV), **kw)
    logits = h @ w.t()
    b = native.select_tokens(logits, torch.empty(N, dtype=torch.int64, device=DEV), **kw)
    same = (a == b).float().mean().item()
    assert same >= (0.99 if N >= 100 else 0.95), same
    lf = logits.float()
    for r in torch.nonzero(a != b).flatten().tolist():
        la, lb = lf[r, a[r]].item(), lf[r, b[r]].item()
        if not sample:
            assert abs(la - lb) <= 2.0 ** -7 * max(abs(la), abs(lb)) + 1e-6
    # finished rows get the pad token, EOS finishes a row
    unf = torch.ones(N, dtype=torch.int32, device=DEV)
    unf[0] = 0
    eos = a[-1:].clone()
    out = native.linear_select_tokens(h, w, torch.empty(N, dtype=torch.int64, device=DEV), pad_token_id=7,
                                      eos_ids=eos, unfinished=unf, **kw)
    assert out[0].item() == 7 or N == 1
    if N > 1:
        assert unf[-1].item() == 0
    assert torch.equal(out[1:], a[1:]) or N == 1


@pytest.mark.parametrize("lanes,do_sample", [(2, False), (2, True), (4, True)])
def test_decode_lanes_equal_per_lane_eager_steps(lanes, do_sample):
    """Row lanes of the graphed decode step (rollout.decode_lanes: each row group's step on its own stream of one
    graph, packed weights shared, workspaces per lane) produce exactly what eager packed steps of each row group
    produce on the same prefilled cache: identical responses, greedy or sampled (lane j's Philox rows start at
    row_base + j * B / lanes)."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.qwen2 import KVCache, KVCacheRows, PackedDecode
    from dots.rl_amd.rollout import MI355XRollout

    B, P, R = 32 * lanes, 16, 12
    cfg, m = _small_model(seed=4)
    g = torch.Generator(device=DEV).manual_seed(6)
    ids = torch.randint(3, 512, (B, P), device=DEV, generator=g)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    for b in range(0, B, 5):
        am[b, : (b % 6)] = 0
    ids = torch.where(am == 0, torch.zeros_like(ids), ids)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    seed, temp = 21, 0.8
    rcfg = to_attr(dict(do_sample=do_sample, temperature=temp, top_k=-1, top_p=1.0, response_length=R,
                        ignore_eos=True, seed=seed, val_kwargs={}, use_hip_graph=True, packed_decode=True,
                        decode_lanes=lanes))
    ro = MI355XRollout(m, rcfg)
    assert ro._decode_lanes(B, 512) == lanes
    out = ro.generate_sequences(DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos},
                                                    meta_info={"eos_token_id": 2, "pad_token_id": 0}))
    resp = out.batch["responses"]
    # eager reference: one prefill of all B rows, then each row group stepped by its own PackedDecode
    cache = KVCache(cfg, B, P + R, DEV, BF)
    h = m.prefill(cache, ids, am, pos)
    sel = dict(do_sample=do_sample, temperature=temp if do_sample else 1.0, top_k=0, top_p=1.0, seed=seed,
               pad_token_id=0)
    toks = torch.empty(B, R, dtype=torch.int64, device=DEV)
    m.select_tokens(h, toks[:, 0], fused=False, step=0, row_base=0, **sel)
    rows = B // lanes
    pks = [PackedDecode(m, rows) for _ in range(lanes)]
    for t in range(1, R):
        kd = torch.tensor([P + t - 1], device=DEV)
        for j in range(lanes):
            r0, r1 = j * rows, (j + 1) * rows
            cj = KVCacheRows(cache, r0, r1)
            hj = pks[j].step(cj, toks[r0:r1, t - 1:t], pos[r0:r1, -1] + t, kd)
            m.select_tokens(hj, toks[r0:r1, t], fused=False, step=t, row_base=r0, **sel)
    assert torch.equal(resp, toks)
