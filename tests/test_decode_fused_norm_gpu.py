"""The fused-norm decode step (csrc/decode_gemm.hip, ABI 8): the decoder layer's RMSNorms folded into the prologue of
the GEMM that consumes them and the residual adds into the epilogue of the GEMM that produces them, five launches per
layer instead of seven (1..128 rows at Qwen2.5-0.5B width). Reference semantics: Qwen2DecoderLayer under the
reference's autocast, per decode token of HF generate (hf_rollout.py:112-124): x += bf16(o) in fp32,
y = bf16(w * (x * rsqrt(mean(x^2) + eps))).

* the residual producer (drl_decode_gemm_resid: K slices summed by the last-arriving slice) == the seven-launch
  step's residual (drl_decode_gemm partials + drl_decode_rmsnorm's add) BIT FOR BIT, every K-slice plan, repeated
  launches, arrival counters back at zero;
* the norm consumers (drl_decode_gemm_norm, drl_decode_qkv_rope_norm) against a plain PyTorch fp32 reference of
  norm -> bf16 -> GEMM -> SwiGLU / bias + RoPE: within one bf16 rounding (the rows' sums of squares and the GEMM's
  fp32 sums run in another order), every kernel configuration, deterministic;
* drl_decode_final_norm from the packed residual == drl_decode_rmsnorm on the row-major residual;
* the whole step: PackedDecode fused vs the seven-launch step on the same cache and tokens (qwen2.5-0.5b width,
  2 layers, prompt groups of 8 as the N = 8 rank runs them), the graphed rollout == eager fused steps.
"""

import pytest
import torch

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0, dtype=BF):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(dtype)


@pytest.fixture
def norm_plan():
    lib = native.lib()
    yield lib.drl_decode_norm_set_plan
    lib.drl_decode_norm_set_plan(-1, 0, 0)


@pytest.mark.parametrize("M", [1, 7, 33, 64, 100, 128])
@pytest.mark.parametrize("N,K", [(896, 896), (896, 4864)])
@pytest.mark.parametrize("max_ks", [0, 1, 2])
def test_resid_equals_partials_then_rmsnorm_add(M, N, K, max_ks, norm_plan):
    norm_plan(-1, 0, max_ks)
    plan = native.decode_norm_plan(M, N, K, native.DECODE_RESID)
    if plan is None:
        pytest.skip("no K-slice plan under this cap")
    ks, mbt, ksw = plan
    x = rnd(M, K, seed=M)
    w = rnd(N, K, scale=0.05, seed=N + K)
    xp = native.pack_activations(x, mbt)
    wp = native.decode_pack_weight(w)
    res = torch.randn(M, N, device=DEV)
    # the seven-launch step: the same one-round-trip kernel's partials (forced to the same shape), then the norm's add
    native.lib().drl_decode_gemm_set_plan(1, ksw)
    try:
        part = native.decode_gemm(xp, wp, M, N, K)
    finally:
        native.lib().drl_decode_gemm_set_plan(0, 0)
    assert part.shape[0] == ks
    x_out = torch.empty_like(res)
    native.decode_rmsnorm(res, part, x_out, torch.ones(N, device=DEV), torch.zeros(mbt * 32 * N, dtype=BF, device=DEV),
                          1e-6, mbt=mbt)
    xr = native.pack_residual(res, mbt)
    partials = torch.empty(ks, M, N, device=DEV)
    cnt = torch.zeros(max(1, native.lib().drl_decode_resid_counter_bytes(M, N, K) // 4), dtype=torch.int32, device=DEV)
    first = None
    for rep in range(4):  # in place: each launch adds the same product again
        native.decode_gemm_resid(xp, wp, M, N, K, xr, mbt, partials, cnt)
        got = native.unpack_residual(xr, M, N, mbt)
        if rep == 0:
            first = got.clone()
            assert torch.equal(got, x_out)
        assert int(cnt.abs().sum()) == 0  # every launch leaves the arrival counters at zero
    # rows past M of the packed residual are never written
    assert torch.count_nonzero(native.unpack_residual(xr, mbt * 32, N, mbt)[M:]) == 0
    # deterministic: the same start gives the same bits
    xr2 = native.pack_residual(res, mbt)
    native.decode_gemm_resid(xp, wp, M, N, K, xr2, mbt, partials, cnt)
    assert torch.equal(native.unpack_residual(xr2, M, N, mbt), first)


def _norm_ref(x, wn, eps):
    r = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)
    return (wn * (x * r)).to(BF)


N_NORM = 4  # csrc/decode_gemm.hip kNorm entries


@pytest.mark.parametrize("M", [1, 5, 32, 64, 100, 128])
def test_gate_up_norm_matches_reference(M, norm_plan):
    I, K, eps = 4864, 896, 1e-6
    gen = torch.Generator(device=DEV).manual_seed(M)  # seeded: the ulp-count bound below is statistical
    x = torch.randn(M, K, device=DEV, generator=gen) * 3
    wn = torch.rand(K, device=DEV, generator=gen) + 0.5
    w = rnd(2 * I, K, scale=0.05, seed=4)
    wp = native.decode_pack_weight(w, swiglu=True)
    y = _norm_ref(x, wn, eps).float()
    gu = (y @ w.float().t()).to(BF).float()
    g, u = gu[:, :I], gu[:, I:]
    ref = ((g / (1 + torch.exp(-g))).to(BF).float() * u).to(BF).float()
    ulp = ref.abs().clamp_min(1e-30) * 2.0 ** -7
    seen = 0
    for ci in [-1] + list(range(N_NORM)):
        norm_plan(ci, 0, 0)
        plan = native.decode_norm_plan(M, 2 * I, K, native.DECODE_SWIGLU)
        if plan is None:
            continue
        seen += 1
        mbt = plan[1]
        xr = native.pack_residual(x, mbt)
        out = torch.zeros(mbt * 32 * I, dtype=BF, device=DEV)
        native.decode_gemm_norm(xr, wn, eps, wp, M, 2 * I, K, out)
        a = native.unpack_activations(out, M, I, mbt).float()
        # three bf16 roundings (gate / up, silu, the product) after an fp32 sum in another order: an element lands
        # more than one ulp off when a rounding boundary flips, ~0.1-0.2 % of them (0.206 % seen on unseeded inputs)
        bad = (a - ref).abs() > ulp * 1.01
        assert bad.float().mean().item() < 4e-3, (ci, bad.float().mean().item())
        assert (a - ref).abs().max().item() <= 2.0 ** -6 * ref.abs().max().item(), ci
        assert torch.count_nonzero(native.unpack_activations(out, mbt * 32, I, mbt)[M:]) == 0
        out2 = torch.zeros_like(out)
        native.decode_gemm_norm(xr, wn, eps, wp, M, 2 * I, K, out2)
        assert torch.equal(out, out2), ci
    assert seen >= 2


@pytest.mark.parametrize("M", [1, 64, 100, 128])
def test_qkv_rope_norm_matches_reference(M, norm_plan):
    K, Hq, Hkv, D, eps = 896, 14, 2, 64, 1e-6
    NQ, G, Tk, koff = (Hq + 2 * Hkv) * D, Hq // Hkv, 32, 9
    gen = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, K, device=DEV, generator=gen) * 2
    wn = torch.rand(K, device=DEV, generator=gen) + 0.5
    w = rnd(NQ, K, scale=0.05, seed=8)
    bias = rnd(NQ, seed=9)
    pos = torch.randint(0, 500, (M,), device=DEV, generator=gen)
    half = D // 2
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    fr = torch.arange(1024, device=DEV).float()[:, None] * inv[None, :half]
    cos_t, sin_t = fr.cos().contiguous(), fr.sin().contiguous()
    kd = torch.tensor([koff], device=DEV)
    # reference: y = norm(x) in bf16, then the unfused one-launch qkv + RoPE on y (drl_decode_qkv_rope)
    y = _norm_ref(x, wn, eps)
    mbt = native.decode_gemm_plan(M, NQ, K)[1]
    ref = (torch.zeros(M, Hkv, G, D, dtype=BF, device=DEV), torch.zeros(M, Hkv, Tk, D, dtype=BF, device=DEV),
           torch.zeros(M, Hkv, D, Tk, dtype=BF, device=DEV))
    wpr = native.decode_pack_weight_rope(w, D)
    native.decode_qkv_rope(native.pack_activations(y, mbt), wpr, bias, pos, cos_t, sin_t, M, K, Hq, Hkv, D, *ref, kd)
    for ci in [-1, 0, 1]:
        norm_plan(ci, 0, 0)
        plan = native.decode_norm_plan(M, NQ, K, native.DECODE_ROPE)
        assert plan is not None and plan[1] == mbt
        xr = native.pack_residual(x, mbt)
        got = (torch.zeros(M, Hkv, G, D, dtype=BF, device=DEV), torch.zeros(M, Hkv, Tk, D, dtype=BF, device=DEV),
               torch.zeros(M, Hkv, D, Tk, dtype=BF, device=DEV))
        native.decode_qkv_rope_norm(xr, wn, eps, wpr, bias, pos, cos_t, sin_t, M, K, Hq, Hkv, D, *got, kd)
        for a, b in zip(got, ref):
            a, b = a.float(), b.float()
            scale = b.abs().max().item()
            # one bf16 rounding of an input (y) or of the projection before the rotation
            assert (a - b).abs().max().item() <= 2.0 ** -5 * scale, ci
            assert ((a - b).abs() > 2.0 ** -8 * b.abs().clamp_min(1e-3)).float().mean().item() < 0.02, ci


@pytest.mark.parametrize("M", [1, 64, 128])
def test_final_norm_from_packed_residual(M):
    H, eps = 896, 1e-6
    x = torch.randn(M, H, device=DEV)
    wn = torch.rand(H, device=DEV) + 0.5
    mbt = native.decode_gemm_plan(M, H, H)[1]
    y0 = torch.empty(M, H, dtype=BF, device=DEV)
    native.decode_rmsnorm(x, None, None, wn, y0, eps, mbt=0)
    y1 = torch.empty(M, H, dtype=BF, device=DEV)
    native.decode_final_norm(native.pack_residual(x, mbt), mbt, wn, y1, M, H, eps)
    assert torch.equal(y0, y1)


def _width896_model(seed=0, layers=2):
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(dict(vocab_size=4096, hidden_size=896, intermediate_size=4864,
                                     num_hidden_layers=layers, num_attention_heads=14, num_key_value_heads=2,
                                     max_position_embeddings=2048, rope_theta=1e6, rms_norm_eps=1e-6,
                                     tie_word_embeddings=True))
    store = ParamStore(cfg, DEV, compute_dtype=BF, trainable=False)
    store.init_random(seed)
    return cfg, Qwen2Model(cfg, store)


@pytest.mark.parametrize("B,group", [(64, 8), (40, 1), (128, 8)])
def test_fused_step_tracks_seven_launch_step(B, group):
    """PackedDecode with the fused-norm layer vs the seven-launch layer on the same prefilled cache and the same
    teacher-forced tokens: the final hidden states and the K / V written agree at bf16 level step after step (the
    norms' sums of squares run in another fp32 order); the residual stream of the first step is bit-identical."""
    from dots.rl_amd.qwen2 import KVCache, KVCacheRows, PackedDecode

    cfg, m = _width896_model()
    P, R = 64, 6
    g = torch.Generator(device=DEV).manual_seed(1)
    n = B // group
    ids = torch.randint(0, cfg.vocab_size, (n, P), device=DEV, generator=g).repeat_interleave(group, 0)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    caches = []
    for _ in range(2):
        c = KVCache(cfg, B, P + R, DEV, BF)
        c.valid[:, :P] = 1
        if group > 1:
            m.prefill(KVCacheRows(c, 0, n), ids[::group].contiguous(), am[::group].contiguous(),
                      pos[::group].contiguous())
            c.share_prompts(group, P)
        else:
            m.prefill(c, ids, am, pos)
        caches.append(c)
    pf, pu = PackedDecode(m, B, fused_norm=True), PackedDecode(m, B, fused_norm=False)
    assert pf.fused and not pu.fused
    toks = torch.randint(0, cfg.vocab_size, (B, R), device=DEV, generator=g)
    for t in range(1, R):
        kd = torch.tensor([P + t - 1], device=DEV)
        h0 = pu.step(caches[0], toks[:, t - 1:t], pos[:, -1] + t, kd).float()
        h1 = pf.step(caches[1], toks[:, t - 1:t], pos[:, -1] + t, kd).float()
        err = (h0 - h1).abs().max().item() / h0.abs().max().item()
        assert err < 3e-2, (t, err)
        assert (h0 - h1).abs().mean().item() < 3e-3 * h0.abs().mean().item() + 1e-6, t
    nn = P + R - 1
    for i in range(cfg.num_hidden_layers):  # the response slots the steps wrote (prompt rows past a group's first
        # cache row are never written under prefix caching)
        for a, b in ((caches[0].k[i][:, :, P:nn], caches[1].k[i][:, :, P:nn]),
                     (caches[0].vt_plain(i)[..., P:nn], caches[1].vt_plain(i)[..., P:nn])):
            assert (a.float() - b.float()).abs().max().item() <= 3e-2 * a.float().abs().max().item()


def test_fused_rollout_graph_equals_eager():
    """The rollout's graphed decode loop on the fused-norm step (64 rows, prompt groups of 8: the N = 8 rank's shape)
    replays exactly what eager fused steps produce (greedy)."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.qwen2 import KVCache, KVCacheRows, PackedDecode
    from dots.rl_amd.rollout import MI355XRollout

    B, P, R, group = 64, 64, 10, 8
    cfg, m = _width896_model(seed=3)
    g = torch.Generator(device=DEV).manual_seed(2)
    ids = torch.randint(3, cfg.vocab_size, (B // group, P), device=DEV, generator=g).repeat_interleave(group, 0)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    rcfg = to_attr(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0, response_length=R, ignore_eos=True,
                        seed=0, val_kwargs={}, use_hip_graph=True, packed_decode=True, n=group,
                        decode_fused_norm=True))
    ro = MI355XRollout(m, rcfg)
    out = ro.generate_sequences(DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos},
                                                    meta_info={"eos_token_id": 2, "pad_token_id": 0}))
    assert ro.last_packed_decode
    resp = out.batch["responses"]
    cache = KVCache(cfg, B, P + R, DEV, BF)
    cache.valid[:, :P] = 1
    h = m.prefill(KVCacheRows(cache, 0, B // group), ids[::group].contiguous(), am[::group].contiguous(),
                  pos[::group].contiguous()).repeat_interleave(group, 0)
    cache.share_prompts(group, P)
    pk = PackedDecode(m, B, fused_norm=True)
    assert pk.fused

    def pick(h):
        o = torch.empty(B, dtype=torch.int64, device=DEV)
        return m.select_tokens(h, o, fused=False, logits_fn=pk.logits)  # the step's own lm_head, as the rollout

    toks = [pick(h)]
    for t in range(1, R):
        kd = torch.tensor([P + t - 1], device=DEV)
        h = pk.step(cache, toks[-1].view(B, 1), pos[:, -1] + t, kd)
        toks.append(pick(h))
    assert torch.equal(resp, torch.stack(toks, 1))


@pytest.mark.parametrize("M", [1, 7, 32, 33, 64])
@pytest.mark.parametrize("V", [151936, 5003])
def test_decode_lm_head_matches_fp32_reference(M, V):
    """The decode lm_head (persistent: the packed h panel in LDS, each workgroup streaming its contiguous range of the
    packed weight, k16 steps split over 8 waves) against the fp32 product of the same bf16 operands rounded once to
    bf16: within one bf16 rounding everywhere (the fp32 sums run in another order), bit-identical run to run; logits
    columns past V untouched."""
    K = 896
    mbt = native.decode_lm_head_plan(M, V, K)
    assert mbt == (2 if M > 32 else 1)
    h = rnd(M, K, seed=M)
    w = rnd(V, K, scale=0.05, seed=V)
    hp = native.pack_activations(h, mbt)
    wp = native.decode_pack_weight(w)
    ld = (V + 3) // 4 * 4 + 8  # the kernel's contract: ld % 4 == 0
    out = torch.full((M, ld), 7.0, dtype=BF, device=DEV)[:, :V]
    native.decode_lm_head(hp, mbt, wp, M, V, K, out)
    ref = h.float() @ w.float().t()
    got = out.float()
    err = (got - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 1e-3).float().mean().item() > 0.999
    assert err.max().item() <= 2.0 ** -7 * ref.abs().max().item()
    out2 = torch.empty(M, ld, dtype=BF, device=DEV)[:, :V]
    native.decode_lm_head(hp, mbt, wp, M, V, K, out2)
    assert torch.equal(out, out2)
    assert torch.all(out.as_strided((M, ld - V), (ld, 1), V).float() == 7.0)


def test_packed_decode_logits_use_the_decode_lm_head():
    """PackedDecode.logits at 64 rows: the decode lm_head on the final norm's packed copy == drl_gemm's lm_head on the
    row-major h within one bf16 rounding; the same h in both forms."""
    from dots.rl_amd.qwen2 import KVCache, PackedDecode

    cfg, m = _width896_model(seed=5)
    B, P = 64, 32
    cache = KVCache(cfg, B, P + 4, DEV, BF)
    ids = torch.randint(0, cfg.vocab_size, (B, P), device=DEV)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    m.prefill(cache, ids, am, pos)
    pk = PackedDecode(m, B)
    assert pk.lm_w is not None
    kd = torch.tensor([P], device=DEV)
    h = pk.step(cache, ids[:, -1:], pos[:, -1] + 1, kd)
    assert torch.equal(native.unpack_activations(pk.h_pk, B, cfg.hidden_size, pk.lm_mbt), h)
    a = pk.logits(h).float()
    b = m.logits(h).float()
    assert (a - b).abs().max().item() <= 2.0 ** -7 * b.abs().max().item()
