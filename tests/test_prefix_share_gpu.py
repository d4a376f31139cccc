"""Prefix sharing in the actor / ref passes (model.share_prompt_prefix, qwen2.PrefixShare): the samples of one prompt
run the prompt's tokens once. The reference computes every sample's copy (dp_actor.py:119-247); the copies are the
same function of the same tokens, so sharing changes the order of the fp32 / bf16 sums only. Checks:

* drl_sum_rows (the adjoint of a shared gather) against torch, both dtypes, missing terms;
* the PrefixShare maps: which positions are packed, and unpack / pack_grad and pack / unpack_grad adjoint pairs;
* fp32 tiny Qwen2 (reference weights): log-probs, entropy and the full gradient with and without sharing, on
  groups of left-padded prompts with EOS-terminated responses, padded and remove-padding layouts: fp32 rounding;
* bf16 at Qwen2.5-0.5B width: within the bf16 rounding of one pass (the same bar as packed vs padded);
* actor.compute_log_prob: the same values whatever the row order of the groups in the batch.
"""

import pytest
import torch

from test_actor_update_gpu import _tiny

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C,dtype", [(64, torch.bfloat16), (1152, torch.bfloat16), (896, torch.float32)])
def test_sum_rows_matches_torch(C, dtype):
    from dots.rl_amd import native

    g = torch.Generator(device="cuda").manual_seed(C)
    src = torch.randn(500, C, device="cuda", generator=g).to(dtype)
    K, m = 5, 90
    idx = torch.randint(0, 500, (K, m), device="cuda", generator=g)
    idx[1:, ::7] = -1
    idx[3, 5::11] = -1
    dst_idx = torch.randperm(120, device="cuda", generator=g)[:m].contiguous()
    out = torch.full((120, C), 7.0, device="cuda", dtype=dtype)
    native.sum_rows(src, idx.contiguous(), out, dst_idx)
    want = torch.zeros(m, C, device="cuda")
    for k in range(K):  # fp32 accumulation in k order
        term = torch.where((idx[k] >= 0)[:, None], src[idx[k].clamp_min(0)].float(), torch.zeros((), device="cuda"))
        want = want + term
    assert torch.equal(out[dst_idx], want.to(dtype))
    rest = torch.ones(120, dtype=torch.bool, device="cuda")
    rest[dst_idx] = False
    assert torch.all(out[rest] == 7.0)


def _groups(prompts, n, P, R, V, seed, eos=2):
    """``prompts`` distinct left-padded prompts, each repeated n times (the trainer's repeat(n, interleave=True)),
    with per-row EOS-terminated responses and the rollout's positions / masks."""
    g = torch.Generator().manual_seed(seed)
    pid = torch.randint(3, V, (prompts, P), generator=g)
    pam = torch.ones(prompts, P, dtype=torch.int64)
    for p in range(prompts):
        lp = int(torch.randint(0, P - 2, (1,), generator=g))
        pam[p, :lp] = 0
        pid[p, :lp] = 0
    B = prompts * n
    resp = torch.randint(3, V, (B, R), generator=g)
    ram = torch.ones(B, R, dtype=torch.int64)
    for b in range(B):
        lr = int(torch.randint(1, R + 1, (1,), generator=g))
        if lr < R:
            resp[b, lr] = eos
            resp[b, lr + 1:] = 0
            ram[b, lr + 1:] = 0
    ids = torch.cat([pid.repeat_interleave(n, 0), resp], 1)
    am = torch.cat([pam.repeat_interleave(n, 0), ram], 1)
    pos = torch.clamp(torch.cumsum(am, -1) - 1, min=0)
    return ids.cuda(), am.cuda(), pos.cuda(), resp.cuda()


def test_prefix_share_maps_and_adjoints():
    from dots.rl_amd.qwen2 import PrefixShare, RmPad

    ids, am, pos, resp = _groups(3, 4, 10, 6, 50, 1)
    B, T = am.shape
    R = resp.shape[1]
    # rows in another order: groups are found by content, not by position
    perm = torch.tensor([0, 5, 9, 1, 4, 2, 10, 11, 3, 6, 7, 8], device="cuda")
    ids, am = ids[perm], am[perm]
    for keep_pads in (False, True):
        ps = PrefixShare.build(ids, am, R, keep_pads=keep_pads)
        assert ps is not None and ps.groups == 3
        S = T - R - 1
        leader = {}
        for b in range(B):
            leader.setdefault(tuple(ids[b, :S].tolist()), b)
        inv = ps.inv.view(B, T)
        for b in range(B):
            lb = leader[tuple(ids[b, :S].tolist())]
            for t in range(T):
                present = keep_pads or bool(am[b, t])
                if t < S:
                    assert inv[b, t].item() == (inv[lb, t].item() if present else -1)
                    if b != lb and present:
                        assert inv[b, t] >= 0
                else:
                    assert (inv[b, t].item() >= 0) == present
        own = (inv.reshape(-1)[ps.idx] == torch.arange(ps.nnz, device="cuda")).all()
        assert own
        # adjoint pairs
        g = torch.Generator(device="cuda").manual_seed(3)
        p = torch.randn(ps.nnz, 16, device="cuda", generator=g)
        y = torch.randn(B * T, 16, device="cuda", generator=g)
        lhs = (ps.unpack(p) * y).sum().double()
        rhs = (p * ps.pack_grad(y)).sum().double()
        assert torch.allclose(lhs, rhs, rtol=1e-5)
        x = torch.randn(B * T, 16, device="cuda", generator=g)
        q = torch.randn(ps.nnz, 16, device="cuda", generator=g)
        assert torch.allclose((ps.pack(x) * q).sum().double(), (x * ps.unpack_grad(q)).sum().double(), rtol=1e-5)
    # fewer tokens than RmPad packs: the copies are gone
    assert PrefixShare.build(ids, am, R).nnz < RmPad(am).nnz
    # no shared prompt: nothing to share
    assert PrefixShare.build(torch.randint(3, 50, (4, 16), device="cuda"), torch.ones(4, 16, device="cuda",
                                                                                      dtype=torch.int64), 6) is None


@pytest.mark.parametrize("rmpad", [False, True])
def test_fp32_prefix_share_matches_unshared(rmpad):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor

    cfg, store, model = _tiny()
    ids, am, pos, resp = _groups(3, 4, 24, 16, cfg.vocab_size, 5)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    res = {}
    for share in (False, True):
        actor = DataParallelPPOActor(to_attr({"use_remove_padding": rmpad, "share_prompt_prefix": share}), model)
        model.training = True
        store.zero_grad()
        ent, lp = actor._forward_micro_batch(mb, 1.0, calculate_entropy=True)
        ((lp - 0.01 * ent) * mask).sum().backward()
        res[share] = (lp.detach(), ent.detach(), store.grad.detach().clone())
    (lp0, e0, g0), (lp1, e1, g1) = res[False], res[True]
    torch.testing.assert_close(lp1[mask], lp0[mask], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1[mask], e0[mask], rtol=1e-5, atol=1e-5)
    if not rmpad:  # padded layout: the pad positions carry the padded forward's values, shared or not
        torch.testing.assert_close(lp1, lp0, rtol=1e-5, atol=1e-5)
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 2e-6, rel


def test_bf16_prefix_share_matches_unshared():
    """Qwen2.5-0.5B width, 2 layers, bf16 (drl_gemm, fused attention): shared vs unshared log-probs at the response
    mask and every parameter gradient of loss = sum(mask * logp) — the bar of packed vs padded (the two differ in
    GEMM row counts and in the bf16 rounding of the summed prompt gradients)."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config(vocab_size=4096, hidden_size=896, intermediate_size=4864, num_hidden_layers=2,
                      num_attention_heads=14, num_key_value_heads=2, tie_word_embeddings=True)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=True)
    store.init_random(7)
    model = Qwen2Model(cfg, store)
    ids, am, pos, resp = _groups(2, 4, 96, 64, cfg.vocab_size, 11)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    res = {}
    for share in (False, True):
        actor = DataParallelPPOActor(to_attr({"share_prompt_prefix": share}), model)
        model.training = True
        store.zero_grad()
        _, lp = actor._forward_micro_batch(mb, 1.0)
        (lp * mask).sum().backward()
        torch.cuda.synchronize()
        res[share] = (lp.detach().float(), store.grad.detach().clone())
    (lp0, g0), (lp1, g1) = res[False], res[True]
    torch.testing.assert_close(lp1[mask], lp0[mask], rtol=0, atol=0.05)
    assert (lp1 - lp0)[mask].abs().mean() < 5e-3
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 2e-2, rel


def test_bf16_prefix_share_skips_unread_q_rows(monkeypatch):
    """RoPE leaves the q rows of the copies' skipped query tiles unwritten (q_skip = q_start): poisoning q with NaN
    before RoPE, and RoPE without the skip, give bit-identical log-probs and gradients — no kernel reads those rows."""
    from dots.rl_amd import native
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config(vocab_size=4096, hidden_size=896, intermediate_size=4864, num_hidden_layers=2,
                      num_attention_heads=14, num_key_value_heads=2, tie_word_embeddings=True)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=True)
    store.init_random(5)
    model = Qwen2Model(cfg, store)
    ids, am, pos, resp = _groups(2, 4, 160, 64, cfg.vocab_size, 13)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    rope = native.rope_qkv_fwd
    seen = []

    def no_skip(*a, q_skip=None, **kw):
        return rope(*a, **kw)

    def poisoned(*a, q_skip=None, **kw):
        seen.append(q_skip is not None and bool((q_skip >= 32).any()))
        a[7].fill_(float("nan"))  # q
        return rope(*a, q_skip=q_skip, **kw)

    res = []
    for wrap in (no_skip, poisoned):
        monkeypatch.setattr(native, "rope_qkv_fwd", wrap)
        actor = DataParallelPPOActor(to_attr({"share_prompt_prefix": True}), model)
        model.training = True
        store.zero_grad()
        _, lp = actor._forward_micro_batch(mb, 1.0)
        (lp * mask).sum().backward()
        torch.cuda.synchronize()
        res.append((lp.detach().clone(), store.grad.detach().clone()))
    assert seen and all(seen)
    assert torch.equal(res[0][0], res[1][0]) and torch.isfinite(res[1][0][mask]).all()
    assert torch.equal(res[0][1], res[1][1])


def test_compute_log_prob_independent_of_group_row_order():
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.protocol import DataProto

    cfg, store, model = _tiny(trainable=False)
    ids, am, pos, resp = _groups(4, 4, 20, 12, cfg.vocab_size, 9)
    B = ids.shape[0]
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(1)).cuda()
    out = {}
    for name, order in (("grouped", torch.arange(B, device="cuda")), ("shuffled", perm)):
        data = DataProto.from_dict({"input_ids": ids[order], "attention_mask": am[order], "position_ids": pos[order],
                                    "responses": resp[order]},
                                   meta_info={"micro_batch_size": 8, "temperature": 1.0, "use_dynamic_bsz": False})
        actor = DataParallelPPOActor(to_attr({"exec_log_prob_tokens": 4096}), model)
        lp, _ = actor.compute_log_prob(data)
        out[name] = torch.empty_like(lp)
        out[name][order] = lp
    unshared = DataParallelPPOActor(to_attr({"share_prompt_prefix": False}), model)
    data = DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp},
                               meta_info={"micro_batch_size": 8, "temperature": 1.0, "use_dynamic_bsz": False})
    ref, _ = unshared.compute_log_prob(data)
    mask = am[:, -resp.shape[1]:].bool()
    for name in out:
        torch.testing.assert_close(out[name][mask], ref[mask], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("D,G", [(64, 7), (128, 4)])
def test_flash_q_start_skips_only_the_copies(D, G):
    """q_start: the skipped query tiles' outputs are never written and nothing of theirs is read — poisoned o / lse
    rows leave every other output bit-identical to the unskipped kernels, dq of the skipped rows is zero, and dk / dv
    equal the unskipped backward's with dout zero on those rows (their terms are exact zeros)."""
    from dots.rl_amd import native

    B, Hkv, T = 4, 2, 160
    g = torch.Generator(device="cuda").manual_seed(D)
    q = torch.randn(B, Hkv, G, T, D, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(B, Hkv, T, D, device="cuda", generator=g).to(torch.bfloat16)
    dout = torch.randn(B, T, Hkv * G * D, device="cuda", generator=g).to(torch.bfloat16)
    valid = torch.zeros(B, T, dtype=torch.uint8, device="cuda")
    valid[:, 5:] = 1
    kt = k.transpose(-1, -2).contiguous()
    vt = v.transpose(-1, -2).contiguous()
    qs = torch.tensor([0, 70, 64, 200], dtype=torch.int32, device="cuda")  # tiles below 64 / 64 / all skipped
    skip = torch.zeros(B, T, dtype=torch.bool, device="cuda")
    for b, s in enumerate(qs.tolist()):
        skip[b, : s // 32 * 32] = True
    dout = torch.where(skip[:, :, None], torch.zeros((), dtype=dout.dtype, device="cuda"), dout)
    o0 = torch.empty(B, T, Hkv * G * D, dtype=torch.bfloat16, device="cuda")
    l0 = torch.empty(B, Hkv, G, T, device="cuda")
    native.flash_attn_fwd(q, k, vt, valid, o0, lse=l0)
    o1 = torch.full_like(o0, float("nan"))
    l1 = torch.full_like(l0, float("nan"))
    native.flash_attn_fwd(q, k, vt, valid, o1, lse=l1, q_start=qs)
    assert torch.equal(o1[~skip], o0[~skip]) and torch.isnan(o1[skip]).all()
    lsk = skip[:, None, None, :].expand_as(l0)
    assert torch.equal(l1[~lsk], l0[~lsk])
    grads = []
    for o, lse, kw in ((o0, l0, {}), (o1, l1, {"q_start": qs})):
        dq = torch.full_like(q, float("nan"))
        dk, dv = torch.empty_like(k), torch.empty_like(v)
        native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv, **kw)
        grads.append((dq, dk, dv))
    (dq0, dk0, dv0), (dq1, dk1, dv1) = grads
    qsk = skip[:, None, None, :, None].expand_as(dq0)
    assert torch.equal(dq1[~qsk], dq0[~qsk]) and torch.all(dq1[qsk] == 0)
    assert torch.equal(dk1, dk0) and torch.equal(dv1, dv0)


def test_flash_packed_rows_equal_packing_the_padded_output():
    """drl_flash_attn_fwd_rows: each query written straight to its packed row equals the padded output packed
    afterwards, bit for bit; rows mapped to -1 (pads, shared copies) leave the packed buffer untouched."""
    from dots.rl_amd import native

    B, Hkv, G, D, T = 4, 2, 7, 64, 160
    g = torch.Generator(device="cuda").manual_seed(3)
    q = torch.randn(B, Hkv, G, T, D, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device="cuda", generator=g).to(torch.bfloat16)
    vt = torch.randn(B, Hkv, D, T, device="cuda", generator=g).to(torch.bfloat16)
    valid = torch.ones(B, T, dtype=torch.uint8, device="cuda")
    valid[1, :9] = 0
    valid[3, :40] = 0
    qs = torch.tensor([0, 70, 0, 64], dtype=torch.int32, device="cuda")
    own = valid.bool().clone()
    for b, s_ in enumerate(qs.tolist()):
        own[b, :s_] = False
    idx = torch.nonzero(own.reshape(-1)).reshape(-1)
    rows = torch.full((B * T,), -1, dtype=torch.int64, device="cuda")
    rows[idx] = torch.arange(idx.numel(), device="cuda")
    pad = torch.empty(B, T, Hkv * G * D, dtype=torch.bfloat16, device="cuda")
    native.flash_attn_fwd(q, k, vt, valid, pad, q_start=qs)
    packed = torch.full((idx.numel() + 3, Hkv * G * D), float("nan"), dtype=torch.bfloat16, device="cuda")
    native.flash_attn_fwd(q, k, vt, valid, packed, q_start=qs, out_rows=rows)
    assert torch.equal(packed[:idx.numel()], pad.reshape(B * T, -1)[idx])
    assert torch.isnan(packed[idx.numel():]).all()
    # the backward reading that packed O through the same map (dout zero at the unmapped rows, as unpack_grad
    # leaves it) equals the backward over the padded O, bit for bit
    lse = torch.empty(B, Hkv, G, T, device="cuda")
    native.flash_attn_fwd(q, k, vt, valid, pad, lse=lse, q_start=qs)
    packed = packed[:idx.numel()].contiguous()
    dout = torch.randn(B * T, Hkv * G * D, device="cuda", generator=g).to(torch.bfloat16)
    dout[rows < 0] = 0
    dout = dout.view(B, T, -1)
    kt = k.transpose(-1, -2).contiguous()
    v = vt.transpose(-1, -2).contiguous()
    res = []
    for o, kw in ((pad, {}), (packed, {"o_rows": rows})):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv, q_start=qs, **kw)
        res.append((dq, dk, dv))
    for a_, b_ in zip(*res):
        assert torch.equal(a_, b_)


def test_fp32_critic_prefix_share_matches_unshared():
    """The critic's values (dp_critic._forward_micro_batch) and its full gradient after a value loss, with and
    without prefix sharing, on the reference tiny critic: fp32 rounding."""
    from test_critic_gpu import _tiny_critic

    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_critic import DataParallelPPOCritic

    cfg, store, model = _tiny_critic()
    ids, am, pos, resp = _groups(3, 4, 24, 16, cfg.vocab_size, 13)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    target = torch.linspace(-1, 1, R, device="cuda")
    res = {}
    for share in (False, True):
        critic = DataParallelPPOCritic(to_attr({"model": {"share_prompt_prefix": share}}), model)
        model.training = True
        store.zero_grad()
        v = critic._forward_micro_batch(mb)
        (((v - target) ** 2) * mask).sum().backward()
        res[share] = (v.detach(), store.grad.detach().clone())
    (v0, g0), (v1, g1) = res[False], res[True]
    torch.testing.assert_close(v1, v0, rtol=1e-5, atol=1e-5)
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 2e-6, rel
