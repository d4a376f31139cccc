"""Remove-padding (varlen) passes — the reference's use_remove_padding=True path (dp_actor.py:119-247,
dp_critic.py:69-107: unpad_input -> packed forward -> pad_input) — on MI355X.

The backbone's norms, GEMMs and MLP run on the nnz attended tokens only (qwen2.RmPad, csrc/rows.hip row gathers /
scatters); RoPE + attention keep the padded layout. Checks:

* the row gather / scatter kernel vs torch indexing (bit-exact, both directions, -1 skips);
* the reference-pinned fp32 actor update (tests/golden/actor_update.npz: left-padded prompts, EOS-terminated
  responses) with use_remove_padding=True: log-probs / entropy at the response-mask positions and 0 at pad
  positions (pad_input), then update_policy's metrics and the post-update parameters under the same tolerances as
  test_actor_update_gpu.py (the loss only reads response-mask positions, so the padded fixture pins it);
* the reference tiny critic (tests/golden/tiny_critic.npz): values under the mask and the gradients after the value
  loss, through the packed path;
* bf16: packed vs padded log-probs and the full-model gradient after the same loss (the two differ only in GEMM
  row counts, i.e. split-K / tile order): within the bf16 rounding of one pass;
* a GAE PPO step with model.use_remove_padding on actor, ref and critic.
"""

import json
import os

import numpy as np
import pytest
import torch

from test_actor_update_gpu import T, TINY, _check_params, _fixture, _metric_lists_close, _tiny

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C,dtype", [(64, torch.bfloat16), (896, torch.bfloat16), (1152, torch.float32)])
def test_copy_rows_matches_indexing(C, dtype):
    from dots.rl_amd import native

    g = torch.Generator(device="cuda").manual_seed(C)
    src = torch.randn(300, C, device="cuda", generator=g).to(dtype)
    idx = torch.randperm(300, device="cuda", generator=g)[:200].contiguous()
    idx[::7] = -1
    out = torch.full((200, C), 3.0, device="cuda", dtype=dtype)
    native.copy_rows(src, out, src_idx=idx)
    keep = idx >= 0
    assert torch.equal(out[keep], src[idx[keep]])
    assert torch.all(out[~keep] == 3.0)
    dst = torch.zeros(300, C, device="cuda", dtype=dtype)
    native.copy_rows(out, dst, dst_idx=idx)
    assert torch.equal(dst[idx[keep]], out[keep])
    rest = torch.ones(300, dtype=torch.bool, device="cuda")
    rest[idx[keep]] = False
    assert torch.all(dst[rest] == 0)
    # strided rows (a column slice of a wider tensor)
    wide = torch.randn(50, C + 64, device="cuda", generator=g).to(dtype)
    o2 = torch.empty(50, C, device="cuda", dtype=dtype)
    native.copy_rows(wide[:, :C], o2)
    assert torch.equal(o2, wide[:, :C])
    # the zero-filling gather (drl_gather_rows): every destination row written, zeros where the index is negative,
    # whatever the destination held (NaN here)
    o3 = torch.full((200, C), float("nan"), device="cuda", dtype=dtype)
    native.gather_rows_zero(src, o3, idx)
    assert torch.equal(o3[keep], src[idx[keep]])
    assert torch.all(o3[~keep] == 0)
    o4 = torch.full((50, C), float("nan"), device="cuda", dtype=dtype)
    native.gather_rows_zero(wide[:, :C], o4, torch.arange(50, device="cuda"))
    assert torch.equal(o4, wide[:, :C])


def test_rmpad_maps():
    from dots.rl_amd.qwen2 import RmPad

    am = torch.tensor([[0, 0, 1, 1, 1], [1, 1, 1, 0, 0], [1, 1, 1, 1, 1]], device="cuda")
    rm = RmPad(am)
    assert rm.nnz == 11
    assert rm.idx.tolist() == [2, 3, 4, 5, 6, 7, 10, 11, 12, 13, 14]
    inv = rm.inv.tolist()
    assert inv[:5] == [-1, -1, 0, 1, 2] and inv[8:10] == [-1, -1]
    x = torch.arange(15 * 8, dtype=torch.float32, device="cuda").view(15, 8)
    p = rm.pack(x)
    assert torch.equal(p, x[rm.idx])
    u = rm.unpack(p)
    assert torch.equal(u[rm.idx], p) and torch.all(u[am.reshape(-1) == 0] == 0)


@pytest.mark.parametrize("ci", [0, 1])
def test_update_policy_rmpad_matches_reference(ci):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor, FlatAdamW
    from dots.rl_amd.protocol import DataProto

    z, meta = _fixture("actor_update.npz")
    case = meta["cases"][ci]
    c = lambda k: T(z[f"c{ci}_{k}"])  # noqa: E731
    cfg, store, model = _tiny()
    before = store.master.detach().cpu().clone()
    acfg = to_attr(dict(case["config"], use_remove_padding=True, exec_micro_batches=0))
    opt = FlatAdamW(store, lr=case["lr"], betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                    max_grad_norm=acfg.grad_clip)
    actor = DataParallelPPOActor(acfg, model, opt)
    assert actor.use_remove_padding
    data = DataProto.from_dict({k: c(k) for k in ("input_ids", "attention_mask", "position_ids", "responses")},
                               meta_info={"micro_batch_size": 4, "temperature": 1.0, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    R = z[f"c{ci}_responses"].shape[1]
    mask = z[f"c{ci}_response_mask"].astype(bool)
    pad = z[f"c{ci}_attention_mask"][:, -R - 1:-1] == 0  # predicting positions that are pads -> exactly 0
    lp, ent = lp.cpu().numpy(), ent.cpu().numpy()
    np.testing.assert_allclose(lp[mask], z[f"c{ci}_log_probs"][mask], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ent[mask], z[f"c{ci}_entropys"][mask], rtol=1e-4, atol=1e-4)
    assert pad.any() and np.all(lp[pad] == 0) and np.all(ent[pad] == 0)
    udata = DataProto.from_dict({k: c(k) for k in ("input_ids", "attention_mask", "position_ids", "responses",
                                                   "response_mask", "old_log_probs", "advantages", "ref_log_prob")},
                                meta_info={"temperature": 1.0})
    metrics = actor.update_policy(udata)
    _metric_lists_close(metrics, case["metrics"])
    _check_params(cfg, store, before, z, f"c{ci}_", case["param_sums"])


def test_tiny_critic_rmpad_matches_reference(golden):
    from test_critic_gpu import _tiny_critic

    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_critic import DataParallelPPOCritic, fused_value_loss

    zr, _ = golden("tiny_qwen2_rollout.npz")
    z, meta = golden("tiny_critic.npz")
    cfg, store, model = _tiny_critic()
    critic = DataParallelPPOCritic(to_attr({"model": {"use_remove_padding": True}}), model)
    assert critic.use_remove_padding
    R = zr["responses"].shape[1]
    mb = {"input_ids": T(zr["sequences"]), "attention_mask": T(zr["attention_mask"]),
          "position_ids": T(zr["position_ids"]), "responses": T(zr["responses"])}
    mask = zr["attention_mask"][:, -R:].astype(bool)
    with torch.no_grad():
        v = critic._forward_micro_batch(mb).cpu().numpy()
    np.testing.assert_allclose(v[mask], z["vpreds"][mask], rtol=1e-4, atol=1e-5)
    assert np.all(v[zr["attention_mask"][:, -R - 1:-1] == 0] == 0)
    model.training = True
    store.zero_grad()
    vp = critic._forward_micro_batch(mb)
    out = fused_value_loss(vp, T(z["values"]), T(z["returns"]), T(zr["attention_mask"][:, -R:]),
                           cliprange_value=meta["cliprange_value"], loss_agg_mode=meta["loss_agg_mode"],
                           loss_scale_factor=meta["loss_scale_factor"])
    out[3].backward()
    np.testing.assert_allclose(out[0].item(), z["vf_loss"], rtol=1e-5)
    g = lambda n: store.g(n).detach().cpu().numpy()  # noqa: E731
    for name, key in [("score.weight", "d_score_weight"), ("score.bias", "d_score_bias"), ("norm", "d_norm"),
                      ("layers.0.input_layernorm", "d_input_layernorm0")]:
        ref = z[key].reshape(g(name).shape)
        np.testing.assert_allclose(g(name), ref, rtol=2e-4, atol=2e-4 * np.abs(ref).max(), err_msg=name)
    emb = np.linalg.norm(g("embed_tokens"), axis=-1)
    np.testing.assert_allclose(emb, z["d_embed_rows"], rtol=2e-4, atol=2e-4 * z["d_embed_rows"].max())


def _ragged_batch(B, P, R, V, seed):
    """Left-padded prompts and EOS-terminated responses (random lengths), with the rollout's positions."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (B, P + R), generator=g)
    am = torch.ones(B, P + R, dtype=torch.int64)
    for b in range(B):
        lp = int(torch.randint(0, P - 1, (1,), generator=g))
        lr = int(torch.randint(1, R + 1, (1,), generator=g))
        am[b, :lp] = 0
        am[b, P + lr:] = 0
    pos = torch.clamp(torch.cumsum(am, -1) - 1, min=0)
    return ids.cuda(), am.cuda(), pos.cuda(), ids[:, P:].contiguous().cuda()


def test_bf16_rmpad_matches_padded_forward_and_gradient():
    """qwen2.5-0.5b width (H 896, 14 / 2 heads), 2 layers, bf16: packed vs padded log-probs at the response mask
    and every parameter gradient of loss = sum(mask * logp)."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config(vocab_size=4096, hidden_size=896, intermediate_size=4864, num_hidden_layers=2,
                      num_attention_heads=14, num_key_value_heads=2, tie_word_embeddings=True)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=True)
    store.init_random(7)
    model = Qwen2Model(cfg, store)
    ids, am, pos, resp = _ragged_batch(6, 96, 64, cfg.vocab_size, 11)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    res = {}
    for rmpad in (False, True):
        for fused in (False, True):
            actor = DataParallelPPOActor(to_attr({"use_remove_padding": rmpad, "use_fused_kernels": fused}), model)
            model.training = True
            store.zero_grad()
            _, lp = actor._forward_micro_batch(mb, 1.0)
            (lp * mask).sum().backward()
            torch.cuda.synchronize()
            res[rmpad, fused] = (lp.detach().float(), store.grad.detach().clone())
    for fused in (False, True):
        lp0, g0 = res[False, fused]
        lp1, g1 = res[True, fused]
        torch.testing.assert_close(lp1[mask], lp0[mask], rtol=0, atol=0.05)
        assert (lp1 - lp0)[mask].abs().mean() < 5e-3
        rel = (g1 - g0).norm() / g0.norm()
        assert rel < 2e-2, (fused, rel.item())
        assert torch.all(lp1[am[:, -R - 1:-1] == 0] == 0)


def test_fp32_rmpad_matches_padded():
    """fp32 tiny Qwen2 (reference weights): packed vs padded log-probs / entropy and the full gradient. The two
    differ only in the fp32 GEMMs' row counts (library kernel choice), so the bar is fp32 rounding: 2e-6 relative
    on the gradient, 1e-5 on log-probs."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor

    cfg, store, model = _tiny()
    ids, am, pos, resp = _ragged_batch(8, 40, 24, cfg.vocab_size, 5)
    R = resp.shape[1]
    mask = am[:, -R:].bool()
    mb = {"input_ids": ids, "attention_mask": am, "position_ids": pos, "responses": resp}
    res = {}
    for rmpad in (False, True):
        actor = DataParallelPPOActor(to_attr({"use_remove_padding": rmpad}), model)
        model.training = True
        store.zero_grad()
        ent, lp = actor._forward_micro_batch(mb, 1.0, calculate_entropy=True)
        ((lp - 0.01 * ent) * mask).sum().backward()
        res[rmpad] = (lp.detach(), ent.detach(), store.grad.detach().clone())
    (lp0, e0, g0), (lp1, e1, g1) = res[False], res[True]
    torch.testing.assert_close(lp1[mask], lp0[mask], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(e1[mask], e0[mask], rtol=1e-5, atol=1e-5)
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-6


def test_gae_step_with_remove_padding():
    from dots.rl_amd.config import apply_overrides, default_config
    from dots.rl_amd.trainer import RayPPOTrainer

    tiny = ("{'hidden_size': 128, 'intermediate_size': 256, 'num_hidden_layers': 2, 'num_attention_heads': 2, "
            "'num_key_value_heads': 1, 'vocab_size': 1024}")
    cfg = apply_overrides(default_config(), [
        "data.train_batch_size=4", "data.max_prompt_length=32", "data.max_response_length=16",
        "actor_rollout_ref.rollout.n=2", "actor_rollout_ref.rollout.response_length=16",
        "actor_rollout_ref.rollout.prompt_length=32", "actor_rollout_ref.actor.ppo_mini_batch_size=2",
        "actor_rollout_ref.actor.ppo_micro_batch_size_per_gpu=2",
        "actor_rollout_ref.rollout.log_prob_micro_batch_size_per_gpu=4",
        "actor_rollout_ref.ref.log_prob_micro_batch_size_per_gpu=4", "critic.ppo_micro_batch_size_per_gpu=2",
        "critic.forward_micro_batch_size_per_gpu=4", "algorithm.adv_estimator=gae",
        "actor_rollout_ref.model.use_remove_padding=True", "critic.model.use_remove_padding=True",
        f"actor_rollout_ref.model.override_config={tiny}", f"critic.model.override_config={tiny}",
    ])
    trainer = RayPPOTrainer(cfg)
    trainer.train_dataloader.vocab_limit = 1000
    trainer.init_workers()
    w = trainer.actor_rollout_wg.worker
    assert w.actor.use_remove_padding and w.ref_policy.use_remove_padding
    m = trainer.fit(num_steps=1)[-1]
    for k in ["critic/vf_loss", "actor/pg_loss", "actor/kl_loss", "critic/grad_norm", "actor/grad_norm"]:
        assert k in m and np.isfinite(m[k]), k


@pytest.mark.parametrize("dtype,heads", [(torch.bfloat16, True), (torch.float32, False)])
def test_rope_reads_packed_rows_like_the_padded_copy(dtype, heads):
    """drl_rope_qkv_fwd_rows (RoPE straight from the packed qkv through the inverse map, zeros at pads) equals RoPE on
    the padded copy pad_input would build, bit for bit: the tiled kernel with head-dim-major copies (bf16) and the
    generic one (fp32, no copies)."""
    from dots.rl_amd import native

    B, T, Hq, Hkv, D = 3, 40, 4, 2, 64
    C = (Hq + 2 * Hkv) * D
    g = torch.Generator(device="cuda").manual_seed(7)
    am = torch.ones(B, T, dtype=torch.int64, device="cuda")
    am[1, :9] = 0
    am[2, :23] = 0
    idx = torch.nonzero(am.reshape(-1)).reshape(-1)
    inv = torch.full((B * T,), -1, dtype=torch.int64, device="cuda")
    inv[idx] = torch.arange(idx.numel(), device="cuda")
    packed = torch.randn(idx.numel(), C, device="cuda", generator=g).to(dtype)
    padded = torch.zeros(B * T, C, device="cuda", dtype=dtype)
    padded[idx] = packed
    pos = (am.cumsum(-1) - 1).clamp_min(0).contiguous()
    cos = torch.randn(64, D // 2, device="cuda", generator=g)
    sin = torch.randn(64, D // 2, device="cuda", generator=g)
    outs = []
    for src, rows in ((padded.view(B, T, C), None), (packed, inv)):
        q = torch.full((B, Hkv, Hq // Hkv, T, D), float("nan"), device="cuda", dtype=dtype)
        k = torch.full((B, Hkv, T, D), float("nan"), device="cuda", dtype=dtype)
        v = torch.full_like(k, float("nan"))
        kt = torch.full((B, Hkv, D, T), float("nan"), device="cuda", dtype=dtype) if heads else None
        vt = torch.full_like(kt, float("nan")) if heads else None
        native.rope_qkv_fwd(src, pos, cos, sin, Hq, Hkv, D, q, k, v, kt=kt, vt=vt, src_rows=rows)
        outs.append([t for t in (q, k, v, kt, vt) if t is not None])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype,heads", [(torch.bfloat16, True), (torch.float32, False)])
def test_rope_q_skip_leaves_only_the_skipped_q_rows(dtype, heads):
    """q_skip (prefix sharing's q_start): q rows t < q_skip[b] & ~31 are left as they were, every other q row and all
    of k / v / kt / vt are bit-identical to the unskipped kernel — the tiled kernel (whole 64-row tiles skipped, the
    rest of a partial tile written) and the generic one (per row)."""
    from dots.rl_amd import native

    B, T, Hq, Hkv, D = 4, 200, 4, 2, 64
    C = (Hq + 2 * Hkv) * D
    g = torch.Generator(device="cuda").manual_seed(11)
    qkv = torch.randn(B, T, C, device="cuda", generator=g).to(dtype)
    pos = torch.arange(T, device="cuda").repeat(B, 1).contiguous()
    cos = torch.randn(T, D // 2, device="cuda", generator=g)
    sin = torch.randn(T, D // 2, device="cuda", generator=g)
    qs = torch.tensor([0, 150, 70, 500], dtype=torch.int32, device="cuda")
    outs = []
    for skip in (None, qs):
        q = torch.full((B, Hkv, Hq // Hkv, T, D), float("nan"), device="cuda", dtype=dtype)
        k = torch.full((B, Hkv, T, D), float("nan"), device="cuda", dtype=dtype)
        v = torch.full_like(k, float("nan"))
        kt = torch.full((B, Hkv, D, T), float("nan"), device="cuda", dtype=dtype) if heads else None
        vt = torch.full_like(kt, float("nan")) if heads else None
        native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q, k, v, kt=kt, vt=vt, q_skip=skip)
        outs.append([t for t in (q, k, v, kt, vt) if t is not None])
    (q0, *rest0), (q1, *rest1) = outs
    for a, b in zip(rest0, rest1):
        assert torch.equal(a, b)
    skipped = torch.zeros(B, T, dtype=torch.bool, device="cuda")
    for b, s in enumerate(qs.tolist()):
        skipped[b, : min(s // 32 * 32, T)] = True
    sk = skipped[:, None, None, :, None].expand_as(q0)
    assert torch.equal(q1[~sk], q0[~sk])
    # what was skipped: all of it (generic kernel) or whole 64-row tiles (tiled), never a row past the bound
    untouched = torch.isnan(q1).all(-1).all(2).all(1)  # (B, T)
    assert not (untouched & ~skipped).any()
    tile = 1 if not heads else 64
    for b, s in enumerate(qs.tolist()):
        lo = min(s // 32 * 32, T) // tile * tile
        assert untouched[b, :lo].all()


@pytest.mark.parametrize("rmpad,share", [(False, False), (True, False), (True, True), (False, True)])
def test_bf16_sequence_length_not_multiple_of_8(rmpad, share):
    """T = P + R with T % 8 != 0 (R = 61, as max_response_length 250 would give): the reference actor takes any T
    (dp_actor.py:90-280); the fused attention needs T % 8 == 0, so _forward_micro_batch right-pads the micro-batch's
    columns (qwen2.pad_seq_columns) and slices the response rows at the original T. Against the same batch with
    three more response columns that are already pads (R = 64, T % 8 == 0): the log-probs of the first 61 columns and
    the gradient of loss = sum(mask * logp) agree up to summation order; prefix sharing (3 rows per prompt) too."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config(vocab_size=4096, hidden_size=896, intermediate_size=4864, num_hidden_layers=2,
                      num_attention_heads=14, num_key_value_heads=2, tie_word_embeddings=True)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=True)
    store.init_random(3)
    model = Qwen2Model(cfg, store)
    P, R = 96, 61
    ids, am, pos, _ = _ragged_batch(6, P, 64, cfg.vocab_size, 17)
    am[:, P + R:] = 0  # the last three response columns are pads in every row
    if share:  # two prompt groups of three rows
        for lead in (0, 3):
            ids[lead + 1:lead + 3, :P] = ids[lead, :P]
            am[lead + 1:lead + 3, :P] = am[lead, :P]
        pos = torch.clamp(torch.cumsum(am, -1) - 1, min=0)
    res = {}
    for r in (R, 64):
        mb = {"input_ids": ids[:, :P + r].contiguous(), "attention_mask": am[:, :P + r].contiguous(),
              "position_ids": pos[:, :P + r].contiguous(), "responses": ids[:, P:P + r].contiguous()}
        actor = DataParallelPPOActor(to_attr({"use_remove_padding": rmpad, "share_prompt_prefix": share}), model)
        model.training = True
        store.zero_grad()
        _, lp = actor._forward_micro_batch(mb, 1.0)
        (lp[:, :R] * am[:, P:P + R]).sum().backward()
        torch.cuda.synchronize()
        res[r] = (lp[:, :R].detach().float(), store.grad.detach().clone())
    (lp0, g0), (lp1, g1) = res[R], res[64]
    mask = am[:, P:P + R].bool()
    torch.testing.assert_close(lp0[mask], lp1[mask], rtol=0, atol=1e-2)
    assert ((g0 - g1).norm() / g1.norm()).item() < 1e-3
