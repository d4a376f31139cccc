"""The PRODUCTION bf16 update path pinned to the reference at model level (VERDICT r03 "next" 1a).

Fixture ``bf16_update.npz`` (tests/golden/make_golden.py::gen_bf16_update): the reference's DataParallelPPOActor
(dp_actor.py:300-482, torch AdamW + clip_grad_norm_) on a Qwen2.5-0.5B-width model (H 896, 14 / 2 heads of 64,
I 4864, V 151936, tied lm_head, 4 layers; weights rebuilt here bit-identically from tests/golden/bf16_update.py)
over 16 left-padded, EOS-terminated sequences (48 + 48 tokens; 2 micro-batches of 8 in one mini-batch), run twice:
in fp32, and under the reference's own torch.autocast(bf16) (dp_actor.py:110, CPU autocast in the generator).

Here the same inputs go through this repository's bf16 path on the GPU — every projection, dgrad and wgrad on
drl_gemm (csrc/gemm_sk.hip) with the weight gradients concurrent with their input gradients, the fused flash
attention forward and backward (csrc/flash_attn.hip), K2 / K1, the HIP AdamW — in three forms: padded, remove-padding
(use_remove_padding) and the fused lm_head (use_fused_kernels: csrc/fused_linear.hip + the vocabulary-blocked
backward on drl_gemm).

The yardstick is the reference's own bf16-vs-fp32 difference, measured on the same inputs: for every compared
quantity q, |q_ours - q_fp32| <= 2 |q_ref_bf16 - q_fp32| + floor, with
  * log-probs / entropy over the response mask: max and mean absolute difference (floor 1e-3 / 1e-4);
  * each update metric, per micro-batch (floor: one sigma of the metric's random walk under the reference's own
    per-token bf16 log-prob error; clip fractions one token of the micro-batch; grad norm 1e-3 relative);
  * a fixed sample of each parameter's gradient elements (relative L2, floor 1e-3) and its gradient norm (relative;
    floor 1e-3 + 3 e / sqrt(n), the norm's sampling noise under the reference's own elementwise error e over n
    elements) — the gradient accumulated over both micro-batches, before clipping;
  * the AdamW update of the same sample: the fraction of elements moving the other way than in fp32 (floor 1e-3 +
    3 sigma of that fraction's binomial noise at the reference's rate over the sampled elements).
"""

import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import bf16_update as bu  # noqa: E402


_SD = {}


@pytest.fixture(scope="module", params=["bf16_update.npz", "bf16_update_grouped.npz"])
def fixture(request):
    """The fixture with 16 distinct prompts, and the grouped one (4 prompts x n = 4, interleaved as the trainer
    repeats them): there the default model.share_prompt_prefix runs each prompt once (qwen2.PrefixShare, flash
    q_start, drl_sum_rows) while the reference ran every row in full — the driver bench's production configuration
    under the same bar."""
    from conftest import load_golden

    z, meta = load_golden(request.param)
    if "sd" not in _SD:
        _SD["sd"] = bu.make_state_dict()
    sd = _SD["sd"]
    assert bu.checksum(sd) == meta["weight_checksum"]
    ref = bu.batch(grouped=bool(meta.get("grouped", False)))
    assert np.array_equal(ref["input_ids"].numpy(), z["input_ids"]), "fixture inputs differ from bf16_update.batch()"
    return z, meta, sd


def _hf_view(store, flat, hf_name):
    """The HF-named parameter ``hf_name`` as a view of one of the store's flat buffers (fused layouts split)."""
    cfg = store.cfg
    H, I = cfg.hidden_size, cfg.intermediate_size
    nq, nkv = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim

    def v(name):
        o, shape, _ = store.offsets[name]
        return flat[o:o + int(np.prod(shape))].view(shape)

    if hf_name == "model.embed_tokens.weight":
        return v("embed_tokens")
    if hf_name == "model.norm.weight":
        return v("norm")
    parts = hf_name.split(".")
    p = f"layers.{parts[2]}."
    mod = parts[-2]
    if mod in ("input_layernorm", "post_attention_layernorm"):
        return v(p + mod)
    if mod in ("q_proj", "k_proj", "v_proj"):
        t = v(p + ("qkv_proj.bias" if parts[-1] == "bias" else "qkv_proj.weight"))
        a, b = {"q_proj": (0, nq), "k_proj": (nq, nq + nkv), "v_proj": (nq + nkv, nq + 2 * nkv)}[mod]
        return t[a:b]
    if mod == "o_proj":
        return v(p + "o_proj")
    if mod == "down_proj":
        return v(p + "down_proj")
    gu = v(p + "gate_up_proj")
    return gu[:I] if mod == "gate_proj" else gu[I:]


def _run(z, meta, sd, extra):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor, FlatAdamW
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(bu.CFG)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=True)
    store.load_state_dict_hf(sd)
    model = Qwen2Model(cfg, store)
    acfg = to_attr(dict(meta["config"], **extra))
    opt = FlatAdamW(store, lr=meta["lr"], betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                    max_grad_norm=acfg.grad_clip)
    grads = {}
    step0 = opt.step

    def step():
        grads["flat"] = store.grad.detach().clone()
        return step0()

    opt.step = step
    actor = DataParallelPPOActor(acfg, model, opt)
    T = lambda k: torch.from_numpy(np.ascontiguousarray(z[k])).cuda()  # noqa: E731
    # the grouped fixture must take the prefix-sharing path (and the other one must not)
    from dots.rl_amd.qwen2 import PrefixShare

    assert actor.share_prompt_prefix
    sh = PrefixShare.build(T("input_ids")[:bu.B // 2], T("attention_mask")[:bu.B // 2], bu.R,
                           keep_pads=not acfg.get("use_remove_padding", False))
    assert (sh is not None) == bool(meta.get("grouped", False)), "prefix sharing engaged on the wrong fixture"
    data = DataProto.from_dict({k: T(k) for k in ("input_ids", "attention_mask", "position_ids", "responses")},
                               meta_info={"micro_batch_size": bu.B // 2, "temperature": 1.0, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    before = store.master.detach().clone()
    udata = DataProto.from_dict({k: T(k) for k in ("input_ids", "attention_mask", "position_ids", "responses",
                                                   "response_mask", "advantages", "old_log_probs", "ref_log_prob")},
                                meta_info={"temperature": 1.0})
    metrics = actor.update_policy(udata)
    assert "flat" in grads, "the optimizer never stepped"
    return store, lp.cpu().numpy(), ent.cpu().numpy(), metrics, grads["flat"], before


_FAILS = []


def _within(name, ours, bf16, fp32, floor):
    """Record one comparison (printed; the test asserts after all of them, so one run shows every quantity)."""
    e_ours, e_ref = abs(ours - fp32), abs(bf16 - fp32)
    ok = e_ours <= 2 * e_ref + floor
    line = f"{'ok ' if ok else 'BAD'} {name}: ours {float(ours):.6g} vs fp32 {float(fp32):.6g} (|d| {e_ours:.3g}); " \
           f"reference bf16 {float(bf16):.6g} (|d| {e_ref:.3g}), floor {floor:.3g}"
    print(line)
    if not ok:
        _FAILS.append(line)


@pytest.mark.parametrize("form", ["padded", "rmpad", "fused_lm_head"])
def test_bf16_update_within_reference_bf16_error(fixture, form):
    z, meta, sd = fixture
    extra = {"padded": {}, "rmpad": {"use_remove_padding": True}, "fused_lm_head": {"use_fused_kernels": True}}[form]
    store, lp, ent, metrics, gflat, before = _run(z, meta, sd, extra)
    m = z["response_mask"].astype(bool)
    _FAILS.clear()

    # log-probs / entropy of the bf16 model
    for key, got in (("log_probs", lp), ("entropys", ent)):
        f32, b16 = z[f"fp32_{key}"][m], z[f"bf16_{key}"][m]
        _within(f"{key} max", np.abs(got[m] - f32).max(), np.abs(b16 - f32).max(), 0.0, 1e-3)
        _within(f"{key} mean", np.abs(got[m] - f32).mean(), np.abs(b16 - f32).mean(), 0.0, 1e-4)

    # update metrics, per micro-batch. A metric is one token-mean: its bf16-vs-fp32 difference is a sum of per-token
    # errors of both signs, so one realisation of it can cancel by chance. The floor is one sigma of that random
    # walk, built from the reference's OWN per-token bf16 log-prob error d_t and the metric's derivative f'_t per
    # token: sqrt(sum_t (f'_t d_t)^2) / n_tokens (one token of the micro-batch for the clip fractions)
    runs = meta["runs"]
    cfg = meta["config"]
    ntok = m.reshape(2, -1).sum(1)
    lp32 = z["fp32_log_probs"].astype(np.float64)
    dlt = (z["bf16_log_probs"].astype(np.float64) - lp32) * m
    old, ref, adv = (z[k].astype(np.float64) for k in ("old_log_probs", "ref_log_prob", "advantages"))
    ratio = np.exp(lp32 - old)
    lo, hi = 1 - cfg["clip_ratio_low"], 1 + cfg["clip_ratio_high"]
    unclipped = (-adv * ratio) >= (-adv * np.clip(ratio, lo, hi))  # the max() takes the unclipped branch
    deriv = {"actor/pg_loss": np.where(unclipped, -adv * ratio, 0.0), "actor/ppo_kl": -np.ones_like(lp32),
             "actor/kl_loss": 1.0 - np.exp(ref - lp32)}  # low_var_kl: exp(ref - lp) - (ref - lp) - 1

    def noise(k, i):
        rows = slice(i * (bu.B // 2), (i + 1) * (bu.B // 2))
        if "clipfrac" in k:
            return 1.0 / ntok[i]
        if k not in deriv:
            return 1e-5 + 1e-3 * abs(np.asarray(runs["fp32"]["metrics"][k], np.float64).reshape(-1)[i])
        return np.sqrt(((deriv[k][rows] * dlt[rows]) ** 2).sum()) / ntok[i]

    for k, want in runs["fp32"]["metrics"].items():
        got = np.asarray(metrics[k], np.float64).reshape(-1)
        w32, w16 = np.asarray(want, np.float64), np.asarray(runs["bf16"]["metrics"][k], np.float64)
        assert got.shape == w32.shape, (k, got.shape, w32.shape)
        for i in range(len(w32)):
            _within(f"{k}[{i}]", got[i], w16[i], w32[i], noise(k, i) if k != "actor/grad_norm" else 1e-3 * w32[i])

    # gradients (before clipping) and the AdamW update, per parameter
    embed_idx = bu.embed_rows_index(z["input_ids"])
    for n, gn32 in runs["fp32"]["grad_norms"].items():
        gv = _hf_view(store, gflat, n).reshape(-1)
        gn16 = runs["bf16"]["grad_norms"][n]
        idx = torch.from_numpy(embed_idx if n == "model.embed_tokens.weight" else bu.sample_index(n, gv.numel()))
        s32, s16 = z[f"fp32_grad.{n}"].astype(np.float64), z[f"bf16_grad.{n}"].astype(np.float64)
        sg = gv[idx.cuda()].double().cpu().numpy()
        nrm = np.linalg.norm(s32) + 1e-30
        e16 = np.linalg.norm(s16 - s32) / nrm
        _within(f"grad sample {n} (relative L2)", np.linalg.norm(sg - s32) / nrm, e16, 0.0, 1e-3)
        # the norm is one scalar of the tensor: elementwise errors of relative size e move it by ~e / sqrt(n) at
        # random (n elements), so a small tensor (a 128-element bias) gets that sampling noise as its floor (3 sigma)
        _within(f"grad norm {n} (relative)", gv.double().norm().item() / gn32, gn16 / gn32, 1.0,
                1e-3 + 3.0 * e16 / np.sqrt(gv.numel()))
        # diagnostics: least-squares scale of each gradient sample against fp32 (1 = no systematic shrink / growth)
        print(f"    scale {n}: ours {float(sg @ s32) / nrm ** 2:.5f}  reference bf16 {float(s16 @ s32) / nrm ** 2:.5f}")
        d = (_hf_view(store, store.master, n) - _hf_view(store, before, n)).reshape(-1)[idx.cuda()].double()
        d = d.cpu().numpy()
        d32, d16 = z[f"fp32_delta.{n}"], z[f"bf16_delta.{n}"]
        flip = lambda a: float(np.mean(np.sign(a) != np.sign(d32)))  # noqa: E731
        nn_ = d32.size  # binomial noise of a flip fraction over n sampled elements (3 sigma at the reference's rate)
        _within(f"update direction {n} (flipped fraction)", flip(d), flip(d16), 0.0,
                1e-3 + 3.0 * np.sqrt(max(flip(d16), 1.0 / nn_) / nn_))
    assert not _FAILS, "\n".join(_FAILS)
