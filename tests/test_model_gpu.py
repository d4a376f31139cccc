"""Model-level parity of the HIP-kernel Qwen2 (rollout A3, log-prob A6/A7, backward A14) on MI355X.

* greedy rollout of a tiny random Qwen2 (fp32 mode) vs HF ``generate`` post-processed as HFRollout
  (golden: tests/golden/tiny_qwen2_rollout.npz) — token ids, masks and positions bit-exact;
* teacher-forced log-probs / entropy vs the reference's logprobs_from_logits / entropy_from_logits on
  HF logits — within 1e-4 (fp32);
* the hand-written layer backward vs torch autograd through ``oracle.qwen2_ref`` (plain fp32 torch
  restatement of the HF math, pinned on CPU by test_oracle_golden.py) — flat gradients within 2e-4 relative;
* the HIP-graph decode loop replays exactly the eager loop (greedy and sampled);
* the bf16 production mode tracks the fp32 model (loose bf16 tolerance).
"""

import json
import os

import numpy as np
import pytest
import torch

from oracle import qwen2_ref

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "golden", "tiny_qwen2")


def build(dtype=torch.float32, trainable=True):
    from safetensors.torch import load_file

    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(json.load(open(os.path.join(TINY, "config.json"))))
    if dtype == torch.bfloat16 and cfg.head_dim not in (64, 128):
        cfg.attn_implementation = "eager"  # head_dim 16: the fused attention kernels take 64 / 128
    store = ParamStore(cfg, "cuda", compute_dtype=dtype, trainable=trainable)
    store.load_state_dict_hf(load_file(os.path.join(TINY, "model.safetensors")))
    return cfg, store, Qwen2Model(cfg, store)


def golden():
    z = np.load(os.path.join(HERE, "golden", "tiny_qwen2_rollout.npz"), allow_pickle=False)
    return z, json.loads(str(z["__meta__"]))


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("use_hip_graph", [True, False])
def test_greedy_rollout_matches_hf_bit_exact(use_hip_graph):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    z, meta = golden()
    cfg, store, model = build()
    rcfg = to_attr(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0, response_length=meta["response_length"],
                        ignore_eos=False, seed=0, val_kwargs={}, use_hip_graph=use_hip_graph))
    ro = MI355XRollout(model, rcfg)
    prompts = DataProto.from_dict({"input_ids": T(z["prompt_ids"]), "attention_mask": T(z["prompt_attention_mask"]),
                                   "position_ids": T(z["prompt_position_ids"])},
                                  meta_info={"eos_token_id": meta["eos_token_id"], "pad_token_id": meta["pad_token_id"]})
    out = ro.generate_sequences(prompts)
    for k, ref in [("input_ids", "sequences"), ("responses", "responses"), ("attention_mask", "attention_mask"),
                   ("position_ids", "position_ids")]:
        np.testing.assert_array_equal(out.batch[k].cpu().numpy(), z[ref], err_msg=k)
    np.testing.assert_array_equal(out.batch["prompts"].cpu().numpy(), z["prompt_ids"])


def test_graphed_sampling_rollout_equals_eager():
    """bf16 temperature sampling: the HIP-graph decode loop replays exactly the eager loop's kernels, so the
    sampled responses (Philox stream indexed by step) must be identical."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    z, meta = golden()
    cfg, store, model = build(torch.bfloat16, trainable=False)
    outs = []
    for g in (True, False):
        rcfg = to_attr(dict(do_sample=True, temperature=0.9, top_k=-1, top_p=1.0, response_length=24, ignore_eos=False,
                            seed=3, val_kwargs={}, use_hip_graph=g))
        prompts = DataProto.from_dict({"input_ids": T(z["prompt_ids"]), "attention_mask": T(z["prompt_attention_mask"]),
                                       "position_ids": T(z["prompt_position_ids"])},
                                      meta_info={"eos_token_id": meta["eos_token_id"], "pad_token_id": meta["pad_token_id"]})
        outs.append(MI355XRollout(model, rcfg).generate_sequences(prompts))
    for k in ("responses", "attention_mask", "position_ids"):
        assert torch.equal(outs[0].batch[k], outs[1].batch[k]), k
    assert len(set(outs[0].batch["responses"].flatten().tolist())) > 20  # actually sampled
    # top-k / top-p sampling (per-row cut kernel) replays identically from the graph
    tk = []
    for g in (True, False):
        rcfg = to_attr(dict(do_sample=True, temperature=0.9, top_k=20, top_p=0.9, response_length=24, ignore_eos=False,
                            seed=3, val_kwargs={}, use_hip_graph=g))
        prompts = DataProto.from_dict({"input_ids": T(z["prompt_ids"]), "attention_mask": T(z["prompt_attention_mask"]),
                                       "position_ids": T(z["prompt_position_ids"])},
                                      meta_info={"eos_token_id": meta["eos_token_id"], "pad_token_id": meta["pad_token_id"]})
        tk.append(MI355XRollout(model, rcfg).generate_sequences(prompts))
    assert torch.equal(tk[0].batch["responses"], tk[1].batch["responses"])
    assert not torch.equal(tk[0].batch["responses"], outs[0].batch["responses"])


@pytest.mark.parametrize("use_hip_graph", [True, False])
def test_rollout_calculate_log_probs(use_hip_graph):
    """rollout.calculate_log_probs (vllm_rollout_spmd.py:350-395): the fp32 greedy rollout's rollout_log_probs are
    the reference HF model's log-probs of the same tokens (golden log_probs, 1e-4) inside the response and -1 past
    it; a bf16 sampled rollout's (T = 0.9) track the actor's compute_log_prob at that temperature (the decode step's
    bf16 logits vs the full-sequence pass: two bf16 roundings) and feed the reference's debug metrics."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.metric_utils import calculate_debug_metrics
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    z, meta = golden()

    def prompts():
        return DataProto.from_dict({"input_ids": T(z["prompt_ids"]), "attention_mask": T(z["prompt_attention_mask"]),
                                    "position_ids": T(z["prompt_position_ids"])},
                                   meta_info={"eos_token_id": meta["eos_token_id"], "pad_token_id": meta["pad_token_id"]})

    cfg, store, model = build()
    rcfg = to_attr(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0, response_length=meta["response_length"],
                        ignore_eos=False, seed=0, val_kwargs={}, use_hip_graph=use_hip_graph, calculate_log_probs=True))
    out = MI355XRollout(model, rcfg).generate_sequences(prompts())
    np.testing.assert_array_equal(out.batch["responses"].cpu().numpy(), z["responses"])
    R = z["responses"].shape[1]
    mask = z["attention_mask"][:, -R:].astype(bool)
    got = out.batch["rollout_log_probs"].cpu().numpy()
    np.testing.assert_allclose(got[mask], z["log_probs"][mask], rtol=1e-4, atol=1e-4)
    assert (got[~mask] == -1.0).all()

    cfg, store, model = build(torch.bfloat16, trainable=False)
    rcfg = to_attr(dict(do_sample=True, temperature=0.9, top_k=-1, top_p=1.0, response_length=24, ignore_eos=False,
                        seed=5, val_kwargs={}, use_hip_graph=use_hip_graph, calculate_log_probs=True))
    out = MI355XRollout(model, rcfg).generate_sequences(prompts())
    plain = MI355XRollout(model, to_attr(dict(rcfg, calculate_log_probs=False))).generate_sequences(prompts())
    assert torch.equal(out.batch["responses"], plain.batch["responses"])  # the log-probs change no token
    actor = DataParallelPPOActor(to_attr({}), model)
    data = out.select(["input_ids", "attention_mask", "position_ids", "responses"])
    data.meta_info.update({"micro_batch_size": 4, "temperature": 0.9, "use_dynamic_bsz": False})
    lp, _ = actor.compute_log_prob(data, calculate_entropy=False)
    m = out.batch["attention_mask"][:, -24:].bool()
    rl = out.batch["rollout_log_probs"]
    assert (rl[~m] == -1.0).all()
    # the decode step's bf16 logits against the full-sequence pass's: two bf16 roundings of logits up to |z| ~ 16
    # (ulp 0.125) over T = 0.9, i.e. at most ~0.14 apart per token, and most tokens far closer
    d = (rl[m] - lp[m]).abs()
    assert d.max().item() < 0.14 and d.mean().item() < 0.02, (d.max().item(), d.mean().item())
    out.batch["old_log_probs"] = lp
    out.batch["response_mask"] = m.to(torch.int64)
    dm = calculate_debug_metrics(out)
    assert dm["training/rollout_probs_diff_max"] < 0.05 and dm["training/rollout_actor_probs_pearson_corr"] > 0.99
    assert dm["training/rollout_probs_diff_valid"] == 1


@pytest.mark.parametrize("temperature,key", [(1.0, "log_probs"), (0.7, "log_probs_t07")])
def test_log_prob_matches_reference(temperature, key):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.protocol import DataProto

    z, meta = golden()
    cfg, store, model = build(trainable=False)
    actor = DataParallelPPOActor(to_attr({}), model)
    data = DataProto.from_dict({"input_ids": T(z["sequences"]), "attention_mask": T(z["attention_mask"]),
                                "position_ids": T(z["position_ids"]), "responses": T(z["responses"])},
                               meta_info={"micro_batch_size": 4, "temperature": temperature, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    np.testing.assert_allclose(lp.cpu().numpy(), z[key], rtol=1e-4, atol=1e-4)
    if temperature == 1.0:
        np.testing.assert_allclose(ent.cpu().numpy(), z["entropy"], rtol=1e-4, atol=1e-4)


def test_layer_backward_matches_autograd():
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor

    z, _ = golden()
    cfg, store, model = build(trainable=True)
    ids, am, pos, resp = T(z["sequences"]), T(z["attention_mask"]), T(z["position_ids"]), T(z["responses"])
    g = torch.Generator(device="cuda").manual_seed(0)
    wl = torch.randn(resp.shape, device="cuda", generator=g)
    we = torch.randn(resp.shape, device="cuda", generator=g)
    # kernel model
    model.training = True
    store.zero_grad()
    actor = DataParallelPPOActor(to_attr({}), model)
    ent, lp = actor._forward_micro_batch({"input_ids": ids, "attention_mask": am, "position_ids": pos,
                                          "responses": resp}, 0.8, calculate_entropy=True)
    torch.autograd.backward([lp, ent], [wl, we])
    # eager autograd (oracle restatement, pinned on CPU against the reference model) on copies of the parameters
    P = {name: store.w(name).detach().clone().float().requires_grad_(True) for name, _, _ in store.specs}
    lp_e, ent_e = qwen2_ref.logp_entropy(cfg, P, ids, am, pos, resp, 0.8)  # oracle: HF math in eager torch
    torch.testing.assert_close(lp, lp_e, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ent, ent_e, rtol=1e-4, atol=1e-4)
    torch.autograd.backward([lp_e, ent_e], [wl, we])
    for name, _, _ in store.specs:
        ref = P[name].grad
        got = store.g(name)
        scale = ref.abs().max().item() + 1e-12
        err = (got - ref).abs().max().item() / scale
        assert err < 2e-4, f"{name}: max rel err {err:.2e}"


def test_bf16_model_tracks_fp32():
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.protocol import DataProto

    z, _ = golden()
    data = DataProto.from_dict({"input_ids": T(z["sequences"]), "attention_mask": T(z["attention_mask"]),
                                "position_ids": T(z["position_ids"]), "responses": T(z["responses"])},
                               meta_info={"micro_batch_size": 6, "temperature": 1.0, "use_dynamic_bsz": False})
    outs = []
    for dt in (torch.float32, torch.bfloat16):
        _, _, model = build(dt, trainable=False)
        lp, _ = DataParallelPPOActor(to_attr({}), model).compute_log_prob(data, calculate_entropy=True)
        outs.append(lp)
    err = (outs[0] - outs[1]).abs().max().item()
    assert err < 0.15, err  # bf16 GEMM inputs over a 0.2-init tiny model


def test_bf16_fused_attention_training_gradients_track_fp32():
    """The bf16 training path (fused attention forward with LSE + fused backward, T % 8 == 0) against the
    fp32 model's gradients on the same data: bf16-level agreement of every parameter gradient."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor

    z, _ = golden()
    ids, am, pos, resp = T(z["sequences"]), T(z["attention_mask"]), T(z["position_ids"]), T(z["responses"])
    Tn = ids.shape[1] // 8 * 8  # fused path needs T % 8 == 0: drop the first prompt columns
    ids, am, pos = ids[:, -Tn:].contiguous(), am[:, -Tn:].contiguous(), pos[:, -Tn:].contiguous()
    g = torch.Generator(device="cuda").manual_seed(1)
    wl = torch.randn(resp.shape, device="cuda", generator=g)
    grads = []
    for dt in (torch.float32, torch.bfloat16):
        cfg, store, model = build(dt, trainable=True)
        model.training = True
        store.zero_grad()
        actor = DataParallelPPOActor(to_attr({}), model)
        _, lp = actor._forward_micro_batch({"input_ids": ids, "attention_mask": am, "position_ids": pos,
                                            "responses": resp}, 1.0, calculate_entropy=False)
        torch.autograd.backward([lp], [wl])
        grads.append({name: store.g(name).clone() for name, _, _ in store.specs})
    for name in grads[0]:
        ref, got = grads[0][name], grads[1][name]
        err = (got - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        assert err < 0.1, f"{name}: bf16 fused-attention grad deviates {err:.3e} from fp32"


def test_fused_lm_head_actor_path_tracks_unfused():
    """actor.use_fused_kernels (A21, csrc/fused_linear.hip) against the unfused bf16 path (lm_head GEMM to bf16
    logits + K2) on the tiny model: log-probs / entropy differ only by the bf16 rounding of the logits, and the
    flat gradient of one micro-batch's (logp, entropy) backward agrees at bf16 level."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor

    z, _ = golden()
    ids, am, pos, resp = T(z["sequences"]), T(z["attention_mask"]), T(z["position_ids"]), T(z["responses"])
    g = torch.Generator(device="cuda").manual_seed(1)
    wl = torch.randn(resp.shape, device="cuda", generator=g)
    we = torch.randn(resp.shape, device="cuda", generator=g)
    outs = []
    for fused in (False, True):
        _, store, model = build(torch.bfloat16, trainable=True)
        model.training = True
        store.zero_grad()
        actor = DataParallelPPOActor(to_attr({"use_fused_kernels": fused}), model)
        ent, lp = actor._forward_micro_batch({"input_ids": ids, "attention_mask": am, "position_ids": pos,
                                              "responses": resp}, 0.9, calculate_entropy=True)
        torch.autograd.backward([lp, ent], [wl, we])
        outs.append((lp.detach(), ent.detach(), store.grad.clone()))
    (lp0, ent0, g0), (lp1, ent1, g1) = outs
    assert (lp0 - lp1).abs().max().item() < 0.05
    assert (ent0 - ent1).abs().max().item() < 0.05
    err = (g0 - g1).abs().max().item() / g0.abs().max().item()
    assert err < 0.05, err
