"""Config #2 at full depth (24 layers, H 896, 14 / 2 heads, V 151 936) against the reference HF model.

Weights: tests/golden/full_depth.py rebuilds the CPU-seeded Qwen2.5-0.5B-shaped tensors bit for bit (2 GB,
never committed); tests/golden/full_depth.npz holds the reference HF Qwen2ForCausalLM's fp32 outputs on 4 x
64-token prompts: greedy tokens (64 steps, HFRollout post-processing) with each step's top-2 logit margin,
teacher-forced log-probs / entropy, and the CPU bf16-autocast error of the top-2 margin at every step.

* fp32 mode: greedy rollout bit-exact (all 256 tokens, masks, positions); log-probs and entropy 1e-4.
* bf16 production mode (the packed decode path the bench runs, HIP graph replay):
  - teacher-forced, the bf16 model's greedy choice equals the reference token at every step whose reference
    margin exceeds BF16_MARGIN (twice the largest CPU bf16 margin error recorded in the fixture);
  - the rollout reproduces the reference tokens until its first divergence, and a divergence is allowed only at
    a step whose reference margin is below BF16_MARGIN (after it the contexts differ);
  - teacher-forced log-probs within 0.3 (the CPU bf16 autocast model is 0.144 off at worst).
"""

import json
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.fixture(scope="module")
def ref():
    z = np.load(os.path.join(HERE, "golden", "full_depth.npz"), allow_pickle=False)
    return z, json.loads(str(z["__meta__"]))


@pytest.fixture(scope="module")
def weights(ref):
    import full_depth as fd

    sd = fd.make_state_dict()
    want = ref[1]["weight_checksum"]
    got = fd.checksum(sd)
    assert got == want, [k for k in want if got[k] != want[k]][:5]  # bit-identical regeneration on this host
    return sd


def _model(sd, dtype):
    import full_depth as fd

    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(fd.QWEN25_05B)
    store = ParamStore(cfg, "cuda", compute_dtype=dtype, trainable=False)
    store.load_state_dict_hf(sd)
    return Qwen2Model(cfg, store)


def _rollout(model, z, meta, **over):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    rcfg = to_attr(dict(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0,
                             response_length=meta["response_length"], ignore_eos=False, seed=0, val_kwargs={},
                             use_hip_graph=True, packed_decode=True, packed_decode_max_rows=512), **over))
    prompts = DataProto.from_dict({"input_ids": T(z["prompt_ids"]), "attention_mask": T(z["prompt_attention_mask"]),
                                   "position_ids": T(z["prompt_position_ids"])},
                                  meta_info={"eos_token_id": meta["eos_token_id"], "pad_token_id": meta["pad_token_id"]})
    ro = MI355XRollout(model, rcfg)
    out = ro.generate_sequences(prompts)
    return out, ro


def _teacher_forced(model, z):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.protocol import DataProto

    actor = DataParallelPPOActor(to_attr({}), model)
    data = DataProto.from_dict({"input_ids": T(z["sequences"]), "attention_mask": T(z["attention_mask"]),
                                "position_ids": T(z["position_ids"]), "responses": T(z["responses"])},
                               meta_info={"micro_batch_size": 4, "temperature": 1.0, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    R = z["responses"].shape[1]
    with torch.no_grad():  # the greedy choice at every teacher-forced response step
        h = model.hidden_states(T(z["sequences"]), T(z["attention_mask"]), T(z["position_ids"]))
        h = h[:, -R - 1:-1].reshape(-1, h.shape[-1])
        am = model.logits(h).float().argmax(-1).view(-1, R)
    return lp.cpu().numpy(), ent.cpu().numpy(), am.cpu().numpy()


def test_fp32_full_depth_matches_reference(ref, weights):
    z, meta = ref
    model = _model(weights, torch.float32)
    out, _ = _rollout(model, z, meta)
    for k, r in [("input_ids", "sequences"), ("responses", "responses"), ("attention_mask", "attention_mask"),
                 ("position_ids", "position_ids")]:
        np.testing.assert_array_equal(out.batch[k].cpu().numpy(), z[r], err_msg=k)
    lp, ent, _ = _teacher_forced(model, z)
    np.testing.assert_allclose(lp, z["log_probs"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ent, z["entropy"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("packed,hip_gemm_rows", [(True, None), (False, None), (True, 1), (False, 1)])
def test_bf16_full_depth_margin_checked(ref, weights, packed, hip_gemm_rows, monkeypatch):
    """hip_gemm_rows=1: every full-sequence qkv / o_proj / gate_up projection (prefill, teacher-forced pass, the
    unpacked decode step) on csrc/gemm.hip's ping-pong GEMM, held to the same reference margins"""
    from dots.rl_amd import qwen2

    if hip_gemm_rows is not None:
        monkeypatch.setattr(qwen2, "HIP_GEMM_MIN_ROWS", hip_gemm_rows)
    z, meta = ref
    bound = 2.0 * meta["cpu_bf16_gap_err_max"]
    gaps = z["top2_gap"]
    model = _model(weights, torch.bfloat16)
    lp, _, argmax = _teacher_forced(model, z)
    confident = gaps > bound
    assert confident.sum() >= 0.1 * confident.size  # the check covers a real share of the steps
    np.testing.assert_array_equal(argmax[confident], z["responses"][confident])
    np.testing.assert_allclose(lp, z["log_probs"], atol=0.3)
    out, ro = _rollout(model, z, meta, packed_decode=packed)
    assert ro.last_packed_decode == packed
    resp = out.batch["responses"].cpu().numpy()
    matched = []
    for b in range(resp.shape[0]):
        diff = np.nonzero(resp[b] != z["responses"][b])[0]
        first = int(diff[0]) if diff.size else resp.shape[1]
        matched.append(first)
        if first < resp.shape[1]:
            assert gaps[b, first] < bound, (b, first, gaps[b, first], bound)
    print(f"bf16 {'packed' if packed else 'unpacked'} rollout: tokens matching the fp32 reference per row {matched}")
