"""Configs #4 / #5 at FULL DEPTH against the reference HF models (VERDICT r03 "missing" 3).

Fixture ``deep.npz`` (tests/golden/make_golden.py::gen_deep): HF LlamaForCausalLM (Llama-3-8B: 32 layers, H 4096,
32 / 8 heads of 128, V 128256) and Qwen2ForCausalLM (Qwen2.5-7B: 28 layers, H 3584, 28 / 4 heads of 128, V 152064,
qkv bias), both untied, on counter-hash weights (tests/golden/deep.py: regenerated here on the GPU bit for bit, the
sampled digest pins it), teacher-forced over 2 x (32 prompt + 32 response) tokens with a left-padded row: the
response tokens' log-probs, entropy and logsumexp, and the top-32 logits of every response-predicting position, in
fp32 and under the CPU bf16 autocast.

This repository's actor (DataParallelPPOActor.compute_log_prob, the production path) on the same weights:
  * fp32 (compute_dtype float32): log-probs and entropy within 5e-4 absolute at these depths (fp32 summation order
    over K up to 18944, 28-32 layers);
  * bf16 (the production kernels: drl_gemm projections, the fused attention at head_dim 128, K2): the distribution
    of |log p - ref| and |entropy - ref| over the 64 response positions against the CPU bf16-autocast model's own
    error distribution on the same positions — median within 1.5x, 90th percentile and maximum within 2x. (Per
    position the two bf16 runs are independent realisations of 28-32 layers of rounding in different summation
    orders: where the CPU model happens to be near-exact says nothing about ours, so the errors are compared as
    distributions.)
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

import deep  # noqa: E402


@pytest.fixture(scope="module")
def ref():
    z = np.load(os.path.join(HERE, "golden", "deep.npz"), allow_pickle=False)
    return z, json.loads(str(z["__meta__"]))


def _log_probs(which, meta, z, dtype):
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    sd = deep.state_dict(which, device="cuda")
    assert deep.sample_digest(sd) == meta["models"][which]["weight_digest"]  # bit-identical regeneration
    cfg = Qwen2Config.from_dict(deep.MODELS[which])
    store = ParamStore(cfg, "cuda", compute_dtype=dtype, trainable=False)
    store.load_state_dict_hf(sd)
    del sd
    torch.cuda.empty_cache()
    actor = DataParallelPPOActor(to_attr({}), Qwen2Model(cfg, store))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    p = which + "_"
    ids = T(z[p + "input_ids"])
    data = DataProto.from_dict({"input_ids": ids, "attention_mask": T(z[p + "attention_mask"]),
                                "position_ids": T(z[p + "position_ids"]), "responses": ids[:, deep.P:].contiguous()},
                               meta_info={"micro_batch_size": deep.B, "temperature": 1.0, "use_dynamic_bsz": False})
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    del actor, store
    torch.cuda.empty_cache()
    return lp.cpu().numpy().astype(np.float64), ent.cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("which", ["llama", "qwen7b"])
def test_full_depth_fp32(ref, which):
    z, meta = ref
    lp, ent = _log_probs(which, meta, z, torch.float32)
    p = which + "_"
    np.testing.assert_allclose(lp, z[p + "log_probs"], rtol=0, atol=5e-4)
    np.testing.assert_allclose(ent, z[p + "entropy"], rtol=0, atol=5e-4)


@pytest.mark.parametrize("which", ["llama", "qwen7b"])
def test_full_depth_bf16_within_reference_bf16_error(ref, which):
    z, meta = ref
    lp, ent = _log_probs(which, meta, z, torch.bfloat16)
    p = which + "_"
    for name, got, want, cpu in (("log-prob", lp, z[p + "log_probs"], z[p + "cpu_bf16_log_probs"]),
                                 ("entropy", ent, z[p + "entropy"], z[p + "cpu_bf16_entropy"])):
        cpu_err = np.abs(cpu.astype(np.float64) - want).reshape(-1)
        err = np.abs(got - want).reshape(-1)
        q = lambda e, f: float(np.quantile(e, f))  # noqa: E731
        print(f"{which} {name}: ours median / p90 / max {q(err, .5):.4f} / {q(err, .9):.4f} / {err.max():.4f}, "
              f"CPU bf16 {q(cpu_err, .5):.4f} / {q(cpu_err, .9):.4f} / {cpu_err.max():.4f}")
        assert q(err, .5) <= 1.5 * q(cpu_err, .5) + 1e-4
        assert q(err, .9) <= 2.0 * q(cpu_err, .9) + 1e-4
        assert err.max() <= 2.0 * cpu_err.max() + 1e-4
