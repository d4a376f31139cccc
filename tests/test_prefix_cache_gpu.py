"""Prefix caching of the n samples' shared prompt (rollout.enable_prefix_caching; the reference's vLLM rollout runs
with enable_prefix_caching=True, vllm_rollout_spmd.py:195): each distinct prompt is prefilled once into cache row p,
and the MFMA decode attention reads the group's prompt keys from that row (drl_decode_attention_vt prompt groups).

* kernel: grouped reads give bit-identical outputs to the same call on a cache where every row holds its own copy
  of the prompt keys (both workgroup mappings — the XCD-grouped one and the plain one —, split plans, device query
  position, left-padded prompts);
* rollout: the same responses, attention masks and positions as prefilling every row, greedy and sampled, with
  prompt lengths on and off the 32-key block grid, on the packed (bf16) and the fp32 decode paths.
"""

import pytest
import torch

from dots.rl_amd import native

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def _blocked(vt_plain, cap):
    B, Hkv, D = vt_plain.shape[:3]
    nb = (cap + 31) // 32
    out = torch.zeros(B, Hkv, D, nb * 32, dtype=vt_plain.dtype, device=vt_plain.device)
    out[..., :cap] = vt_plain[..., :cap]
    return out.view(B, Hkv, D, nb, 32).permute(0, 1, 3, 2, 4).contiguous()


# (B, group, Hkv, G, D, cap, L, shared): 512 rows in groups of 8 (the bench: XCD-grouped mapping, 128 units); the same
# with 24 own blocks per row (3 per class: multi-block units of the balanced schedule) and with 5 shared blocks (waves
# without a shared item); 12 rows in groups of 4 over 2 heads (6 units: the plain mapping); a small grid (split plan);
# head_dim 128
@pytest.mark.parametrize("B,group,Hkv,G,D,cap,L,shared", [(512, 8, 2, 7, 64, 768, 640, 512),
                                                          (512, 8, 2, 7, 64, 1024, 1000, 256),
                                                          (512, 8, 2, 7, 64, 400, 390, 160),
                                                          (12, 4, 2, 7, 64, 300, 290, 96),
                                                          (8, 4, 1, 8, 64, 2048, 2000, 1024),
                                                          (16, 2, 4, 4, 128, 200, 170, 160)])
def test_decode_attention_prompt_groups_equal_expanded(B, group, Hkv, G, D, cap, L, shared):
    g = torch.Generator(device=DEV).manual_seed(B + L)
    Bu = B // group
    src = torch.arange(B, device=DEV) // group
    q = torch.randn(B, Hkv, G, D, device=DEV, generator=g).to(BF)
    k = torch.randn(B, Hkv, cap, D, device=DEV, generator=g).to(BF)
    vt = torch.randn(B, Hkv, D, (cap + 7) // 8 * 8, device=DEV, generator=g).to(BF)
    valid = torch.zeros(B, (cap + 3) // 4 * 4, dtype=torch.uint8, device=DEV)
    valid[:, :L] = 1
    for b in range(B):
        valid[b, : min(5 * (b // group), shared - 1)] = 0  # left padding per prompt
    # the expanded cache: every row its own copy of its group's prompt keys
    k[:, :, :shared] = k[src, :, :shared]
    vt[..., :shared] = vt[src][..., :shared]
    valid[:, :shared] = valid[src, :shared]
    # the grouped cache: prompt p's keys only in row p, garbage in every other row's prompt region; the key-valid
    # bytes are every row's own (KVCache.share_prompts copies the mask to each row: row p < Bu is itself a sample
    # of prompt p // group and carries that prompt's mask, not prompt p's)
    kg, vtg, vg = k.clone(), vt.clone(), valid.clone()
    kg[:, :, :shared] = torch.randn(B, Hkv, shared, D, device=DEV, generator=g).to(BF)
    vtg[..., :shared] = torch.randn(B, Hkv, D, shared, device=DEV, generator=g).to(BF)
    kg[:Bu, :, :shared] = k[::group, :, :shared]
    vtg[:Bu, ..., :shared] = vt[::group, ..., :shared]
    vb, vbg = _blocked(vt, cap), _blocked(vtg, cap)
    qp = torch.tensor([L - 3], device=DEV)
    lib = native.lib()
    # the grouped kernels (decode_group_kernel: own blocks by block class; decode_group_bal_kernel: own blocks balanced
    # over the waves through class states in LDS) run the per-row kernel's arithmetic at its wave count without key
    # splits: 8 waves at head_dim 64, 4 at 128 by default; forced plans apply to both; 2 rows per column tile as well
    try:
        for nw in ((0, 2, 4, 16) if D == 64 else (0, 2)):
            for kw in ({}, {"qpos_dev": qp}):
                lib.drl_decode_attention_set_plan(nw or (8 if D == 64 else 4), 1)
                a = native.decode_attention_vt(q, k, vb, valid[:, :cap], L, torch.empty_like(q), **kw)
                lib.drl_decode_attention_set_plan(nw, 0)
                for bal, rpt, xmap in ((0, 0, 0), (1, 0, 0), (1, 2, 0), (0, 0, 1)):
                    lib.drl_decode_group_set_plan(rpt, xmap, bal)
                    b = native.decode_attention_vt(q, kg, vbg, vg[:, :cap], L, torch.empty_like(q), group=group,
                                                   shared_keys=shared, **kw)
                    assert torch.equal(a, b), (nw, kw, bal, rpt, xmap)
    finally:
        lib.drl_decode_attention_set_plan(0, 0)
        lib.drl_decode_group_set_plan(0, 0, -1)
    # and close to the per-row kernel's own default plan (another wave count / key split: another fp32 order)
    a = native.decode_attention_vt(q, k, vb, valid[:, :cap], L, torch.empty_like(q))
    b = native.decode_attention_vt(q, kg, vbg, vg[:, :cap], L, torch.empty_like(q), group=group, shared_keys=shared)
    torch.testing.assert_close(a.float(), b.float(), rtol=2e-2, atol=2e-2)


def test_decode_attention_prompt_groups_rejects_bad_args():
    q = torch.zeros(8, 1, 4, 64, dtype=BF, device=DEV)
    k = torch.zeros(8, 1, 64, 64, dtype=BF, device=DEV)
    vt = torch.zeros(8, 1, 2, 64, 32, dtype=BF, device=DEV)
    valid = torch.ones(8, 64, dtype=torch.uint8, device=DEV)
    for group, shared in ((3, 32), (2, 16), (1, 32), (2, 96)):
        with pytest.raises(RuntimeError):
            native.decode_attention_vt(q, k, vt, valid, 64, torch.empty_like(q), group=group, shared_keys=shared)


def _model(dtype, seed=4):
    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config, Qwen2Model

    cfg = Qwen2Config.from_dict(dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                     num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=512,
                                     rope_theta=10000.0, rms_norm_eps=1e-6, tie_word_embeddings=True))
    store = ParamStore(cfg, DEV, compute_dtype=dtype, trainable=False)
    store.init_random(seed)
    return Qwen2Model(cfg, store)


@pytest.mark.parametrize("dtype,P,do_sample,nprompt", [(BF, 40, False, 5), (BF, 40, True, 5), (BF, 64, True, 5),
                                                        (torch.float32, 40, True, 5), (BF, 40, True, 128)])
def test_rollout_prefix_caching_equals_prefill_per_row(dtype, P, do_sample, nprompt):
    """128 prompts x 8 (1024 rows, one KV head): 128 prompt workgroups, so the grouped decode attention runs
    decode_group_kernel; both rollouts at its 8-wave plan without key splits (the per-row kernel would take 2 waves
    at 1024 rows: another fp32 summation order)."""
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    m = _model(dtype)
    n, R = 8, 20
    if nprompt > 5:
        native.lib().drl_decode_attention_set_plan(8, 1)
    g = torch.Generator(device=DEV).manual_seed(P)
    ids = torch.randint(3, 512, (nprompt, P), device=DEV, generator=g)
    am = torch.ones(nprompt, P, dtype=torch.int64, device=DEV)
    for p in range(nprompt):
        am[p, : 3 * (p % 5)] = 0
        ids[p, : 3 * (p % 5)] = 0
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    rep = lambda t: t.repeat_interleave(n, 0)  # noqa: E731  (the trainer's repeat(n, interleave=True))
    outs = []
    for share in (True, False):
        rcfg = to_attr(dict(do_sample=do_sample, temperature=1.0, top_k=-1, top_p=1.0, response_length=R, n=n,
                            ignore_eos=False, seed=11, val_kwargs={}, use_hip_graph=True, packed_decode=True,
                            enable_prefix_caching=share))
        ro = MI355XRollout(m, rcfg)
        out = ro.generate_sequences(DataProto.from_dict(
            {"input_ids": rep(ids), "attention_mask": rep(am), "position_ids": rep(pos)},
            meta_info={"eos_token_id": 2, "pad_token_id": 0}))
        assert ro.last_prompt_group == (n if share else 1)
        outs.append(out.batch)
    native.lib().drl_decode_attention_set_plan(0, 0)
    for key in ("responses", "input_ids", "attention_mask", "position_ids"):
        assert torch.equal(outs[0][key], outs[1][key]), key
    if do_sample:  # the group's samples differ from each other (each row its own Philox stream)
        assert not torch.equal(outs[0]["responses"][0], outs[0]["responses"][1])


def test_rollout_without_runs_of_identical_prompts_prefills_every_row():
    from dots.rl_amd.config import to_attr
    from dots.rl_amd.protocol import DataProto
    from dots.rl_amd.rollout import MI355XRollout

    m = _model(BF)
    B, P = 16, 32
    ids = torch.randint(3, 512, (B, P), device=DEV)
    am = torch.ones(B, P, dtype=torch.int64, device=DEV)
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    rcfg = to_attr(dict(do_sample=False, temperature=1.0, top_k=-1, top_p=1.0, response_length=4, n=8,
                        ignore_eos=True, seed=0, val_kwargs={}, use_hip_graph=True))
    ro = MI355XRollout(m, rcfg)
    ro.generate_sequences(DataProto.from_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos},
                                              meta_info={"eos_token_id": 2, "pad_token_id": 0}))
    assert ro.last_prompt_group == 1
