"""ZeRO-style sharded optimizer (ParamStore(shard=(rank, world)) + FlatAdamW._step_sharded) against the
replicated optimizer on gloo world-size 2 (CPU). The HIP grad-norm / AdamW kernels are replaced, in the child
processes only, by the oracle's float32 restatement (oracle.adamw_step, tested against torch.optim.AdamW
below): what is under test is the sharding itself — layout, AVG reduce-scatter of the GEMM region, AVG
all-reduce of the small region, the sharded total norm, the per-shard step and the all-gather of the compute
copy. Without clipping the sharded step is bit-identical to the replicated one (AdamW is elementwise); with
clipping the total norm is summed in another order, so the parameters agree to float32 rounding."""

import numpy as np
import pytest
import torch
import torch.distributed as dist

from test_distributed_cpu import spawn


def _tiny_cfg():
    from dots.rl_amd.qwen2 import Qwen2Config

    return Qwen2Config.from_dict(dict(vocab_size=96, hidden_size=32, intermediate_size=64, num_hidden_layers=3,
                                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64,
                                      tie_word_embeddings=True))


def _patch_native():
    import oracle
    from dots.rl_amd import native

    def grad_norm(g, out=None):
        v = torch.tensor([oracle.grad_norm(g.detach().numpy())], dtype=torch.float32)
        if out is None:
            return v
        out.copy_(v)
        return out

    def adamw_step(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, step, max_grad_norm, grad_norm_t=None,
                   params_bf16=None):
        pn, mn, vn = p.detach().numpy(), m.detach().numpy(), v.detach().numpy()  # views: updated in place
        oracle.adamw_step(pn, g.detach().numpy(), mn, vn, lr=lr, beta1=beta1, beta2=beta2, eps=eps,
                          weight_decay=weight_decay, step=step, max_grad_norm=max_grad_norm,
                          grad_norm_value=float(grad_norm_t.item()))
        if params_bf16 is not None:
            params_bf16.copy_(p)

    native.grad_norm = grad_norm
    native.adamw_step = adamw_step


def _shard_case(rank, world, max_norm):
    from dots.rl_amd.dp_actor import FlatAdamW
    from dots.rl_amd.qwen2 import ParamStore

    _patch_native()
    cfg = _tiny_cfg()
    rep = ParamStore(cfg, "cpu", compute_dtype=torch.float32, trainable=True)
    sh = ParamStore(cfg, "cpu", compute_dtype=torch.float32, trainable=True, shard=(rank, world))
    rep.init_random(7)
    sh.init_random(7)
    init_equal = all(torch.equal(rep.w(n), sh.w(n)) for n, _, _ in rep.specs)
    o_rep = FlatAdamW(rep, lr=1e-2, weight_decay=0.01, max_grad_norm=max_norm)
    o_sh = FlatAdamW(sh, lr=1e-2, weight_decay=0.01, max_grad_norm=max_norm)
    norms = []
    for step in range(3):
        gen = torch.Generator().manual_seed(100 * step + rank)  # rank-dependent gradients
        for name, shape, _ in rep.specs:
            g = torch.randn(shape, generator=gen)
            rep.g(name).copy_(g)
            sh.g(name).copy_(g)
        n1 = float(o_rep.step().item())
        n2 = float(o_sh.step().item())
        norms.append((n1, n2))
    diffs = {n: float((rep.w(n) - sh.w(n)).abs().max()) for n, _, _ in rep.specs}
    exact = all(torch.equal(rep.w(n), sh.w(n)) for n, _, _ in rep.specs)
    # shard sizes: the sharded master holds the small region + 1/world of the GEMM region
    return dict(init_equal=init_equal, norms=norms, exact=exact, maxdiff=max(diffs.values()),
                master=(rep.master.numel(), sh.master.numel(), sh.n_small, sh.shard_len),
                moments=(o_rep.exp_avg.numel(), o_sh.exp_avg.numel()))


def _case_noclip(rank, world):
    return _shard_case(rank, world, max_norm=1e9)


def _case_clip(rank, world):
    return _shard_case(rank, world, max_norm=0.5)


def test_sharded_adamw_bit_identical_without_clipping():
    out = spawn(_case_noclip)
    for r in (0, 1):
        o = out[r]
        assert o["init_equal"]
        assert o["exact"], o["maxdiff"]
        for n1, n2 in o["norms"]:
            assert abs(n1 - n2) <= 2e-6 * n1
        rep_master, sh_master, n_small, shard_len = o["master"]
        assert sh_master == n_small + shard_len and shard_len * 2 >= rep_master - n_small
        assert o["moments"][1] == sh_master < o["moments"][0]


def test_sharded_adamw_with_clipping():
    out = spawn(_case_clip)
    for r in (0, 1):
        o = out[r]
        assert all(n1 > 0.5 for n1, _ in o["norms"])  # clipping active
        for n1, n2 in o["norms"]:
            assert abs(n1 - n2) <= 2e-6 * n1
        assert o["maxdiff"] <= 1e-6, o["maxdiff"]


def test_oracle_adamw_matches_torch():
    """oracle.adamw_step == torch.optim.AdamW after clip_grad_norm_ (the reference's _optimizer_step)."""
    import oracle

    rng = np.random.default_rng(3)
    p0 = rng.standard_normal(1000).astype(np.float32)
    p = p0.copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    tp = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = torch.optim.AdamW([tp], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    for step in range(1, 4):
        g = rng.standard_normal(1000).astype(np.float32) * 3
        tp.grad = torch.from_numpy(g.copy())
        tn = torch.nn.utils.clip_grad_norm_([tp], max_norm=1.0)
        opt.step()
        oracle.adamw_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=step,
                          max_grad_norm=1.0, grad_norm_value=oracle.grad_norm(g))
        assert abs(float(tn) - float(oracle.grad_norm(g))) <= 1e-5 * float(tn)
        np.testing.assert_allclose(p, tp.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_shard_spec_auto():
    """fsdp_config.shard='auto' shards the 7-8 B configs (#4 / #5) at DP > 1 and leaves Qwen2.5-0.5B
    replicated; the per-GPU footprint of the sharded 8 B actor + critic + reference fits 288 GB."""
    from dots.rl_amd.config import LLAMA3_8B, QWEN25_05B, QWEN25_7B
    from dots.rl_amd.qwen2 import Qwen2Config, param_specs
    from dots.rl_amd.workers import _shard_spec

    sec = {"fsdp_config": {"shard": "auto"}}
    small = Qwen2Config.from_dict(QWEN25_05B)
    assert _shard_spec(sec, small, 0, 8) is None
    for d in (LLAMA3_8B, QWEN25_7B):
        c = Qwen2Config.from_dict(d)
        assert _shard_spec(sec, c, 3, 8) == (3, 8)
        assert _shard_spec(sec, c, 0, 1) is None
        assert _shard_spec({"fsdp_config": {"shard": False}}, c, 3, 8) is None
        n = sum(int(np.prod(s)) for _, s, _ in param_specs(c))
        # actor (bf16 compute 2 B + fp32 grad 4 B + master/moments 12 B / 8) + critic (same) + ref (bf16)
        per_gpu = 2 * n * (2 + 4 + 12 / 8) + 2 * n
        assert per_gpu < 150e9, per_gpu
        assert 2 * n * (2 + 4 + 12) + 2 * n > 288e9  # replicated would not fit
