"""Actor / critic checkpoint files (workers._save_store / _load_store, the worker's save_checkpoint /
load_checkpoint of fsdp_workers.py:844-911): a round trip restores the flat fp32 master and the AdamW state bit for
bit, and a file whose flat-buffer layout differs from the store (an unversioned file from before the small-region
layout, another sharding, another model) is refused instead of loading permuted weights."""

import os

import pytest
import torch

from dots.rl_amd.dp_actor import FlatAdamW
from dots.rl_amd.qwen2 import ParamStore, Qwen2Config
from dots.rl_amd.workers import _load_store, _save_store

CFG = dict(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=2,
           num_key_value_heads=1)


def _store(seed=0, **over):
    cfg = Qwen2Config(**dict(CFG, **over))
    st = ParamStore(cfg, "cpu", compute_dtype=torch.float32)
    st.init_random(seed)
    opt = FlatAdamW(st, lr=1e-3)
    g = torch.Generator().manual_seed(seed + 1)
    opt.exp_avg.copy_(torch.randn(opt.exp_avg.shape, generator=g))
    opt.exp_avg_sq.copy_(torch.rand(opt.exp_avg_sq.shape, generator=g))
    opt.step_count, opt.sched_step = 7, 3
    return st, opt


def test_round_trip(tmp_path):
    st, opt = _store(0)
    _save_store(st, opt, str(tmp_path), "model_optim_rng", {"global_step": 5}, 0)
    st2, opt2 = _store(1)
    sd = _load_store(st2, opt2, str(tmp_path), "model_optim_rng")
    assert sd["global_step"] == 5
    assert torch.equal(st2.master, st.master)
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
    assert (opt2.step_count, opt2.sched_step) == (7, 3)


def test_rejects_unversioned_file(tmp_path):
    """A payload without the layout record (what the writer produced before it existed) is refused."""
    st, opt = _store(0)
    torch.save({"master": st.master.clone(), "n_small": st.n_small, "world": 1,
                "optim": {k: (v.clone() if torch.is_tensor(v) else v) for k, v in opt.state_dict().items()}},
               os.path.join(tmp_path, "model_optim_rng.pt"))
    st2, opt2 = _store(1)
    before = st2.master.clone()
    with pytest.raises(ValueError, match="without a layout record"):
        _load_store(st2, opt2, str(tmp_path), "model_optim_rng")
    assert torch.equal(st2.master, before)


def test_rejects_other_layout(tmp_path):
    """Same element count, different parameter order: refused (a shape check alone would pass this one)."""
    st, opt = _store(0)
    _save_store(st, opt, str(tmp_path), "critic_model_optim", {}, 0)
    sd = torch.load(os.path.join(tmp_path, "critic_model_optim.pt"), weights_only=True)
    sd["layout"]["offsets"] = sd["layout"]["offsets"][::-1]
    torch.save(sd, os.path.join(tmp_path, "critic_model_optim.pt"))
    st2, opt2 = _store(1)
    with pytest.raises(ValueError, match="offsets"):
        _load_store(st2, opt2, str(tmp_path), "critic_model_optim")
    other, other_opt = _store(1, intermediate_size=192)
    _save_store(other, other_opt, str(tmp_path / "b"), "m", {}, 0)
    with pytest.raises(ValueError):
        _load_store(st2, opt2, str(tmp_path / "b"), "m")
