"""DP correctness on the GPU before any hardware scaling curve.

Two fresh child processes (tests/dp2_child.py, started with subprocess: the test process never execs
itself) form a gloo world of 2 sharing cuda:0 and run one GRPO-style actor update through the SPMD worker
group: rank r receives the r-th chunk of an 8-sequence batch (DP_COMPUTE_PROTO, decorator.py:213-241),
takes 2 mini-batches x 2 micro-batches over its 4 rows with its own token-mean per micro-batch, and FlatAdamW
AVG-all-reduces the flat gradient before clip + AdamW. The reference's semantics (dp_actor.py:413-417 with
FSDP's gradient averaging) make the applied gradient the mean of the two ranks' accumulated gradients; the
test restates that composition in this process (DP = 1: every micro-batch of both ranks, loss scaled by
1/grad_accum/world, one optimizer step per mini-batch) and checks
* both ranks end with bit-identical parameters (one all-reduced gradient, the same AdamW);
* those parameters equal the restatement's (AdamW updates within 2 % for 99.9 % of elements, the bar of
  test_actor_update_gpu.py) and the per-rank metrics are the restatement's per-rank micro-batch values.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _restated_dp1(world=2):
    """The reference composition of a DP=world update, in one process."""
    import dp2_child

    from dots.rl_amd.core_algos import fused_actor_loss
    from dots.rl_amd.dp_actor import DataParallelPPOActor
    from dots.rl_amd.workers import ActorRolloutRefWorker

    cfg = dp2_child.build_config(1)
    w = ActorRolloutRefWorker(cfg, role="actor")  # dp 1: ppo_mini_batch_size stays the global 4
    w.init_model()
    a = cfg.actor
    data = dp2_child.batch("cuda").batch
    B = data["input_ids"].shape[0]
    per_rank = B // world
    mini = a.ppo_mini_batch_size // world  # the per-rank normalised size (fsdp_workers.py:209-214)
    micro = a.ppo_micro_batch_size_per_gpu
    grad_accum = mini // micro
    actor: DataParallelPPOActor = w.actor
    opt = w.actor_optimizer
    per_rank_metrics = [dict() for _ in range(world)]
    for i in range(per_rank // mini):
        opt.zero_grad()
        w.actor_module.training = True
        for r in range(world):
            for j in range(grad_accum):
                lo = r * per_rank + i * mini + j * micro
                mb = {k: v[lo:lo + micro] for k, v in data.items()}
                ent, lp = actor._forward_micro_batch(mb, 1.0, calculate_entropy=False)
                out = fused_actor_loss(lp, ent, mb["old_log_probs"], mb["advantages"], mb["response_mask"],
                                       mb["ref_log_prob"], clip_ratio_low=a.clip_ratio_low,
                                       clip_ratio_high=a.clip_ratio_high, clip_ratio_c=a.clip_ratio_c,
                                       entropy_coeff=a.entropy_coeff, use_kl_loss=a.use_kl_loss,
                                       kl_loss_type=a.kl_loss_type, kl_loss_coef=a.kl_loss_coef,
                                       loss_agg_mode=a.loss_agg_mode, loss_scale_factor=1.0 / grad_accum / world)
                out[6].backward()
                row = out.detach().cpu().tolist()
                m = per_rank_metrics[r]
                # the rank's own metric scaling (dp_actor.py:458-466): loss_scale_factor = 1 / grad_accum
                for k, v in (("actor/pg_loss", row[0] / grad_accum), ("actor/pg_clipfrac", row[1]),
                             ("actor/ppo_kl", row[2]), ("actor/kl_loss", row[5] / grad_accum)):
                    m.setdefault(k, []).append(v)
        gn = opt.step()
        for r in range(world):
            per_rank_metrics[r].setdefault("actor/grad_norm", []).append(float(gn.item()))
    return w.store.master.detach().cpu(), per_rank_metrics


def _run_pair(tmp_path, tag, extra=()):
    port = _free_port()
    procs, outs = [], []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK="0")
        out = str(tmp_path / f"{tag}_rank{r}.pt")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp2_child.py"), out, *extra], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [torch.load(o, weights_only=True) for o in outs]


def test_dp2_sharded_optimizer_equals_replicated(tmp_path):
    """ZeRO-style sharding (fsdp_config.shard=true: fp32 master + AdamW moments split over the 2 ranks, AVG
    reduce-scatter of the gradient, all-gather of the compute copy) against the replicated optimizer
    (all-reduce) on the same DP=2 update, real HIP kernels: the same parameters on both ranks, equal to the
    replicated run's up to the total-norm summation order (AdamW is elementwise)."""
    rep = _run_pair(tmp_path, "rep")
    sh = _run_pair(tmp_path, "shard", ("shard",))
    assert sh[0]["sharded"] and not rep[0]["sharded"]
    assert torch.equal(sh[0]["master"], sh[1]["master"])
    n = rep[0]["master"].numel()  # the sharded layout pads the GEMM region to a multiple of world * 64
    assert sh[0]["master"].numel() >= n and not sh[0]["master"][n:].any()
    d = (sh[0]["master"][:n] - rep[0]["master"]).abs().max().item()
    step = (rep[0]["master"]).abs().max().item()
    assert d <= 1e-6 * max(step, 1.0), d
    for r in range(2):
        a, b = json.loads(sh[r]["metrics"]), json.loads(rep[r]["metrics"])
        np.testing.assert_allclose(a["actor/grad_norm"], b["actor/grad_norm"], rtol=1e-5)
        np.testing.assert_allclose(a["actor/pg_loss"], b["actor/pg_loss"], rtol=1e-6, atol=1e-7)


def test_dp2_update_equals_mean_of_rank_gradients(tmp_path):
    res = _run_pair(tmp_path, "rep")
    assert res[0]["mini_batch_size"] == res[1]["mini_batch_size"] == 2
    assert torch.equal(res[0]["master"], res[1]["master"])
    want_master, want_metrics = _restated_dp1()
    from safetensors.torch import load_file

    from dots.rl_amd.qwen2 import ParamStore, Qwen2Config

    cfg = Qwen2Config.from_dict(json.load(open(os.path.join(HERE, "golden", "tiny_qwen2", "config.json"))))
    init = ParamStore(cfg, "cpu", compute_dtype=torch.float32, trainable=False)
    init.load_state_dict_hf(load_file(os.path.join(HERE, "golden", "tiny_qwen2", "model.safetensors")))
    d_got = (res[0]["master"] - init.master).numpy()
    d_ref = (want_master - init.master).numpy()
    step = np.abs(d_ref)
    bad = np.abs(d_got - d_ref) > 0.02 * np.maximum(step, np.median(step[step > 0]))
    assert bad.mean() < 1e-3, f"{bad.sum()} of {bad.size} updates differ from the mean-of-rank-gradients step"
    for r in range(2):
        got = json.loads(res[r]["metrics"])
        for k, v in want_metrics[r].items():
            tol = dict(rtol=1e-4) if k == "actor/grad_norm" else dict(rtol=1e-4, atol=1e-5)
            np.testing.assert_allclose(got[k], v, err_msg=f"rank {r} {k}", **tol)
