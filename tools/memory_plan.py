"""Per-GPU HBM plan of the parameter / gradient / optimizer state for configs #4 and #5 at DP = 8 (and #2 / #3
for comparison), from the real ParamStore layout (padding included) and the fsdp_config.shard='auto' rule
(workers._shard_spec). Also the rollout KV cache for the config's per-rank batch. Prints a markdown table.
Usage: python tools/memory_plan.py"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dots.rl_amd.config import LLAMA3_8B, QWEN25_05B, QWEN25_7B  # noqa: E402
from dots.rl_amd.qwen2 import Qwen2Config, param_specs  # noqa: E402
from dots.rl_amd.workers import _shard_spec  # noqa: E402

GB = 1e9


def store_bytes(cfg, world, trainable, sharded):
    """Bytes of a ParamStore (bf16 compute copy) without allocating it: the same layout arithmetic."""
    A = 64
    pad = lambda n: (n + A - 1) // A * A  # noqa: E731
    specs = param_specs(cfg)
    n_small = sum(pad(math.prod(s)) for _, s, k in specs if k == "small")
    gemm = sum(pad(math.prod(s)) for _, s, k in specs if k != "small")
    w = world if sharded else 1
    gemm = (gemm + A * w - 1) // (A * w) * (A * w)
    numel = n_small + gemm
    if not trainable:
        return {"compute_bf16": 2 * numel, "master_fp32": 4 * n_small}
    master = n_small + (gemm // w if sharded else gemm)
    return {"compute_bf16": 2 * numel, "grad_fp32": 4 * numel, "master_fp32": 4 * master,
            "adam_moments_fp32": 8 * master}


def activation_bytes(cfg, micro_seqs, mini_seqs, seq_len, budget_gb=40):
    """Saved activations of one update pass under dp_actor.exec_groups (micro-batches per pass chosen to stay under
    exec_activation_gb, at least one): per token and layer x, x2 fp32; h1, h2, attn bf16; q / k / v / k^T; gate|up and
    the SwiGLU output. The weights are read in place by drl_gemm (no transposed copies)."""
    nq = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * cfg.head_dim
    H, I = cfg.hidden_size, cfg.intermediate_size
    per_tok = cfg.num_hidden_layers * (8 * H + 6 * H + 4 * nq + 6 * I)
    toks = micro_seqs * seq_len
    n = max(1, min(mini_seqs // micro_seqs, int(budget_gb * 2 ** 30 // (per_tok * toks))))
    return per_tok * toks * n


def plan(name, arch, world, critic, seqs_per_rank, seq_len, micro=8, mini=32):
    actor = Qwen2Config.from_dict(arch)
    sec = {"fsdp_config": {"shard": "auto"}}
    sh = _shard_spec(sec, actor, 0, world) is not None
    rows = {"actor": store_bytes(actor, world, True, sh), "ref": store_bytes(actor, world, False, False)}
    if sh:  # the sharded step's reduce-scattered gradient buffer (FlatAdamW.grad_work) = master size
        rows["actor"]["grad_shard_fp32"] = rows["actor"]["master_fp32"]
    if critic:
        c = Qwen2Config.from_dict(dict(arch, num_labels=1))
        csh = _shard_spec(sec, c, 0, world) is not None
        rows["critic"] = store_bytes(c, world, True, csh)
        if csh:
            rows["critic"]["grad_shard_fp32"] = rows["critic"]["master_fp32"]
    kv = 2 * actor.num_key_value_heads * actor.head_dim * 2 * actor.num_hidden_layers * seqs_per_rank * seq_len
    act = activation_bytes(actor, micro, mini, seq_len)  # the actor's and the critic's updates run one after another
    total = sum(sum(r.values()) for r in rows.values()) + max(kv, act)
    return name, world, sh, rows, kv, act, total


def main():
    cases = [plan("#2/#3 Qwen2.5-0.5B GRPO", QWEN25_05B, 8, False, 64, 768),
             plan("#4 Llama-3-8B PPO (actor+critic)", LLAMA3_8B, 8, True, 64, 768),
             plan("#5 Qwen2.5-7B DAPO", QWEN25_7B, 8, False, 64, 512 + 1024, micro=2, mini=4)]
    print("| config (DP=8, per GPU) | sharded | actor | ref | critic | rollout KV cache | update activations | "
          "peak (state + max(KV, activations)) |")
    print("|---|---|---|---|---|---|---|---|")
    for name, world, sh, rows, kv, act, total in cases:
        fmt = lambda r: f"{sum(r.values()) / GB:.1f} GB" if r else "—"  # noqa: E731
        print(f"| {name} | {'yes' if sh else 'no'} | {fmt(rows['actor'])} | {fmt(rows['ref'])} | "
              f"{fmt(rows.get('critic'))} | {kv / GB:.1f} GB | {act / GB:.1f} GB | **{total / GB:.1f} GB** of 288 |")
    # the same configs replicated (what fails)
    for arch, name, critic in ((LLAMA3_8B, "#4 replicated", True), (QWEN25_7B, "#5 replicated", False)):
        a = Qwen2Config.from_dict(arch)
        t = sum(store_bytes(a, 8, True, False).values()) + sum(store_bytes(a, 8, False, False).values())
        if critic:
            t += sum(store_bytes(Qwen2Config.from_dict(dict(arch, num_labels=1)), 8, True, False).values())
        print(f"| {name} (no sharding) | no | | | | | {t / GB:.1f} GB of 288 |")


if __name__ == "__main__":
    main()
