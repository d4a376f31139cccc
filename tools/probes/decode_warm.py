"""How much of a decode projection is the cold weight stream: each projection of the Qwen2.5-0.5B decode step timed
inside one HIP graph over the 24 layers' own packed weights (cold: 713 MB of weights per pass, as in the step) and over
layer 0's weight 24 times (warm: 2-17 MB, MALL / L2 resident). python tools/probes/decode_warm.py [rows ...]"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402
from dots.rl_amd.config import QWEN25_05B  # noqa: E402
from dots.rl_amd.qwen2 import KVCache, PackedDecode, ParamStore, Qwen2Config, Qwen2Model  # noqa: E402


def graph_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    rows = [int(x) for x in sys.argv[1:]] or [64, 512]
    cfg = Qwen2Config.from_dict(QWEN25_05B)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=False)
    store.init_random(0)
    model = Qwen2Model(cfg, store)
    H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    for B in rows:
        pd = PackedDecode(model, B)
        cache = KVCache(cfg, B, 768, "cuda", torch.bfloat16)
        pd.h_p.normal_()
        pd.attn_p.normal_()
        pd.a_p.normal_()
        pos = torch.full((B,), 600, dtype=torch.int64, device="cuda")
        kpos = torch.full((1,), 600, dtype=torch.int64, device="cuda")
        part = torch.empty(max(H, I) // 16 * B * max(H, 2 * I), device="cuda")
        projs = {
            "qkv_rope": lambda i: native.decode_qkv_rope(pd.h_p, pd.w[i]["qkv"], model.qkv_bias(i), pos, model.cos,
                                                         model.sin, B, H, Hq, Hkv, D, pd.q, cache.k[i], cache.vt[i],
                                                         kpos),
            "o": lambda i: native.decode_gemm(pd.attn_p, pd.w[i]["o"], B, H, Hq * D,
                                              partials=part[:native.decode_gemm_plan(B, H, Hq * D)[0] * B * H].view(-1, B, H)),
            "gate_up": lambda i: native.decode_gemm(pd.h_p, pd.w[i]["gu"], B, 2 * I, H, swiglu=True, out_packed=pd.a_p),
            "down": lambda i: native.decode_gemm(pd.a_p, pd.w[i]["d"], B, H, I,
                                                 partials=part[:native.decode_gemm_plan(B, H, I)[0] * B * H].view(-1, B, H)),
        }
        for name, fn in projs.items():
            row = {"rows": B, "proj": name}
            row["cold_us"] = round(graph_time(lambda: [fn(i) for i in range(L)]) / L, 2)
            row["warm_us"] = round(graph_time(lambda: [fn(0) for _ in range(L)]) / L, 2)
            print(json.dumps(row), flush=True)
        # a whole layer's projections back to back, cold and warm
        row = {"rows": B, "proj": "all4"}
        row["cold_us"] = round(graph_time(lambda: [f(i) for i in range(L) for f in projs.values()]) / L, 2)
        row["warm_us"] = round(graph_time(lambda: [f(0) for _ in range(L) for f in projs.values()]) / L, 2)
        print(json.dumps(row), flush=True)
        del pd, cache, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
