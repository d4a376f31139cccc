"""The packed decode step (graph-replayed, Qwen2.5-0.5B shapes, random weights, per-row cache filled to L keys) under
each cap on the K slices of the partial-sum projections (o_proj, down_proj): fewer slices write fewer fp32 partials
for the next RMSNorm launch to read, at the cost of fewer workgroups in the projection itself. Usage (GPU box):
python tools/probes/decode_splits_probe.py [B] [L]
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402
from dots.rl_amd.qwen2 import KVCache, PackedDecode, ParamStore, Qwen2Config, Qwen2Model  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    dev = "cuda"
    cfg = Qwen2Config()
    store = ParamStore(cfg, dev, compute_dtype=torch.bfloat16, trainable=False)
    store.init_random(0)
    m = Qwen2Model(cfg, store)
    cache = KVCache(cfg, B, 768, dev, torch.bfloat16)
    for i in range(cfg.num_hidden_layers):
        cache.k[i].normal_()
        cache.vt[i].normal_()
    cache.valid[:, :L].fill_(1)
    tok = torch.randint(0, 1000, (B, 1), device=dev)
    pos = torch.full((B,), L, dtype=torch.int64, device=dev)
    kd = torch.tensor([L], device=dev)
    res = {}
    for rep in range(2):
        for ks in (4, 2, 1):
            native.lib().drl_decode_gemm_set_max_splits(ks)
            pk = PackedDecode(m, B)
            plans = {k: v[0] for k, v in pk.plans.items()}

            def body():
                pk.step(cache, tok, pos, kd)

            body()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(30):
                g.replay()
            b.record()
            b.synchronize()
            res.setdefault(f"max_splits_{ks}", {"ksplit": plans, "step_us": []})["step_us"].append(
                round(a.elapsed_time(b) / 30 * 1e3, 1))
            del g, pk
    native.lib().drl_decode_gemm_set_max_splits(4)
    print(json.dumps(dict(B=B, L=L, **res)), flush=True)


if __name__ == "__main__":
    main()
