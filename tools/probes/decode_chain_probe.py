"""Marginal cost of each launch kind inside the graph-replayed packed decode step (Qwen2.5-0.5B shapes, random
weights, KV cache filled to L keys): the step is a dependent chain of short launches, so a kernel's cost is
what removing it from the chain saves, not its isolated duration. Variants drop one launch kind (wrong
numbers, right timing). Usage (GPU box): python tools/decode_chain_probe.py [B] [L]
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dots.rl_amd import native  # noqa: E402
from dots.rl_amd.qwen2 import KVCache, PackedDecode, ParamStore, Qwen2Config, Qwen2Model  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
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
    pk = PackedDecode(m, B)
    tok = torch.randint(0, 1000, (B, 1), device=dev)
    pos = torch.full((B,), L, dtype=torch.int64, device=dev)
    kd = torch.tensor([L], device=dev)
    out = torch.empty(B, dtype=torch.int64, device=dev)
    orig = {n: getattr(native, n) for n in ("decode_rmsnorm", "decode_qkv_rope", "decode_attention_vt", "decode_gemm")}

    def noop(*a, **k):
        return None

    def gemm_skip(which):
        def f(x, w, M, N, K, **kw):
            kind = "gu" if kw.get("swiglu") else ("d" if K == cfg.intermediate_size else "o")
            return None if kind == which else orig["decode_gemm"](x, w, M, N, K, **kw)
        return f

    variants = {
        "full": {},
        "no_rmsnorm": {"decode_rmsnorm": lambda x, p, xo, w, y, eps, mbt=0, **kw: None if mbt else
                       orig["decode_rmsnorm"](x, p, xo, w, y, eps, mbt=mbt, **kw)},
        "no_qkv": {"decode_qkv_rope": noop},
        "no_attention": {"decode_attention_vt": noop},
        "no_o": {"decode_gemm": gemm_skip("o")},
        "no_gu": {"decode_gemm": gemm_skip("gu")},
        "no_down": {"decode_gemm": gemm_skip("d")},
    }
    res = {}
    for head in (False, True):
        for name, patch in variants.items():
            if head and name != "full":
                continue
            for k, v in patch.items():
                setattr(native, k, v)

            def body():
                h = pk.step(cache, tok, pos, kd)
                if head:
                    m.select_tokens(h, out, fused=False, do_sample=True, seed=1, dev_step=kd)

            body()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            for k in patch:
                setattr(native, k, orig[k])
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                g.replay()
            b.record()
            b.synchronize()
            res[name + ("+head" if head else "")] = round(a.elapsed_time(b) / 20 * 1e3, 1)
            del g
    full = res["full"]
    print(json.dumps(dict(B=B, L=L, step_us=res, marginal_per_layer_us={
        k[3:]: round((full - v) / cfg.num_hidden_layers, 2) for k, v in res.items() if k.startswith("no_")},
        head_us=round(res["full+head"] - full, 1))), flush=True)


if __name__ == "__main__":
    main()
