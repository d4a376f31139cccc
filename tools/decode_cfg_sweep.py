"""Decode-step projections (csrc/decode_gemm.hip) in situ: every configuration of the packed decode GEMM for each
projection of a Qwen2.5-0.5B decode step (qkv + bias + RoPE + cache writes, o_proj partials, gate_up + SwiGLU,
down_proj partials), each timed over the 24 layers' own packed weights inside one HIP graph (every weight read
cold, as in the step). One JSON line per (rows, projection): planner choice and every forced configuration.

  python tools/decode_cfg_sweep.py [--rows 512 64]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dots.rl_amd import native  # noqa: E402
from dots.rl_amd.config import QWEN25_05B  # noqa: E402
from dots.rl_amd.qwen2 import KVCache, PackedDecode, ParamStore, Qwen2Config, Qwen2Model  # noqa: E402

NCFG = 23  # kTiled entries


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="*", default=[512, 256])
    args = ap.parse_args()
    cfg = Qwen2Config.from_dict(QWEN25_05B)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=False)
    store.init_random(0)
    model = Qwen2Model(cfg, store)
    H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    lib = native.lib()
    for B in args.rows:
        pd = PackedDecode(model, B)
        cache = KVCache(cfg, B, 768, "cuda", torch.bfloat16)
        pd.h_p.normal_()
        pd.attn_p.normal_()
        pd.a_p.normal_()
        pos = torch.full((B,), 600, dtype=torch.int64, device="cuda")
        kpos = torch.full((1,), 600, dtype=torch.int64, device="cuda")
        part = torch.empty(max(H, I) // 16 * B * max(H, 2 * I), device="cuda")
        NQ = (Hq + 2 * Hkv) * D
        wq = [native.decode_pack_weight(store.w(f"layers.{i}.qkv_proj.weight")) for i in range(L)]

        def qkv_split(i):  # qkv partials over K slices, then one bias + RoPE + cache-write launch
            ks = native.decode_gemm_plan(B, NQ, H)[0]
            pq = part[:ks * B * NQ].view(ks, B, NQ)
            native.decode_gemm(pd.h_p, wq[i], B, NQ, H, partials=pq)
            native.decode_rope(pq, model.qkv_bias(i), pos, model.cos, model.sin, Hq, Hkv, D, pd.q, cache.k[i],
                               vt_cache=cache.vt[i], koff_dev=kpos)

        projs = {
            "qkv_split_rope": qkv_split,
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
            for ci in [-1] + (list(range(NCFG)) if B >= 64 else []):
                lib.drl_decode_gemm_force_tiled(ci, 1 if ci >= 0 else 0)
                try:
                    us = graph_time(lambda: [fn(i) for i in range(L)]) / L
                    row["planner" if ci < 0 else f"cfg{ci}"] = round(us, 2)
                except RuntimeError as e:  # a configuration that does not take this shape
                    row["planner" if ci < 0 else f"cfg{ci}"] = str(e)[:40]
            lib.drl_decode_gemm_force_tiled(-1, 0)
            if name in ("down", "o") and B >= 256:  # long / short K partials with more K slices
                for ks in (8, 16):
                    lib.drl_decode_gemm_set_max_splits(ks)
                    for ci in range(NCFG):
                        lib.drl_decode_gemm_force_tiled(ci, 1)
                        try:
                            row[f"cfg{ci}_ks{ks}"] = round(graph_time(lambda: [fn(i) for i in range(L)]) / L, 2)
                        except RuntimeError as e:
                            row[f"cfg{ci}_ks{ks}"] = str(e)[:40]
                    lib.drl_decode_gemm_force_tiled(-1, 0)
                lib.drl_decode_gemm_set_max_splits(4)
            # the one-round-trip kernel (4 waves per workgroup each on a K quarter, reduced in LDS) at these rows
            for mb in (1, 2):
                lib.drl_decode_gemm_set_tiled(0)
                lib.drl_decode_gemm_set_plan(mb, 0)
                try:
                    row[f"untiled_mb{mb}"] = round(graph_time(lambda: [fn(i) for i in range(L)]) / L, 2)
                except (RuntimeError, AssertionError) as e:
                    row[f"untiled_mb{mb}"] = str(e)[:40]
                lib.drl_decode_gemm_set_plan(0, 0)
                lib.drl_decode_gemm_set_tiled(1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
