"""Fused-norm decode step (csrc/decode_gemm.hip, ABI 8) in situ: every configuration of the norm consumers
(qkv + RoPE, gate_up + SwiGLU) and K-slice cap of the residual producers (o_proj, down_proj), each timed over the 24
layers' own packed weights inside one HIP graph (weights read cold, as in the step), next to the seven-launch step's
kernels; then the whole layer stack (PackedDecode._layers) fused vs unfused. One JSON line per rows.

  python tools/decode_norm_sweep.py [--rows 64 128]
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


def graph_time(fn, reps=10):
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
    ap.add_argument("--rows", type=int, nargs="*", default=[64, 128])
    args = ap.parse_args()
    cfg = Qwen2Config.from_dict(QWEN25_05B)
    store = ParamStore(cfg, "cuda", compute_dtype=torch.bfloat16, trainable=False)
    store.init_random(0)
    model = Qwen2Model(cfg, store)
    H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    Hq, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    NQ, HD, eps = (Hq + 2 * Hkv) * D, Hq * D, cfg.rms_norm_eps
    lib = native.lib()
    for B in args.rows:
        pf = PackedDecode(model, B, fused_norm=True)
        pu = PackedDecode(model, B, fused_norm=False, weights=pf.w)
        assert pf.fused, "rows outside the fused form"
        cache = KVCache(cfg, B, 768, "cuda", torch.bfloat16)
        cache.valid[:, :600] = 1
        for t in (pf.attn_p, pf.a_p, pu.h_p, pu.attn_p, pu.a_p):
            t.normal_()
        pf.xr.normal_()
        pu.x.normal_()
        pos = torch.full((B,), 600, dtype=torch.int64, device="cuda")
        kpos = torch.full((1,), 600, dtype=torch.int64, device="cuda")
        mbt = pf.mbt
        w = pf.w
        nw = lambda i, k: store.w(f"layers.{i}.{k}")  # noqa: E731
        row = {"rows": B, "mbt": mbt, "plans": {k: list(v) for k, v in pf.fplans.items()}}

        def per_layer(fn):
            return round(graph_time(lambda: [fn(i) for i in range(L)]) / L, 2)

        # the seven-launch step's kernels
        row["unfused"] = {
            "norm": per_layer(lambda i: native.decode_rmsnorm(pu.x, pu.part_d, pu.x, nw(i, "input_layernorm"), pu.h_p,
                                                              eps, mbt=mbt)),
            "qkv_rope": per_layer(lambda i: native.decode_qkv_rope(pu.h_p, w[i]["qkv"], model.qkv_bias(i), pos,
                                                                   model.cos, model.sin, B, H, Hq, Hkv, D, pu.q,
                                                                   cache.k[i], cache.vt[i], kpos)),
            "o": per_layer(lambda i: native.decode_gemm(pu.attn_p, w[i]["o"], B, H, HD, partials=pu.part_o)),
            "gate_up": per_layer(lambda i: native.decode_gemm(pu.h_p, w[i]["gu"], B, 2 * I, H, swiglu=True,
                                                              out_packed=pu.a_p)),
            "down": per_layer(lambda i: native.decode_gemm(pu.a_p, w[i]["d"], B, H, I, partials=pu.part_d)),
        }
        fused = {}
        for ci in (-1, 0, 1, 2, 3):
            lib.drl_decode_norm_set_plan(ci, 0, 0)
            for name, fn in (("qkv_norm", lambda i: native.decode_qkv_rope_norm(
                                 pf.xr, nw(i, "input_layernorm"), eps, w[i]["qkv"], model.qkv_bias(i), pos, model.cos,
                                 model.sin, B, H, Hq, Hkv, D, pf.q, cache.k[i], cache.vt[i], kpos)),
                             ("gu_norm", lambda i: native.decode_gemm_norm(
                                 pf.xr, nw(i, "post_attention_layernorm"), eps, w[i]["gu"], B, 2 * I, H, pf.a_p))):
                try:
                    fused[f"{name}_cfg{ci}"] = per_layer(fn)
                except (RuntimeError, AssertionError) as e:
                    fused[f"{name}_cfg{ci}"] = str(e)[:50]
        lib.drl_decode_norm_set_plan(-1, 0, 0)
        for ks in (0, 1, 2, 4):
            lib.drl_decode_norm_set_plan(-1, 0, ks)
            for name, N_, K_, src, key, part in (("o_resid", H, HD, pf.attn_p, "o", pf.part_o),
                                                 ("d_resid", H, I, pf.a_p, "d", pf.part_d)):
                plan = native.decode_norm_plan(B, N_, K_, native.DECODE_RESID)
                if plan is None:
                    continue
                part_ = torch.empty(plan[0], B, N_, device="cuda")
                try:
                    fused[f"{name}_ks{plan[0]}_ksw{plan[2]}"] = per_layer(
                        lambda i: native.decode_gemm_resid(src, w[i][key], B, N_, K_, pf.xr, mbt, part_, pf.cnt))
                except (RuntimeError, AssertionError) as e:
                    fused[f"{name}_ks{ks}"] = str(e)[:50]
        lib.drl_decode_norm_set_plan(-1, 0, 0)
        row["fused"] = fused
        row["layers_unfused_us"] = round(graph_time(lambda: pu._layers(cache, pos, kpos)), 1)
        row["layers_fused_us"] = round(graph_time(lambda: pf._layers(cache, pos, kpos)), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
