"""Per-kernel roofline sweep of the hand-written HIP kernels (HIP events on the launch stream).

Algorithmic bytes per unit:
  K1 ppo loss fwd+bwd : 36 B / token  (read old, logp, adv, entropy, ref: 5 x 4 B; mask int64 8 B;
                                       write dlogp, dentropy: 2 x 4 B)
  K2 logprob fwd      : 2V + 16 B / row (bf16 logits row, label int64, write logp + entropy fp32)
  K2 logprob bwd      : 4V + 8+16 B / row (read bf16 logits, write bf16 dlogits; per-row scalars)
  K4 select (greedy)  : 2V + 8 B / row
  AdamW step          : 28 B / param (+2 B bf16 copy) ; grad norm : 4 B / param
  decode attention    : 4 D B / key (K and V rows, bf16) per (sequence, KV head) + q/out rows
Usage: python tools/kernel_bench.py [--quick] > out.jsonl
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dots.rl_amd import native  # noqa: E402

PEAK_HBM = 8.0e12  # MI355X HBM3E spec peak, B/s (MI355X_MICROARCH.md)


def time_it(fn, iters=20, warmup=3):
    s = torch.cuda.current_stream()
    for _ in range(warmup):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def time_graph(fn, n):
    """GPU time per call of n back-to-back calls captured in one HIP graph (no host launch cost: the decode
    step replays its kernels from a graph too)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (3 * n) * 1e-3


def k1_sweep(exps):
    rows = []
    for e in exps:
        N = 1 << e
        R = 1024 if N >= 1024 else N
        B = N // R
        g = torch.Generator(device="cuda").manual_seed(e)
        old = -torch.rand(B, R, device="cuda", generator=g) * 5
        lp = old + torch.randn(B, R, device="cuda", generator=g) * 0.3
        adv = torch.randn(B, R, device="cuda", generator=g)
        mask = (torch.rand(B, R, device="cuda", generator=g) > 0.05).to(torch.int64)
        ent = torch.rand(B, R, device="cuda", generator=g)
        ref = lp + 0.1
        out = torch.empty(8, device="cuda")
        dlp = torch.empty_like(lp)
        dent = torch.empty_like(lp)
        kw = dict(entropy_coeff=0.001, kl_loss_coef=0.001, kl_loss_type="low_var_kl", loss_agg_mode="token-mean",
                  want_dentropy=True, out=out, dlogp=dlp, dentropy=dent)
        t = time_it(lambda: native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, **kw))
        byt = 36 * N
        rows.append(dict(kernel="K1_ppo_loss_fwd_bwd", tokens=N, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
        # one-pass form: the batch's token count is already known (computed once, outside the timed region)
        tc = mask.to(torch.float64).sum().reshape(1)
        t1 = time_it(lambda: native.ppo_loss_fwd_bwd(old, lp, adv, mask, ent, ref, token_count=tc, **kw))
        rows.append(dict(kernel="K1_ppo_loss_fwd_bwd_one_pass", tokens=N, seconds=t1, GBps=byt / t1 / 1e9,
                         frac=byt / t1 / PEAK_HBM))
        del old, lp, adv, mask, ent, ref, dlp, dent
        torch.cuda.empty_cache()
    return rows


def k2(rows_n=4096, V=151936):
    x = torch.randn(rows_n, V, device="cuda", dtype=torch.bfloat16) * 3
    lab = torch.randint(0, V, (rows_n,), device="cuda")
    res = []
    t = time_it(lambda: native.logprob_entropy_fwd(x, lab))
    byt = rows_n * (2 * V + 16)
    res.append(dict(kernel="K2_logprob_entropy_fwd", rows=rows_n, V=V, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
    lp, ent, lse = native.logprob_entropy_fwd(x, lab)
    dl = torch.randn(rows_n, device="cuda")
    out = torch.empty_like(x)
    t = time_it(lambda: native.logprob_entropy_bwd(x, lab, 1.0, dl, dl, lse, ent, out=out))
    byt = rows_n * (4 * V + 24)
    res.append(dict(kernel="K2_logprob_entropy_bwd", rows=rows_n, V=V, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
    tok = torch.empty(rows_n, dtype=torch.int64, device="cuda")
    sub = x[:512]
    t = time_it(lambda: native.select_tokens(sub, tok[:512]))
    byt = 512 * (2 * V + 8)
    res.append(dict(kernel="K4_select_greedy", rows=512, V=V, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
    t = time_it(lambda: native.select_tokens(sub, tok[:512], do_sample=True, temperature=1.0, seed=1))
    res.append(dict(kernel="K4_select_sample", rows=512, V=V, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
    return res


def adam(n=494_032_768):
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    pbf = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    nrm = torch.empty(1, device="cuda")
    res = []
    t = time_it(lambda: native.grad_norm(g, out=nrm))
    res.append(dict(kernel="A15_grad_norm", params=n, seconds=t, GBps=4 * n / t / 1e9, frac=4 * n / t / PEAK_HBM))
    t = time_it(lambda: native.adamw_step(p, g, m, v, lr=1e-6, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01,
                                          step=1, max_grad_norm=1.0, grad_norm_t=nrm, params_bf16=pbf))
    res.append(dict(kernel="A15_adamw_step", params=n, seconds=t, GBps=30 * n / t / 1e9, frac=30 * n / t / PEAK_HBM))
    return res


def decode_attn(B=512, Hkv=2, G=7, D=64, Tk=768, L=640):
    dev = "cuda"
    q = torch.randn(B, Hkv, G, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, Tk, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    valid = torch.ones(B, Tk, dtype=torch.uint8, device=dev)
    out = torch.empty_like(q)
    t = time_graph(lambda: native.decode_attention(q, k, v, valid, L, out), 50)
    nbytes = B * Hkv * (2 * L * D * 2 + 2 * G * D * 2)
    vt = v.transpose(-1, -2).contiguous()
    t2 = time_graph(lambda: native.decode_attention_vt(q, k, vt, valid, L, out), 50)
    return [dict(kernel="A3_decode_attention", B=B, L=L, seconds=t, GBps=nbytes / t / 1e9, frac=nbytes / t / PEAK_HBM),
            dict(kernel="A3_decode_attention_vt_mfma", B=B, L=L, seconds=t2, GBps=nbytes / t2 / 1e9,
                 frac=nbytes / t2 / PEAK_HBM)]


def decode_sweep(Bs=(64, 128, 256, 512), Ls=(513, 768), Hkv=2, G=7, D=64):
    """MFMA decode attention over (waves per workgroup, key splits) plans, graph-timed."""
    dev = "cuda"
    res = []
    for B in Bs:
        for L in Ls:
            q = torch.randn(B, Hkv, G, D, device=dev, dtype=torch.bfloat16)
            k = torch.randn(B, Hkv, 768, D, device=dev, dtype=torch.bfloat16)
            vt = torch.randn(B, Hkv, D, 768, device=dev, dtype=torch.bfloat16)
            valid = torch.ones(B, 768, dtype=torch.uint8, device=dev)
            out = torch.empty_like(q)
            sweep = {}
            for lean in (0, 1):
                native.lib().drl_decode_attention_set_variant(lean)
                for nw in (0, 2, 4, 8, 16):
                    for sp in (0, 1, 2):
                        if (nw == 0) != (sp == 0):
                            continue
                        native.lib().drl_decode_attention_set_plan(nw, sp)
                        sweep[f"{'L' if lean else ''}{nw}x{sp}"] = round(time_graph(
                            lambda: native.decode_attention_vt(q, k, vt, valid, L, out), 50) * 1e6, 2)
            native.lib().drl_decode_attention_set_variant(0)
            native.lib().drl_decode_attention_set_plan(0, 0)
            best = min(sweep, key=sweep.get)
            res.append(dict(kernel="decode_attention_vt_sweep", B=B, L=L, auto_us=sweep["0x0"], best=best,
                            best_us=sweep[best], sweep_us=sweep))
    return res


def decode_sweep_cold(Bs=(64, 128, 256, 512), L=640, Hkv=2, G=7, D=64, footprint=768 << 20):
    """As decode_sweep, but each call reads a different cache copy (footprint > the 256 MB MALL), the in-situ
    pattern of 24 layers' caches per decode step: HBM-cold numbers."""
    dev = "cuda"
    res = []
    for B in Bs:
        per = B * Hkv * 768 * D * 2 * 2
        n = max(2, -(-footprint // per))
        qs = [torch.randn(B, Hkv, G, D, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        ks = [torch.randn(B, Hkv, 768, D, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        # the rollout's key-blocked V^T cache (KVCache); DECODE_VT_PLAIN=1 for the head-dim-major layout
        vshape = (B, Hkv, D, 768) if os.environ.get("DECODE_VT_PLAIN") == "1" else (B, Hkv, 24, D, 32)
        vts = [torch.randn(*vshape, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        valid = torch.ones(B, 768, dtype=torch.uint8, device=dev)
        out = torch.empty_like(qs[0])

        def run():
            for i in range(n):
                native.decode_attention_vt(qs[i], ks[i], vts[i], valid, L, out)

        sweep = {}
        for var in (0, 1, 3, 4):  # 0: two blocks in flight, 1: lean, 3/4: ring depth
            native.lib().drl_decode_attention_set_variant(var)
            for nw in (0, 2, 4, 8):
                for sp in (0, 1, 2):
                    if (nw == 0) != (sp == 0) or (var and nw == 0) or (var > 1 and (sp > 1 or nw < 4)):
                        continue
                    native.lib().drl_decode_attention_set_plan(nw, sp)
                    tag = {0: "", 1: "L", 3: "R3_", 4: "R4_"}[var]
                    sweep[f"{tag}{nw}x{sp}"] = round(time_graph(run, 4) / n * 1e6, 2)
        native.lib().drl_decode_attention_set_variant(0)
        native.lib().drl_decode_attention_set_plan(0, 0)
        best = min(sweep, key=sweep.get)
        nbytes = B * Hkv * L * D * 4
        res.append(dict(kernel="decode_attention_vt_cold", B=B, L=L, copies=n, auto_us=sweep["0x0"], best=best,
                        best_us=sweep[best], best_GBps=round(nbytes / sweep[best] / 1e3, 1), sweep_us=sweep))
        del qs, ks, vts
    return res


def decode_split_sweep(Bs=(64, 128), L=640, Hkv=2, G=7, D=64, footprint=768 << 20):
    """Key-split plans for small decode grids (HBM-cold as decode_sweep_cold): workgroups = B x Hkv x splits."""
    dev = "cuda"
    res = []
    for B in Bs:
        per = B * Hkv * 768 * D * 2 * 2
        n = max(2, -(-footprint // per))
        qs = [torch.randn(B, Hkv, G, D, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        ks = [torch.randn(B, Hkv, 768, D, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        # the rollout's key-blocked V^T cache (KVCache); DECODE_VT_PLAIN=1 for the head-dim-major layout
        vshape = (B, Hkv, D, 768) if os.environ.get("DECODE_VT_PLAIN") == "1" else (B, Hkv, 24, D, 32)
        vts = [torch.randn(*vshape, device=dev, dtype=torch.bfloat16) for _ in range(n)]
        valid = torch.ones(B, 768, dtype=torch.uint8, device=dev)
        out = torch.empty_like(qs[0])

        def run():
            for i in range(n):
                native.decode_attention_vt(qs[i], ks[i], vts[i], valid, L, out)

        sweep = {"auto": round(time_graph(run, 4) / n * 1e6, 2)}
        for nw in (2, 4, 8):
            for sp in (1, 2, 4, 8):
                native.lib().drl_decode_attention_set_plan(nw, sp)
                sweep[f"{nw}x{sp}"] = round(time_graph(run, 4) / n * 1e6, 2)
        native.lib().drl_decode_attention_set_plan(0, 0)
        best = min(sweep, key=sweep.get)
        res.append(dict(kernel="decode_attention_split_sweep", B=B, L=L, best=best, best_us=sweep[best],
                        sweep_us=sweep))
        del qs, ks, vts
    return res


def rope(B=16, T=768, Hq=14, Hkv=2, D=64):
    """RoPE + head split of the qkv projection (rope_qkv_fwd) at the log-prob (V^T copy) and training (k, v, K^T,
    V^T copies) micro-batch shapes; bytes = qkv read + every output written once."""
    dev, bf = "cuda", torch.bfloat16
    G = Hq // Hkv
    qkv = torch.randn(B, T, (Hq + 2 * Hkv) * D, device=dev, dtype=bf)
    pos = torch.arange(T, device=dev).expand(B, T).contiguous()
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, device=dev).float() / D))
    ang = torch.arange(32768, device=dev).float()[:, None] * inv[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    q = torch.empty(B, Hkv, G, T, D, device=dev, dtype=bf)
    k = torch.empty(B, Hkv, T, D, device=dev, dtype=bf)
    v = torch.empty_like(k)
    kt, vt = torch.empty(B, Hkv, D, T, device=dev, dtype=bf), torch.empty(B, Hkv, D, T, device=dev, dtype=bf)
    res = []
    for name, kw in (("logprob", dict(v=None, vt=vt)), ("train", dict(v=v, kt=kt, vt=vt))):
        vv = kw.pop("v")
        t = time_it(lambda: native.rope_qkv_fwd(qkv, pos, cos, sin, Hq, Hkv, D, q, k, vv, **kw))
        nbytes = B * T * D * 2 * (Hq + 2 * Hkv) + B * T * D * 2 * (Hq + Hkv * (4 if name == "train" else 2))
        res.append(dict(kernel="rope_qkv_fwd", form=name, B=B, T=T, us=t * 1e6, GBps=nbytes / t / 1e9,
                        frac=nbytes / t / PEAK_HBM))
    dqkv = torch.empty_like(qkv)
    t = time_it(lambda: native.rope_qkv_bwd(q, k, v, pos, cos, sin, Hq, Hkv, D, dqkv))
    nbytes = 2 * B * T * D * 2 * (Hq + 2 * Hkv)
    res.append(dict(kernel="rope_qkv_bwd", form="train", B=B, T=T, us=t * 1e6, GBps=nbytes / t / 1e9,
                    frac=nbytes / t / PEAK_HBM))
    return res


def flash(B=16, Hkv=2, G=7, D=64, T=768):
    """Fused attention forward vs the unfused path (fp32-score GEMM + masked softmax + PV GEMM)."""
    import math
    dev = "cuda"
    q = torch.randn(B, Hkv, G, T, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16)
    vt = v.transpose(-1, -2).contiguous()
    valid = torch.ones(B, T, dtype=torch.uint8, device=dev)
    out = torch.empty(B, T, Hkv * G * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, Hkv, G, T, device=dev)
    t = time_it(lambda: native.flash_attn_fwd(q, k, vt, valid, out, lse=lse), iters=20)
    flops = 4.0 * B * Hkv * G * D * T * (T + 1) / 2  # causal half of QK^T and PV

    def unfused():
        S = torch.bmm(q.view(B * Hkv, G * T, D), k.view(B * Hkv, T, D).transpose(1, 2), out_dtype=torch.float32)
        P = torch.empty(B * Hkv, G * T, T, device=dev, dtype=torch.bfloat16)
        native.masked_softmax_fwd(S, P, valid, B, Hkv * G, T, T, 0, 1.0 / math.sqrt(D))
        return torch.bmm(P, v.view(B * Hkv, T, D))
    t2 = time_it(unfused, iters=10) if B <= 16 else float("nan")
    return [dict(kernel="flash_attn_fwd", B=B, T=T, seconds=t, TFLOPs=flops / t / 1e12, frac_mfma=flops / t / 2.5e15,
                 unfused_seconds=t2)]


def flash_bwd(B=8, Hkv=2, G=7, D=64, T=768):
    """Fused attention backward (dq + dkdv launches) at the update micro-batch shape."""
    dev = "cuda"
    bf = torch.bfloat16
    q = torch.randn(B, Hkv, G, T, D, device=dev, dtype=bf)
    k = torch.randn(B, Hkv, T, D, device=dev, dtype=bf)
    v = torch.randn(B, Hkv, T, D, device=dev, dtype=bf)
    kt = k.transpose(-1, -2).contiguous()
    vt = v.transpose(-1, -2).contiguous()
    valid = torch.ones(B, T, dtype=torch.uint8, device=dev)
    o = torch.empty(B, T, Hkv * G * D, device=dev, dtype=bf)
    lse = torch.empty(B, Hkv, G, T, device=dev)
    native.flash_attn_fwd(q, k, vt, valid, o, lse=lse)
    dout = torch.randn(B, T, Hkv * G * D, device=dev, dtype=bf)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    t = time_it(lambda: native.flash_attn_bwd(q, k, kt, v, o, dout, lse, valid, dq, dk, dv), iters=20)
    tf = time_it(lambda: native.flash_attn_fwd(q, k, vt, valid, o, lse=lse), iters=20)
    flops = 4.0 * B * Hkv * G * D * T * (T + 1) / 2
    return [dict(kernel="flash_attn_bwd", B=B, T=T, seconds=t, TFLOPs=2.5 * flops / t / 1e12,
                 frac_mfma=2.5 * flops / t / 2.5e15, fwd_seconds=tf)]


def fused_linear(Ns=(2048, 4096), H=896, V=151936):
    """A21 fused lm_head + logp + entropy vs the unfused path (bf16 logits GEMM + K2), forward and backward.
    MFMA-bound: 2*N*H*V FLOP per forward (and per d_logits recompute)."""
    dev, bf = "cuda", torch.bfloat16
    w = torch.randn(V, H, device=dev, dtype=bf) * 0.05
    gw = torch.zeros(V, H, device=dev, dtype=torch.float32)
    res = []
    for N in Ns:
        h = torch.randn(N, H, device=dev, dtype=bf)
        lab = torch.randint(0, V, (N,), device=dev)
        dlp = torch.randn(N, device=dev)
        fl = 2.0 * N * H * V
        t_f = time_it(lambda: native.linear_logprob_fwd(h, w, lab, 1.0))
        t_u = time_it(lambda: native.logprob_entropy_fwd(h @ w.t(), lab, 1.0))
        _, ent, lse = native.linear_logprob_fwd(h, w, lab, 1.0)

        def fused_bwd():
            dlt = native.linear_logprob_dlogits(h, w, lab, 1.0, dlp, None, lse, None)
            dh = dlt.t() @ w
            torch.addmm(gw, dlt, h, out_dtype=torch.float32, out=gw)
            return dh

        logits = h @ w.t()

        def unfused_bwd():
            dl = native.logprob_entropy_bwd(logits, lab, 1.0, dlp, None, lse, None, out=logits)
            dh = dl @ w
            torch.addmm(gw, dl.t(), h, out_dtype=torch.float32, out=gw)
            return dh

        t_dl = time_it(lambda: native.linear_logprob_dlogits(h, w, lab, 1.0, dlp, None, lse, None))
        t_fb = time_it(fused_bwd)
        t_ub = time_it(unfused_bwd)
        res.append(dict(kernel="fused_linear", N=N, H=H, V=V, fwd_us=t_f * 1e6, fwd_TFLOPs=fl / t_f / 1e12,
                        fwd_frac=fl / t_f / 2.5e15, unfused_fwd_us=t_u * 1e6, dlogits_us=t_dl * 1e6,
                        dlogits_TFLOPs=fl / t_dl / 1e12, bwd_us=t_fb * 1e6, unfused_bwd_us=t_ub * 1e6))
    return res


def decode_gemm(Ms=(32, 64, 128, 256, 512)):
    """Decode projections on fragment-packed operands (csrc/decode_gemm.hip) vs hipBLASLt at the Qwen2.5-0.5B
    shapes, weights rotating over > 600 MB of copies (each call streams W from HBM), graph-timed."""
    dev, bf = "cuda", torch.bfloat16
    shapes = [("qkv_proj", 1152, 896, False), ("o_proj", 896, 896, False), ("gate_up_swiglu", 9728, 896, True),
              ("down_proj", 896, 4864, False)]
    res = []
    for name, N, K, sw in shapes:
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        ws = [torch.randn(N, K, device=dev, dtype=bf) * 0.05 for _ in range(ncopy)]
        wps = [native.decode_pack_weight(w, swiglu=sw) for w in ws]
        for M in Ms:
            ks, mbt = native.decode_gemm_plan(M, N, K, sw)
            x = torch.randn(M, K, device=dev, dtype=bf)
            xp = native.pack_activations(x, mbt)
            part = torch.empty(K // 16, M, N, device=dev)  # room for the deepest K split (1 step per wave)
            outp = torch.zeros(mbt * 32 * (N // 2), device=dev, dtype=bf)
            it = iter(range(1 << 30))

            def ours():
                return native.decode_gemm(xp, wps[next(it) % ncopy], M, N, K, swiglu=sw, partials=part,
                                          out_packed=outp)

            def lib():
                y = x @ ws[next(it) % ncopy].t()
                if sw:
                    a = torch.empty(M, N // 2, device=dev, dtype=bf)
                    native.swiglu_fwd(y, a)
                    return a
                return y
            sweep = {}
            native.lib().drl_decode_gemm_set_tiled(0)  # the one-round-trip form's plans
            for mbw in (2, 1):
                for ksw in (19, 14, 7, 4, 2, 1):
                    native.lib().drl_decode_gemm_set_plan(mbw, ksw)
                    if native.decode_gemm_plan(M, N, K, sw) is None:
                        continue
                    sweep[f"{mbw}x{ksw}"] = round(time_graph(ours, ncopy) * 1e6, 2)
            native.lib().drl_decode_gemm_set_plan(0, 0)
            t_rt = time_graph(ours, ncopy)
            native.lib().drl_decode_gemm_set_tiled(1)
            tiled = {}
            for ci in range(9):  # every tiled configuration (0-3 LDS-staged, 4-8 register ring), from 97 rows
                native.lib().drl_decode_gemm_force_tiled(ci, 97)
                if native.decode_gemm_plan(M, N, K, sw) is not None and M >= 97:
                    tiled[ci] = round(time_graph(ours, ncopy) * 1e6, 2)
            native.lib().drl_decode_gemm_force_tiled(-1, 0)
            ks, _ = native.decode_gemm_plan(M, N, K, sw)
            t = time_graph(ours, ncopy)  # the automatic plan (MFMA-tiled form from 192 rows)
            t2 = time_graph(lib, ncopy)
            nbytes = 2 * N * K + 2 * M * K
            res.append(dict(kernel="decode_gemm", layer=name, M=M, N=N, K=K, ksplit=ks, us=t * 1e6,
                            one_round_trip_us=t_rt * 1e6, GBps=nbytes / t / 1e9, TFLOPs=2 * M * N * K / t / 1e12,
                            hipblaslt_us=t2 * 1e6, sweep_us=sweep, tiled_us=tiled))
    return res


def train_gemms(Ms=(6144, 12288)):
    """hipBLASLt on the transformer GEMMs of the log-prob / update micro-batches (hipBLASLt's default heuristics; a comparison only):
    forward y = x W^T, backward dx = dy W and dW += dy^T x (fp32 accumulate in place)."""
    dev, bf = "cuda", torch.bfloat16
    res = []
    for name, N, K in (("qkv", 1152, 896), ("o_proj", 896, 896), ("gate_up", 9728, 896), ("down", 896, 4864)):
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.05
        gw = torch.zeros(N, K, device=dev)
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            dy = torch.randn(M, N, device=dev, dtype=bf)
            fl = 2.0 * M * N * K
            tf = time_it(lambda: x @ w.t())
            tb = time_it(lambda: dy @ w)
            tw = time_it(lambda: torch.addmm(gw, dy.t(), x, out_dtype=torch.float32, out=gw))
            res.append(dict(kernel="train_gemm", layer=name, M=M, N=N, K=K, fwd_us=tf * 1e6, fwd_TF=fl / tf / 1e12,
                            dx_us=tb * 1e6, dx_TF=fl / tb / 1e12, dw_us=tw * 1e6, dw_TF=fl / tw / 1e12))
    return res


def swiglu(Ns=(6144, 12288), I=4864):
    """SwiGLU forward / backward at the training (8 x 768) and log-prob (16 x 768) micro-batch rows, HBM GB/s."""
    dev, bf = "cuda", torch.bfloat16
    res = []
    for N in Ns:
        gu = torch.randn(N, 2 * I, device=dev, dtype=bf)
        a = torch.empty(N, I, device=dev, dtype=bf)
        da = torch.randn(N, I, device=dev, dtype=bf)
        dgu = torch.empty_like(gu)
        t = time_it(lambda: native.swiglu_fwd(gu, a))
        byt = N * I * 6  # read gate + up, write out (bf16)
        res.append(dict(kernel="swiglu_fwd", N=N, I=I, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
        t = time_it(lambda: native.swiglu_bwd(gu, da, dgu))
        byt = N * I * 10  # read gate, up, d out; write d gate, d up
        res.append(dict(kernel="swiglu_bwd", N=N, I=I, seconds=t, GBps=byt / t / 1e9, frac=byt / t / PEAK_HBM))
    return res


def launch_floor(B=64, H=896, I=4864):
    """Per-call time of tiny kernels replayed back to back from a HIP graph: the launch/dependency floor of a
    decode step, next to the small hand-written decode kernels at B rows."""
    dev, bf = "cuda", torch.bfloat16
    z = torch.zeros(1, device=dev)
    x = torch.randn(B, 1, H, device=dev)
    d = torch.randn(B, 1, H, device=dev, dtype=bf)
    w = torch.ones(H, device=dev)
    y = torch.empty(B, 1, H, device=dev, dtype=bf)
    x2 = torch.empty_like(x)
    gu = torch.randn(B, 2 * I, device=dev, dtype=bf)
    a = torch.empty(B, I, device=dev, dtype=bf)
    res = []
    xs = torch.randn(B, H, device=dev)
    hp = torch.zeros(64 * H, device=dev, dtype=bf)
    for name, fn in [("torch_zero_1elem", lambda: z.zero_()),
                     ("decode_rmsnorm", lambda: native.decode_rmsnorm(xs, None, xs, w, hp, 1e-6, mbt=2)),
                     ("add_rmsnorm_fwd", lambda: native.add_rmsnorm_fwd(x, d, x2, w, y, None, 1e-6)),
                     ("swiglu_fwd", lambda: native.swiglu_fwd(gu, a))]:
        res.append(dict(kernel="graph_floor", op=name, B=B, seconds=time_graph(fn, 200)))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    if args.only == "decode":
        for B in (512, 64):
            for L in (513, 640, 768):
                for r in decode_attn(B=B, L=L):
                    print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "flash":
        for B in (8, 16):
            for r in flash(B=B):
                print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "swiglu":
        for r in swiglu():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "floor":
        for r in launch_floor():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "rope":
        for r in rope() + rope(B=8) + rope(B=256):
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "decode_split":
        for r in decode_split_sweep():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "decode_cold":
        for r in decode_sweep_cold():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "decode_sweep":
        for r in decode_sweep():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "train_gemms":
        for r in train_gemms():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "decode_gemm":
        for r in decode_gemm():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "fused_linear":
        for r in fused_linear():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "flash":
        for r in flash() + flash_bwd():
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only == "k2":
        for r in k2(1024):
            print(json.dumps(r), flush=True)
        sys.exit(0)
    if args.only in ("k1", "k1big"):
        for r in k1_sweep([26] if args.only == "k1big" else [17, 20, 22, 24, 25, 26]):
            print(json.dumps(r), flush=True)
        sys.exit(0)
    exps = [17, 20, 22, 24] if args.quick else [17, 18, 20, 22, 23, 24, 25, 26]
    for r in k1_sweep(exps) + k2(1024 if args.quick else 4096) + adam(1 << 24 if args.quick else 494_032_768):
        print(json.dumps(r), flush=True)
