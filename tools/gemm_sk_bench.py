"""drl_gemm (csrc/gemm_sk.hip) vs hipBLASLt on every GEMM of the actor's passes at config #2 (Qwen2.5-0.5B):
forward (y = x W^T), dgrad (dx = dy W) and wgrad (dW += dy^T x, fp32) of qkv / o / gate_up / down at the update
(8 x 768) and log-prob (16 x 768) micro-batch rows, and the lm_head over the response rows. One JSON line per
shape: microseconds and TFLOP/s of both, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).

  python tools/gemm_sk_bench.py [--quick] [--tune] [--groups 1 2 4 8]

The first shape a process times runs ~10-15 % slow (clocks / caches still cold: ours_us of the first shape against
its own --groups / --tune entries, profiles/r04_decode_lm_head_sweep.jsonl); compare a shape's entries with each other.
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dots.rl_amd import native  # noqa: E402


def bench(fn, iters=20, warmup=3, rounds=3):
    for _ in range(warmup):
        fn()
    best = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        best.append(a.elapsed_time(b) * 1e3 / iters)
    best.sort()
    return best[len(best) // 2]


def shapes(quick, rows=None, decode=None):
    H, I, NQ, V = 896, 4864, 1152, 151936
    out = []
    if decode:  # the decode step's projections at `decode` rows (one token per sequence)
        M = decode
        return [("dec_qkv", "fwd", M, NQ, H), ("dec_o", "fwd", M, H, H), ("dec_gate_up_swiglu", "swiglu", M, 2 * I, H),
                ("dec_down", "fwd", M, H, I), ("dec_lm_head", "fwd", M, V, H)]
    train = rows or [6144]
    for M in sorted(set(train + ([] if quick else [12288]))):
        out += [("qkv_fwd", "fwd", M, NQ, H), ("o_fwd", "fwd", M, H, H), ("gate_up_fwd_swiglu", "swiglu", M, 2 * I, H),
                ("down_fwd", "fwd", M, H, I)]
        if M in train:
            out += [("qkv_dgrad", "dgrad", M, H, NQ), ("o_dgrad", "dgrad", M, H, H), ("gate_up_dgrad", "dgrad", M, H, 2 * I),
                    ("down_dgrad", "dgrad", M, I, H), ("down_dgrad_swiglu_bwd", "dgrad_swiglu", M, I, H),
                    ("qkv_wgrad", "wgrad", NQ, H, M), ("o_wgrad", "wgrad", H, H, M),
                    ("gate_up_wgrad", "wgrad", 2 * I, H, M), ("down_wgrad", "wgrad", H, I, M)]
    R = (max(train) // 768) * 256  # response rows of the pass (256 of every 768-token sequence)
    out += [("lm_head_fwd", "fwd", R, V, H), ("lm_head_dgrad", "dgrad", R, H, V), ("lm_head_wgrad", "wgrad", V, H, R)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--tune", action="store_true", help="also sweep grid / dp_mode / group of drl_gemm")
    ap.add_argument("--rows", type=int, nargs="*", default=None, help="token rows of the training passes")
    ap.add_argument("--no-lib", action="store_true", help="skip the hipBLASLt timing")
    ap.add_argument("--decode", type=int, default=None, help="only the decode-step shapes at this many rows")
    ap.add_argument("--only", nargs="*", default=None, help="only these shape names (e.g. gate_up_wgrad o_wgrad)")
    ap.add_argument("--groups", type=int, nargs="*", default=None, help="also time these rasterization groups")
    args = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    for name, kind, M, N, K in shapes(args.quick, args.rows, args.decode):
        if args.only and name not in args.only:
            continue
        fl = 2.0 * M * N * K
        if kind in ("fwd", "swiglu") and args.decode:
            # decode: weights rotate over > 600 MB of copies (each call streams W from HBM, as in the step)
            x = torch.randn(M, K, generator=g, device=dev).to(bf)
            nc = max(2, int(600e6 // (N * K * 2)) + 1)
            ws = [(torch.randn(N, K, generator=g, device=dev) * 0.05).to(bf) for _ in range(nc)]
            sw = kind == "swiglu"
            a = torch.empty(M, N // 2, device=dev, dtype=bf)
            ctr = iter(range(1 << 40))
            ours = lambda: native.linear_fwd(x, ws[next(ctr) % nc], swiglu=sw)  # noqa: E731
            lib = ((lambda: native.swiglu_fwd(x @ ws[next(ctr) % nc].t(), a)) if sw
                   else (lambda: x @ ws[next(ctr) % nc].t()))  # noqa: E731
        elif kind in ("fwd", "swiglu"):
            x = torch.randn(M, K, generator=g, device=dev).to(bf)
            w = (torch.randn(N, K, generator=g, device=dev) * 0.05).to(bf)
            sw = kind == "swiglu"
            a = torch.empty(M, N // 2, device=dev, dtype=bf)
            ours = lambda: native.linear_fwd(x, w, swiglu=sw)  # noqa: E731
            lib = (lambda: native.swiglu_fwd(x @ w.t(), a)) if sw else (lambda: x @ w.t())  # noqa: E731
        elif kind == "dgrad_swiglu":  # da (M, N) = dy (M, K) @ Wd (K, N), then the SwiGLU backward into dgu (M, 2N)
            dy = torch.randn(M, K, generator=g, device=dev).to(bf)
            w = (torch.randn(K, N, generator=g, device=dev) * 0.05).to(bf)
            gu = torch.randn(M, 2 * N, generator=g, device=dev).to(bf)
            ours = lambda: native.linear_dgrad_swiglu_bwd(dy, w, gu)  # noqa: E731
            lib = lambda: native.swiglu_bwd(gu, dy @ w, torch.empty_like(gu))  # noqa: E731
        elif kind == "dgrad":  # dx (M, N) = dy (M, K) @ W (K, N)
            dy = torch.randn(M, K, generator=g, device=dev).to(bf)
            w = (torch.randn(K, N, generator=g, device=dev) * 0.05).to(bf)
            ours = lambda: native.linear_dgrad(dy, w)  # noqa: E731
            lib = lambda: dy @ w  # noqa: E731
        else:  # gw (M=out, N=in) += dy^T x, dy (K, M), x (K, N)
            dy = torch.randn(K, M, generator=g, device=dev).to(bf)
            x = torch.randn(K, N, generator=g, device=dev).to(bf)
            gw = torch.zeros(M, N, device=dev)
            ours = lambda: native.linear_wgrad(gw, dy, x)  # noqa: E731
            lib = lambda: torch.addmm(gw, dy.t(), x, out_dtype=torch.float32, out=gw)  # noqa: E731
        row = dict(shape=name, M=M, N=N, K=K)
        t_lib = float("nan") if args.no_lib else bench(lib)
        t_ours = bench(ours)
        row.update(hipblaslt_us=t_lib, hipblaslt_TF=fl / t_lib / 1e6, ours_us=t_ours, ours_TF=fl / t_ours / 1e6)
        if args.tune:
            sweep = {}
            for grid, mode, param in [(0, 1, 0), (0, 1, 8), (0, 1, 32), (0, 2, 0), (0, 3, 2), (0, 3, 3), (0, 3, 4),
                                      (0, 3, 5), (0, 3, 6), (0, 3, 8), (0, 3, 10), (0, 3, 12), (0, 3, 16), (0, 3, 32)]:
                if mode == 3 and param and param * ((M + 255) // 256) * ((N + 255) // 256) > 256:
                    continue
                native.lib().drl_gemm_set_sk_tuning(grid, 0, mode, param)
                sweep[f"g{grid}_m{mode}_p{param}"] = round(bench(ours, iters=10, rounds=2), 2)
            native.lib().drl_gemm_set_sk_tuning(0, 0, 0, 0)
            row["sweep_us"] = sweep
        if args.groups:
            row["group_us"] = {}
            for gm in args.groups:
                native.lib().drl_gemm_set_sk_tuning(0, gm, 0, 0)
                row["group_us"][gm] = round(bench(ours, iters=10, rounds=3), 2)
            native.lib().drl_gemm_set_sk_tuning(0, 0, 0, 0)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
