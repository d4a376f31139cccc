"""drl_gemm (csrc/gemm_sk.hip) on each shape class of config #2's update pass (82144 token rows, Qwen2.5-0.5B) for
rocprofv3 counter passes: every shape REPS times in a fixed order (SHAPES), so dispatch i belongs to shape i // REPS
(each shape is one launch). The summary (tools/pmc_shapes_summary.py) pairs them with the algorithmic bytes.
python tools/probes/pmc_shapes.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

T = 82144
H, I, NQ = 896, 4864, 1152
REPS = 3
# name, kind, M, N, K (kind: fwd / swiglu / dgrad / dgrad_swiglu / wgrad)
SHAPES = [
    ("qkv_fwd", "bias", T, NQ, H), ("o_fwd", "fwd", T, H, H), ("gate_up_fwd", "swiglu", T, 2 * I, H),
    ("down_fwd", "fwd", T, H, I),
    ("qkv_dgrad", "dgrad", T, H, NQ), ("o_dgrad", "dgrad", T, H, H), ("gate_up_dgrad", "dgrad", T, H, 2 * I),
    ("down_dgrad_swiglu", "dgrad_swiglu", T, I, H),
    ("qkv_wgrad", "wgrad", NQ, H, T), ("o_wgrad", "wgrad", H, H, T), ("gate_up_wgrad", "wgrad", 2 * I, H, T),
    ("down_wgrad", "wgrad", H, I, T),
]


def algorithmic_bytes(kind, M, N, K):
    """A + B read once, C written once (fp32 wgrad: read + written, beta = 1); SwiGLU: the I-wide output plus the
    saved [gate | up]; the SwiGLU backward reads gu (M, 2N) and writes dgu (M, 2N)."""
    ab = 2 * (M * K + N * K)
    if kind == "wgrad":
        return ab + 8 * M * N
    if kind == "swiglu":
        return ab + 2 * M * (N // 2) + 2 * M * N
    if kind == "dgrad_swiglu":
        return ab + 2 * 2 * M * (2 * N)
    return ab + 2 * M * N


def main():
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g).to(bf)  # noqa: E731
    meta = []
    for name, kind, M, N, K in SHAPES:
        if kind in ("fwd", "bias", "swiglu"):
            x, w = rnd(M, K), rnd(N, K) * 0.05
            b = rnd(N) if kind == "bias" else None
            gu = torch.empty(M, N, dtype=bf, device="cuda") if kind == "swiglu" else None
            fn = lambda x=x, w=w, b=b, gu=gu, kind=kind: native.linear_fwd(x, w, bias=b, swiglu=kind == "swiglu",  # noqa: E731
                                                                           out_gu=gu)
        elif kind == "dgrad":
            dy, w = rnd(M, K), rnd(K, N) * 0.05
            fn = lambda dy=dy, w=w: native.linear_dgrad(dy, w)  # noqa: E731
        elif kind == "dgrad_swiglu":
            dy, w, gu = rnd(M, K), rnd(K, N) * 0.05, rnd(M, 2 * N)
            fn = lambda dy=dy, w=w, gu=gu: native.linear_dgrad_swiglu_bwd(dy, w, gu)  # noqa: E731
        else:
            dy, x = rnd(K, M), rnd(K, N)
            gw = torch.zeros(M, N, device="cuda")
            fn = lambda dy=dy, x=x, gw=gw: native.linear_wgrad(gw, dy, x)  # noqa: E731
        for _ in range(REPS):
            fn()
        torch.cuda.synchronize()
        meta.append({"shape": name, "kind": kind, "M": M, "N": N, "K": K, "plan": list(native.gemm_plan(M, N, K, {
            "swiglu": 2, "bias": 1, "dgrad_swiglu": 3}.get(kind, 0))), "algorithmic_bytes": algorithmic_bytes(kind, M, N, K),
                     "flop": 2 * M * N * K})
        del fn
        torch.cuda.empty_cache()
    print(json.dumps({"reps": REPS, "shapes": meta}), flush=True)


if __name__ == "__main__":
    main()
