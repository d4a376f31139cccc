"""Launches drl_gemm (csrc/gemm_sk.hip) on one fused-micro-batch shape for rocprofv3 counter passes:
python tools/probes/sk_probe.py <shape> <reps> [mode param]; shapes at 24576 token rows (Qwen2.5-0.5B)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

T = 24576
SHAPES = {  # kind, M, N, K
    "gate_up_fwd": ("swiglu", T, 9728, 896), "down_fwd": ("fwd", T, 896, 4864), "qkv_fwd": ("fwd", T, 1152, 896),
    "gate_up_dgrad": ("dgrad", T, 896, 9728), "down_dgrad": ("dgrad", T, 4864, 896), "o_dgrad": ("dgrad", T, 896, 896),
    "gate_up_wgrad": ("wgrad", 9728, 896, T), "down_wgrad": ("wgrad", 896, 4864, T), "qkv_wgrad": ("wgrad", 1152, 896, T),
}


def main():
    name, reps = sys.argv[1], int(sys.argv[2])
    if len(sys.argv) > 4:
        native.lib().drl_gemm_set_sk_tuning(0, 0, int(sys.argv[3]), int(sys.argv[4]))
    kind, M, N, K = SHAPES[name]
    bf = torch.bfloat16
    if kind in ("fwd", "swiglu"):
        x = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(N, K, device="cuda", dtype=bf) * 0.05
        fn = lambda: native.linear_fwd(x, w, swiglu=kind == "swiglu")  # noqa: E731
    elif kind == "dgrad":
        dy = torch.randn(M, K, device="cuda", dtype=bf)
        w = torch.randn(K, N, device="cuda", dtype=bf) * 0.05
        fn = lambda: native.linear_dgrad(dy, w)  # noqa: E731
    else:
        dy = torch.randn(K, M, device="cuda", dtype=bf)
        x = torch.randn(K, N, device="cuda", dtype=bf)
        gw = torch.zeros(M, N, device="cuda")
        fn = lambda: native.linear_wgrad(gw, dy, x)  # noqa: E731
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
