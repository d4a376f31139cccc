"""Launches the ping-pong projection GEMM (csrc/gemm.hip, tile 9) on one model shape for counter passes:
python tools/probes/gemm_probe.py <shape> <reps>, shape in lm_head | gate_up | down."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

from dots.rl_amd import native  # noqa: E402

SHAPES = {"lm_head": (4096, 151936, 896, False), "gate_up": (12288, 9728, 896, True), "down": (12288, 896, 4864, False)}


def main():
    name, reps = sys.argv[1], int(sys.argv[2])
    M, N, K, sw = SHAPES[name]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    native.lib().drl_gemm_set_tile(9)
    for _ in range(reps):
        native.gemm_nt(x, w, swiglu=sw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
