"""Weight-gradient GEMM forms on MI355X for the update micro-batch (M = 8 x 768 tokens): which call form gets
hipBLASLt / rocBLAS onto a fast kernel. dW (N, K) fp32 += dy^T (N, M) x (M, K) with bf16 operands.
  v1: torch.addmm(gw, dy.t(), x, out_dtype=fp32, out=gw)         (current: fp32 output, beta = 1)
  v2: bf16 torch.mm(dy.t(), x) (TunableOp-tuned here) + gw.add_   (bf16-rounded per-micro-batch dW, the
      reference's autocast numerics, then fp32 accumulation)
  v3: torch.addmm(gw.t(), x.t(), dy, out_dtype=fp32, out=gw.t())  (transposed problem, same math as v1)
Usage (GPU box): python tools/dw_probe.py
"""

import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_bench import time_it  # noqa: E402


def main():
    import torch.cuda.tunable as tunable

    from dots.rl_amd.workers import _TUNING_FILE

    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(os.path.join(tempfile.gettempdir(), "dw_probe_tunableop.csv"), insert_device_ordinal=False)
    tunable.read_file(_TUNING_FILE)
    dev, bf = "cuda", torch.bfloat16
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 6144
    for name, N, K in (("qkv", 1152, 896), ("o_proj", 896, 896), ("gate_up", 9728, 896), ("down", 896, 4864)):
        x = torch.randn(M, K, device=dev, dtype=bf)
        dy = torch.randn(M, N, device=dev, dtype=bf)
        gw = torch.zeros(N, K, device=dev)
        fl = 2.0 * M * N * K
        t1 = time_it(lambda: torch.addmm(gw, dy.t(), x, out_dtype=torch.float32, out=gw))
        for _ in range(2):
            torch.mm(dy.t(), x)  # tune
        torch.cuda.synchronize()
        t2m = time_it(lambda: torch.mm(dy.t(), x))
        t2 = time_it(lambda: gw.add_(torch.mm(dy.t(), x)))
        gwt = gw.t()
        t3 = time_it(lambda: torch.addmm(gwt, x.t(), dy, out_dtype=torch.float32, out=gwt))
        # v4: explicit transposed copies, then the forward's layout (reduction dim contiguous in both operands)
        t4 = time_it(lambda: torch.addmm(gw, dy.t().contiguous(), x.t().contiguous().t(), out_dtype=torch.float32,
                                         out=gw))
        dyt, xt = dy.t().contiguous(), x.t().contiguous()
        t4g = time_it(lambda: torch.addmm(gw, dyt, xt.t(), out_dtype=torch.float32, out=gw))
        t4b = time_it(lambda: torch.mm(dyt, xt.t()))
        print(json.dumps(dict(layer=name, M=M, N=N, K=K, v1_us=t1 * 1e6, v1_TF=fl / t1 / 1e12, v2_mm_us=t2m * 1e6,
                              v2_us=t2 * 1e6, v2_TF=fl / t2 / 1e12, v3_us=t3 * 1e6, v3_TF=fl / t3 / 1e12, v4_us=t4 * 1e6,
                              v4_gemm_us=t4g * 1e6, v4_bf16_gemm_us=t4b * 1e6)), flush=True)
    print("\n".join(",".join(map(str, r)) for r in tunable.get_results()), file=sys.stderr)


if __name__ == "__main__":
    main()
