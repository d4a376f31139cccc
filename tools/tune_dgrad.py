"""TunableOp search (hipBLASLt + rocBLAS solutions) for the update's dgrad in both call forms at the update
micro-batch rows: NN dy @ W and TN dy @ (W^T)^T with the transposed weight copy (Qwen2Model.wt). Prints the tuned
time of each form per layer; writes the merged results file to --out.
Usage (GPU box): python tools/tune_dgrad.py --out gpurun_out/tunableop_dgrad.csv"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--rows", type=int, default=6144)
    args = ap.parse_args()
    import torch.cuda.tunable as tunable

    from dots.rl_amd.workers import _TUNING_FILE

    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(os.path.abspath(args.out), insert_device_ordinal=False)
    tunable.read_file(_TUNING_FILE)
    bf = torch.bfloat16
    M = args.rows
    for name, N, K in (("qkv", 1152, 896), ("o", 896, 896), ("gate_up", 9728, 896), ("down", 896, 4864)):
        w = torch.randn(N, K, device="cuda", dtype=bf)
        wt = w.t().contiguous()
        dy = torch.randn(M, N, device="cuda", dtype=bf)
        for _ in range(2):
            dy @ w
            dy @ wt.t()
        torch.cuda.synchronize()
    for r in tunable.get_results():  # (op, shape key, solution, ms)
        if f"_{M}_" in str(r[1]):
            print(r)


if __name__ == "__main__":
    main()
