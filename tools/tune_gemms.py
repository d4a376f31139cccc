"""Offline GEMM tuning for the decode-step shapes of a DP rank (PyTorch TunableOp on hipBLASLt / rocBLAS).

The shipped results file (dots.rl_amd/tuning/tunableop_gfx950.csv) is replayed read-only at run time
(workers._enable_gemm_tuning). This script loads it, tunes the decode projections and lm_head at the token
rows a rank decodes with at 1/2/4/8 GPUs (global batch 512 -> 512/256/128/64 rows), in the exact call forms
the model uses (so the TunableOp keys match), and writes the merged file to --out.merged (--out receives TunableOp's own dump of this run).
Usage (GPU box): python tools/tune_gemms.py --out gpurun_out/tunableop_gfx950.csv
"""

import argparse
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--rows", default="64,128,256,512")
    args = ap.parse_args()
    import torch.cuda.tunable as tunable

    from dots.rl_amd.workers import _TUNING_FILE

    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(os.path.abspath(args.out), insert_device_ordinal=False)
    tunable.read_file(_TUNING_FILE)
    dev, bf = "cuda", torch.bfloat16
    H, I, V, QKV = 896, 4864, 151936, 1152
    w_qkv = torch.randn(QKV, H, device=dev, dtype=bf)
    b_qkv = torch.randn(QKV, device=dev, dtype=bf)
    w_o = torch.randn(H, H, device=dev, dtype=bf)
    w_gu = torch.randn(2 * I, H, device=dev, dtype=bf)
    w_dn = torch.randn(H, I, device=dev, dtype=bf)
    emb = torch.randn(V, H, device=dev, dtype=bf)
    for M in [int(m) for m in args.rows.split(",")]:
        h = torch.randn(M, H, device=dev, dtype=bf)
        a = torch.randn(M, I, device=dev, dtype=bf)
        for _ in range(2):
            torch.addmm(b_qkv, h, w_qkv.t())  # qkv_proj (qwen2._layer_forward)
            h @ w_o.t()  # o_proj
            h @ w_gu.t()  # gate_up_proj
            a @ w_dn.t()  # down_proj
            F.linear(h, emb)  # lm_head (tied embedding, Qwen2Model.logits)
        torch.cuda.synchronize()
        print(f"tuned rows={M}", flush=True)
    # merged file: the shipped validators + results, then every result of this process not already there
    shipped = open(_TUNING_FILE).read().splitlines()
    keys = {tuple(line.split(",")[:2]) for line in shipped}
    new = [",".join(str(v) for v in r) for r in tunable.get_results() if tuple(map(str, r[:2])) not in keys]
    with open(args.out + ".merged", "w") as f:
        f.write("\n".join(shipped + new) + "\n")
    print("\n".join(new))


if __name__ == "__main__":
    main()
