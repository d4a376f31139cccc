"""Per-call HBM traffic of K1 (drl_ppo_loss_fwd_bwd) from two rocprofv3 PMC passes of `bench.py --k1-only FORM`
-> profiles/pmc_drl_ppo_loss_fwd_bwd[_one_pass].json. One call is the K1a mask pre-pass (two_pass form) + K1b;
the bytes of every dispatch of either kernel are summed and divided by the number of K1b dispatches.
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE doubled for 16-B/lane streaming reads, WRITE_SIZE as is.
Usage: python tools/pmc_k1.py FORM <fetch-dir> <write-dir>"""
import csv
import glob
import json
import os
import sys


def rows(d, counter):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                out.append((r.get("Kernel_Name", ""), float(r["Counter_Value"])))
    if not out:
        raise SystemExit(f"no {counter} rows under {d}")
    return out


def main():
    form, dfetch, dwrite = sys.argv[1:4]
    f, w = rows(dfetch, "FETCH_SIZE"), rows(dwrite, "WRITE_SIZE")
    calls = sum(1 for k, _ in f if "ppo_loss_kernel" in k)
    calls_w = sum(1 for k, _ in w if "ppo_loss_kernel" in k)
    fetch = sum(v for _, v in f) / calls
    write = sum(v for _, v in w) / calls_w
    by_kernel = {}
    for k, v in f:
        name = "mask_pack_kernel" if "mask_pack" in k else "ppo_loss_kernel"
        by_kernel.setdefault(name, [0.0, 0.0])[0] += 2.0 * v * 1024.0 / calls
    for k, v in w:
        name = "mask_pack_kernel" if "mask_pack" in k else "ppo_loss_kernel"
        by_kernel.setdefault(name, [0.0, 0.0])[1] += v * 1024.0 / calls_w
    sym = "drl_ppo_loss_fwd_bwd" + ("_one_pass" if form == "one_pass" else "")
    tokens = 1 << 26
    out = {"symbol": sym, "form": form, "tokens": tokens, "calls": {"fetch_pass": calls, "write_pass": calls_w},
           "fetch_size_kib_per_call_raw": fetch, "write_size_kib_per_call": write,
           "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
           "hbm_bytes_per_token": (2.0 * fetch + write) * 1024.0 / tokens,
           "algorithmic_bytes_per_token": 36,
           "per_kernel_read_write_bytes_per_call": by_kernel,
           "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), WRITE_SIZE as is"}
    os.makedirs("profiles", exist_ok=True)
    with open(os.path.join("profiles", f"pmc_{sym}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
