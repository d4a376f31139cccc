"""Per-launch HBM traffic of one kernel from two rocprofv3 PMC passes -> profiles/pmc_<symbol>.json.

Recipe (MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots): FETCH_SIZE and WRITE_SIZE cannot share a
pass, so run the benchmark twice with counter collection restricted to the kernel, e.g.

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex masked_softmax_fwd -f csv -d gpurun_out/pmc_f -o f \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
  rocprofv3 --pmc WRITE_SIZE --kernel-include-regex masked_softmax_fwd -f csv -d gpurun_out/pmc_w -o w \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline
  python tools/pmc_traffic.py drl_masked_softmax_fwd gpurun_out/pmc_f gpurun_out/pmc_w

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. gfx950 correction: FETCH_SIZE counts half the bytes of
wide (16 B/lane) coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B stores.
"""

import csv
import glob
import json
import os
import sys


def _per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                vals.append((row.get("Kernel_Name", ""), float(row["Counter_Value"])))
    if not vals:
        raise SystemExit(f"counter {counter} not found in {files}")
    return vals


def main():
    symbol, dfetch, dwrite = sys.argv[1:4]
    f = _per_dispatch(dfetch, "FETCH_SIZE")
    w = _per_dispatch(dwrite, "WRITE_SIZE")
    fetch_kib = sum(v for _, v in f) / len(f)
    write_kib = sum(v for _, v in w) / len(w)
    out = {
        "symbol": symbol,
        "kernel_names": sorted({k for k, _ in f})[:4],
        "dispatches": {"fetch_pass": len(f), "write_pass": len(w)},
        "fetch_size_kib_per_launch_raw": fetch_kib,
        "write_size_kib_per_launch": write_kib,
        "hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), WRITE_SIZE as is",
    }
    os.makedirs("profiles", exist_ok=True)
    path = os.path.join("profiles", f"pmc_{symbol}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
