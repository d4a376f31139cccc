"""Mean per-dispatch SQ counters by kernel from rocprofv3 --pmc counter_collection.csv files (one directory per
pass), with the derived ratios the flash / GEMM notes quote (VALU and LDS instructions per MFMA, the share of wave
cycles spent waiting). usage: python tools/pmc_sq.py <out.json> <kernel substring>[,<substring>...] <pass dir>..."""
import collections
import csv
import glob
import json
import sys


def main():
    out, names, dirs = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = next((n for n in names if n in r["Kernel_Name"]), None)
                if k is not None:
                    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        mean = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
        d = {"dispatches": max(len(v) for v in cs.values()), "counters_mean_per_dispatch": mean}
        mf = mean.get("SQ_INSTS_MFMA")
        if mf:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in mean:
                    d[c.replace("SQ_INSTS_", "").lower() + "_per_mfma"] = round(mean[c] / mf, 2)
        if mean.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in mean:
                    d[c.lower() + "_frac_of_wave_cycles"] = round(mean[c] / mean["SQ_WAVE_CYCLES"], 3)
        res[k] = d
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: {x: y for x, y in v.items() if x != "counters_mean_per_dispatch"} for k, v in res.items()}))


if __name__ == "__main__":
    main()
