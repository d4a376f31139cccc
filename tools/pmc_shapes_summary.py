"""Per-shape HBM traffic of drl_gemm from the two PMC passes over tools/probes/pmc_shapes.py (FETCH_SIZE x 2 +
WRITE_SIZE per dispatch, the gfx950 correction of tools/pmc_traffic.py), against each shape's algorithmic bytes.
python tools/pmc_shapes_summary.py <probe stdout json> <fetch dir> <write dir> <kernel_trace csv> > out.json"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                rows.append((int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))), float(r["Counter_Value"])))
    rows.sort()
    return [v for _, v in rows]


def durations(path):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
                  if "gemm_sk_kernel" in r["Kernel_Name"])
    return [(e - s) / 1e3 for s, e in rows]


def main():
    meta = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
    f, w = per_dispatch(sys.argv[2], "FETCH_SIZE"), per_dispatch(sys.argv[3], "WRITE_SIZE")
    dur = durations(sys.argv[4]) if len(sys.argv) > 4 else []
    reps = meta["reps"]
    out = []
    for i, sh in enumerate(meta["shapes"]):
        idx = range(i * reps + 1, (i + 1) * reps)  # the first of each shape warms
        fb = sum(f[j] for j in idx) / len(idx) * 1024 * 2
        wb = sum(w[j] for j in idx) / len(idx) * 1024
        row = dict(sh, hbm_bytes=fb + wb, fetch_bytes=fb, write_bytes=wb, ratio=(fb + wb) / sh["algorithmic_bytes"])
        if dur:
            us = sum(dur[j] for j in idx) / len(idx)
            row.update(us=us, tflops=sh["flop"] / us / 1e6)
        out.append(row)
    print(json.dumps({"source": "FETCH_SIZE x 2 + WRITE_SIZE per dispatch (tools/probes/pmc_shapes.py, 82144 rows)",
                      "shapes": out}, indent=1))


if __name__ == "__main__":
    main()
