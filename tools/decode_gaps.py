"""Decode-step anatomy from a rocprofv3 kernel_trace.csv: steps are delimited by the K4 selection kernel that
ends each decode step; per step, wall time (end of one selection to the end of the next), kernel-busy time and
launch count, then each kernel's mean duration per step. Usage: python tools/decode_gaps.py trace.csv"""
import collections
import csv
import statistics
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, (_, _, n) in enumerate(rows) if "select_pick_kernel" in n or "select_finish_kernel" in n]
    walls, busy, counts = [], [], []
    per = collections.defaultdict(list)
    for a, b in zip(ends, ends[1:]):
        seg = rows[a + 1:b + 1]
        if len(seg) > 400:  # not consecutive decode steps (a prefill or training phase in between)
            continue
        walls.append(rows[b][1] - rows[a][1])
        busy.append(sum(e - s for s, e, _ in seg))
        counts.append(len(seg))
        step = collections.defaultdict(int)
        for s, e, n in seg:
            step[n.replace("(anonymous namespace)::", "").split("(")[0][:90]] += e - s
        for n, d in step.items():
            per[n].append(d)
    nsteps = len(walls)
    if not walls:
        print("no decode steps found")
        return
    w, bsy = statistics.median(walls), statistics.median(busy)
    print(f"decode steps: {len(walls)}  median wall {w / 1e3:.1f} us  kernel-busy {bsy / 1e3:.1f} us "
          f"({bsy / w:.0%})  launches/step {statistics.median(counts):.0f}")
    for n, ds in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {sum(ds) / nsteps / 1e3:8.1f} us/step (in {len(ds)} of {nsteps} steps)  {n}")


if __name__ == "__main__":
    main()
