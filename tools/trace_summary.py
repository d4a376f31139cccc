"""Summarise a rocprofv3 kernel_trace.csv: for the kernels with the most total time, the distinct launch
shapes (grid x workgroup) with call counts and mean duration. Usage: python tools/trace_summary.py trace.csv [N]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    tot = collections.Counter()
    shapes = collections.defaultdict(collections.Counter)
    durs = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[name] += d
        key = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
               r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))
        shapes[name][key] += 1
        durs[(name, key)] += d
    for name, t in tot.most_common(top):
        print(f"{t / 1e6:9.1f} ms  {name[:110]}")
        for key, n in shapes[name].most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 6):
            print(f"      grid={key[0]}x{key[1]} wg={key[2]}  calls={n}  mean={durs[(name, key)] / n / 1e3:.1f} us")


if __name__ == "__main__":
    main()
