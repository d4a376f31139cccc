"""Summarise a rocprofv3 kernel_trace.csv (or .csv.gz): for the kernels with the most total time, the distinct launch
shapes (grid x workgroup) with call counts and mean duration, and how much of each kernel's time other kernels ran
beside it (the concurrent streams of the update pass: a kernel's in-situ duration then includes sharing the chip).
Usage: python tools/trace_summary.py trace.csv [N]"""
import collections
import csv
import gzip
import sys


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def overlapped(sel):
    """sel: sorted (start, end, name) -> {name: ns during which at least one other kernel was running}"""
    ev = []
    for i, (a, b, _) in enumerate(sel):
        ev.append((a, 1, i))
        ev.append((b, 0, i))  # ends before starts at equal timestamps
    ev.sort()
    shared = collections.Counter()
    active, prev = set(), None
    for t, kind, i in ev:
        if prev is not None and len(active) >= 2 and t > prev:
            for j in active:
                shared[sel[j][2]] += t - prev
        prev = t
        if kind:
            active.add(i)
        else:
            active.discard(i)
    return shared


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    tot = collections.Counter()
    shapes = collections.defaultdict(collections.Counter)
    durs = collections.defaultdict(float)
    for r in csv.DictReader(_open(path)):
        name = r["Kernel_Name"]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[name] += d
        key = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
               r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))
        shapes[name][key] += 1
        durs[(name, key)] += d
    # GPU idle time: the union of every kernel interval against the trace's span, and the longest gaps between
    # consecutive busy intervals (host-bound stretches: launches behind a synchronisation)
    rows = list(csv.DictReader(_open(path)))
    # bench.py with DRL_TRACE_MARK=1 brackets its timed steps with two spin kernels: the window between them
    marks = sorted(int(r["End_Timestamp"]) for r in rows if "spin_kernel" in r["Kernel_Name"])
    lo, hi = (marks[0], marks[-1]) if len(marks) >= 2 else (0, 1 << 62)
    sel = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
                  if lo <= int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= hi
                  and "spin_kernel" not in r["Kernel_Name"]))
    iv = [(a, b) for a, b, _ in sel]
    names = {}  # end timestamp of a busy stretch -> (last kernel of it, first kernel after the gap)
    if len(marks) >= 2:
        print(f"window: the timed steps between the two DRL_TRACE_MARK spin kernels ({(hi - lo) / 1e6:.1f} ms)")
    if iv:
        busy, gaps, cs, ce, cn = 0, [], iv[0][0], iv[0][1], sel[0][2]
        for a, b, nm in sel[1:]:
            if a > ce:
                busy += ce - cs
                gaps.append((a - ce, ce))
                names[ce] = (cn, nm)
                cs, ce, cn = a, b, nm
            else:
                if b >= ce:
                    cn = nm
                ce = max(ce, b)
        busy += ce - cs
        span = iv[-1][1] - iv[0][0]
        gaps.sort(reverse=True)
        idle = span - busy
        print(f"span {span / 1e6:.1f} ms, GPU busy (union of kernels) {busy / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms "
              f"({100.0 * idle / span:.1f} %) in {len(gaps)} gaps; gaps > 50 us: "
              f"{sum(g for g, _ in gaps if g > 50000) / 1e6:.1f} ms in {sum(1 for g, _ in gaps if g > 50000)}; "
              f"longest {[round(g / 1e3, 1) for g, _ in gaps[:8]]} us")
        # a gap of seconds is not a step's idle time: the first barrier of a run builds the communicator (older
        # bench.py versions marked the window before it); report the idle net of such gaps beside the raw figure
        big = sum(g for g, _ in gaps if g > 1_000_000_000)
        if big:
            print(f"net of {sum(1 for g, _ in gaps if g > 1_000_000_000)} gap(s) > 1 s (communicator setup): span "
                  f"{(span - big) / 1e6:.1f} ms, idle {(idle - big) / 1e6:.1f} ms ({100.0 * (idle - big) / (span - big):.1f} %)")
        short = lambda n: n.replace("void ", "").replace("drl::(anonymous namespace)::", "")[:60]  # noqa: E731
        for g, at in gaps[:16]:
            before, after = names[at]
            print(f"  gap {g / 1e3:9.1f} us at {(at - lo) / 1e6 if lo else at / 1e6:9.1f} ms: after {short(before)} | "
                  f"before {short(after)}")
    if len(marks) >= 2:
        # per-kernel totals over the window only (the trace also holds the warmup steps and the setup)
        tot = collections.Counter()
        shapes = collections.defaultdict(collections.Counter)
        durs = collections.defaultdict(float)
        for r in rows:
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if not (lo <= a and b <= hi) or "spin_kernel" in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            key = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
                   r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))
            tot[name] += b - a
            shapes[name][key] += 1
            durs[(name, key)] += b - a
        print("per-kernel totals below: inside the window only")
    shared = overlapped(sel) if len(marks) >= 2 and sel else collections.Counter()
    if shared:
        print(f"kernel time beside another kernel (concurrent streams): {sum(shared.values()) / 1e6:.1f} ms of "
              f"{sum(tot.values()) / 1e6:.1f} ms")
    for name, t in tot.most_common(top):
        ov = f"  ({100.0 * shared[name] / t:.0f} % of it beside another kernel)" if shared.get(name) else ""
        print(f"{t / 1e6:9.1f} ms  {name[:110]}{ov}")
        for key, n in shapes[name].most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 6):
            print(f"      grid={key[0]}x{key[1]} wg={key[2]}  calls={n}  mean={durs[(name, key)] / n / 1e3:.1f} us")


if __name__ == "__main__":
    main()
