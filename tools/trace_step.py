"""Decode-step anatomy from a rocprofv3 --kernel-trace CSV: per-kernel average duration, the gap
before each launch (previous kernel's end -> this start), and the busy / gap totals per step.
    python tools/trace_step.py <run_kernel_trace.csv> [--last N_STEPS]
A decode step is delimited by the k_eos_step launch; steps are taken from the last --last of the trace."""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 50
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "k_eos_step" in r[2]]
    # decode steps: between consecutive eos launches
    steps = [(ends[j - 1] + 1, ends[j] + 1) for j in range(1, len(ends))]
    steps = steps[-last:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    busy_t, gap_t, wall_t = 0, 0, 0
    seq = None
    for a, b in steps:
        names = []
        for i in range(a, b):
            s, e, n = rows[i]
            pos = i - a
            key = (pos, n)
            names.append(n)
            dur[key].append(e - s)
            if i > a:
                gap[key].append(s - rows[i - 1][1])
            busy_t += e - s
            if i > a:
                gap_t += max(0, s - rows[i - 1][1])
        wall_t += rows[b - 1][1] - rows[a][0]
        seq = names
    ns = len(steps)
    print(f"steps {ns}, launches/step {len(seq)}; per step: wall {wall_t / ns / 1e3:.1f} us, "
          f"busy {busy_t / ns / 1e3:.1f} us, gaps {gap_t / ns / 1e3:.1f} us")
    agg = defaultdict(lambda: [0, 0, 0.0, 0.0])
    for (pos, n), v in dur.items():
        g = gap.get((pos, n), [0])
        a = agg[n]
        a[0] += 1
        a[1] += len(v)
        a[2] += sum(v) / len(v)
        a[3] += sum(g) / len(g)
    print(f"{'kernel':70s} {'n/step':>6s} {'us each':>8s} {'us/step':>8s} {'gap us':>7s}")
    for n, (k, cnt, tot, gtot) in sorted(agg.items(), key=lambda x: -x[1][2]):
        print(f"{n:70s} {k:6d} {tot / k / 1e3:8.2f} {tot / 1e3:8.1f} {gtot / k / 1e3:7.2f}")
    if "--seq" in sys.argv:
        for pos, n in enumerate(seq[:40]):
            d = dur[(pos, n)]
            g = gap.get((pos, n), [0])
            print(f"{pos:3d} {n:60s} {sum(d) / len(d) / 1e3:7.2f} gap {sum(g) / len(g) / 1e3:5.2f}")


if __name__ == "__main__":
    main()
