"""Summarise a rocprofv3 --kernel-trace CSV of a decode run: for the decode steps (the launches after
the prefill), per kernel the mean in-step duration and the mean idle gap before it (end of the
previous kernel to its start), and the step's span vs the sum of its kernel durations.

    python tools/trace_gaps.py gpurun_out/r5_trace/c3
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "at::" not in r["Kernel_Name"] and "k_pack_w" not in r["Kernel_Name"]]
    # decode steps start at each k_embed_ln launched with one position per row (after the prefill)
    starts = [i for i, r in enumerate(rows) if "k_embed_ln" in r["Kernel_Name"]]
    starts = starts[len(starts) // 4:]                 # skip the first quarter (warm-up, prefill)
    dur, gap = defaultdict(list), defaultdict(list)
    spans, sums = [], []
    for a, b in zip(starts, starts[1:]):
        seg = rows[a:b]
        spans.append((int(rows[b]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3)
        sums.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3)
        for j, r in enumerate(seg):
            n = short(r["Kernel_Name"])
            dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            prev = rows[a + j - 1]
            gap[n].append((int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
    ns = len(spans)
    print(f"{d}: {ns} decode steps, span {sum(spans) / ns:.1f} us, kernel sum {sum(sums) / ns:.1f} us, "
          f"gaps {(sum(spans) - sum(sums)) / ns:.1f} us per step")
    print(f"{'kernel':60s} {'n/step':>6s} {'dur us':>8s} {'gap us':>8s} {'us/step':>8s}")
    for n in sorted(dur, key=lambda k: -sum(dur[k])):
        c = len(dur[n]) / ns
        print(f"{n:60s} {c:6.1f} {sum(dur[n]) / len(dur[n]):8.2f} {sum(gap[n]) / len(gap[n]):8.2f} "
              f"{sum(dur[n]) / ns:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
