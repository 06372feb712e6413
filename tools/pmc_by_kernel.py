"""Per-kernel HBM bytes from rocprofv3 --pmc passes (one counter per pass): FETCH_SIZE (x2, the gfx950
correction for 16-B streaming reads, MI355X_MICROARCH.md) and WRITE_SIZE, mean per dispatch of each
(kernel, grid), in MB. Developer tool.
    python tools/pmc_by_kernel.py FETCH_DIR WRITE_DIR [--match NAME]"""
import argparse
import csv
import glob
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("fetch")
ap.add_argument("write")
ap.add_argument("--match", default="")
a = ap.parse_args()


def load(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r.get("Kernel_Name", "?").replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if a.match in name:
                acc[(name, r.get("Grid_Size", "?"))].append(float(r["Counter_Value"]))
    return acc


fe, wr = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
for k in sorted(set(fe) | set(wr), key=lambda k: -sum(fe.get(k, [0])) * 2):
    f = 2 * sum(fe.get(k, [0])) / max(1, len(fe.get(k, [1]))) * 1024 / 1e6     # FETCH_SIZE is in KB
    w = sum(wr.get(k, [0])) / max(1, len(wr.get(k, [1]))) * 1024 / 1e6
    print(f"{k[0][-70:]:70s} grid {k[1]:>9s} n={len(fe.get(k, [])):3d}  fetch {f:9.2f} MB  write {w:9.2f} MB")
