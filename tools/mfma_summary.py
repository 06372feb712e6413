"""MFMA utilisation per kernel from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass.

SQ_VALU_MFMA_BUSY_CYCLES sums the busy cycles of every MFMA the kernel issued (16 per
v_mfma_f32_16x16x32_{bf16,f16}); GRBM_GUI_ACTIVE sums the kernel's active cycles over the 8 XCDs
(MI355X_MICROARCH.md, DVFS give-back). Utilisation = busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
the fraction of the chip's MFMA issue capacity at the clock it actually ran (dense peak at that
clock = 1024 SIMDs x 1024 bf16 FLOP per cycle).

    python tools/mfma_summary.py DIR [--match NAME] [--json OUT]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--match", default="")
ap.add_argument("--json")
a = ap.parse_args()

busy = defaultdict(float)
gui = defaultdict(float)
n = defaultdict(set)
for d in a.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "?").replace("void ", "").replace("(anonymous namespace)::", "")
            name = name.split("(")[0]
            if a.match not in name:
                continue
            key = name
            n[key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "?")))
            if r["Counter_Name"] == "SQ_VALU_MFMA_BUSY_CYCLES":
                busy[key] += float(r["Counter_Value"])
            elif r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                gui[key] += float(r["Counter_Value"])
out = {}
tb, tg = 0.0, 0.0
for k in sorted(busy, key=lambda k: -gui[k]):
    cyc = gui[k] / 8
    util = busy[k] / (1024 * cyc) if cyc else 0.0
    tb += busy[k]
    tg += gui[k]
    out[k] = dict(dispatches=len(n[k]), mfma_busy_cycles=busy[k], active_cycles=cyc, mfma_util=util)
    print(f"{k[-60:]:60s} n={len(n[k]):4d} active {cyc / 1e6:9.3f} Mcyc  MFMA util {100 * util:6.2f} %")
if tg:
    print(f"{'all matched':60s} MFMA util {100 * tb / (1024 * tg / 8):6.2f} %")
    out["all"] = dict(mfma_util=tb / (1024 * tg / 8))
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
