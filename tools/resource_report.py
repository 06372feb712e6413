"""Print per-kernel VGPR / scratch / occupancy of the HIP sources (hipcc -Rpass-analysis).

Developer tool, not part of the product package: `python tools/resource_report.py`."""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd.build import ARCH, CSRC, HIPCC  # noqa: E402

KEYS = ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]")


def report(src: str) -> None:
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, src),
                        "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur, info = None, {}
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur, info = m.group(1), {}
        for key in KEYS:
            m = re.search(key + r": (\d+)", line)
            if m and cur:
                info[key.split(" ")[0].replace("\\", "")] = int(m.group(1))
                if key.startswith("LDS"):
                    flag = " <-- SCRATCH" if info.get("ScratchSize", 0) else ""
                    print(f"{src:12s} {cur[:60]:60s} {info}{flag}")


def main(argv) -> None:
    srcs = argv or sorted(s for s in os.listdir(CSRC) if s.endswith(".hip"))
    for src in srcs:
        report(src)


if __name__ == "__main__":
    main(sys.argv[1:])
