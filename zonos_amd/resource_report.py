"""Print per-kernel VGPR / scratch / occupancy of the HIP sources (hipcc -Rpass-analysis)."""
import os
import re
import subprocess
import sys

from .build import ARCH, CSRC, HIPCC

for src in sorted(os.listdir(CSRC)):
    if not src.endswith(".hip"):
        continue
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, src),
                        "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            info = {}
        for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
            m = re.search(key + r": (\d+)", line)
            if m and cur:
                info[key.split(" ")[0].replace("\\", "")] = int(m.group(1))
                if key.startswith("LDS"):
                    flag = " <-- SCRATCH" if info.get("ScratchSize", 0) else ""
                    print(f"{src:12s} {cur[:60]:60s} {info}{flag}")
