"""Build the decode-GEMM tuning variants listed here into zonos_amd/lib/variants/."""
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd.build import LIBDIR, build_variant  # noqa: E402

VARIANTS = {
    "noa": {"ZK_DBG_NOALOAD": 1},        # activation LDS-DMA compiled out (diagnostic, wrong results)
    "pf8": {"ZK_WS_PF": 8},              # 8 weight chunks in flight per compute wave
    "nld1": {"ZK_WS_NLD": 1},            # one loader wave
}
if __name__ == "__main__":
    shutil.rmtree(os.path.join(LIBDIR, "variants"), ignore_errors=True)
    for name, d in VARIANTS.items():
        print(name, build_variant(name, d), flush=True)
