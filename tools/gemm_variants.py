"""Build the decode-GEMM tuning variants listed here into zonos_amd/lib/variants/."""
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd.build import LIBDIR, build_variant  # noqa: E402

VARIANTS = {
    "nt": {"ZK_WS_NT": 1},
    "nt_noa": {"ZK_WS_NT": 1, "ZK_DBG_NOALOAD": 1},
    "nt_nom": {"ZK_WS_NT": 1, "ZK_DBG_NOMFMA": 1},
    "nt_noboth": {"ZK_WS_NT": 1, "ZK_DBG_NOALOAD": 1, "ZK_DBG_NOMFMA": 1},
    "ws2all": {"ZK_WS2_MIN_CHUNKS": 8},
    "occ2": {"ZK_WS_NB": 4, "ZK_WS_DA": 2, "ZK_WS_OCC": 2},
    "pf8": {"ZK_WS_PF": 8},
}
if __name__ == "__main__":
    shutil.rmtree(os.path.join(LIBDIR, "variants"), ignore_errors=True)
    for name, d in VARIANTS.items():
        print(name, build_variant(name, d), flush=True)
