"""Build libzonos_hip.so in-tree (zonos_amd/lib/) with hipcc for gfx950.

    python -m zonos_amd.build [--force]

Each translation unit is compiled in parallel, then linked with hipcc -shared. The
library is git-ignored but travels to the GPU box with the working tree.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libzonos_hip.so")
SOURCES = ["sampler.hip", "backbone.hip", "gemm.hip", "gemm_pf.hip", "dac.hip", "dac_mfma.hip", "dac_cl.hip", "post.hip", "mamba.hip", "cond.hip", "capi.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ZK_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no implicit FMA contraction -- the reference rounds every elementwise op
# (torch CPU kernels are unfused) and __fmul_rn / __fadd_rn are plain operators in HIP, so
# contraction would make results depend on how each kernel happens to be scheduled.
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result", "-ffp-contract=off"]


def _deps_mtime() -> float:
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    files.append(os.path.join(os.path.dirname(HERE), "include", "zonos_hip.h"))
    files.append(os.path.abspath(__file__))
    return max(os.path.getmtime(f) for f in files)


def _compile(src: str, libdir: str = LIBDIR, extra=()) -> str:
    obj = os.path.join(libdir, src.rsplit(".", 1)[0] + ".o")
    cmd = [HIPCC, *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        return LIB
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    tmp = LIB + ".tmp"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[zonos_amd] built {LIB}", file=sys.stderr)
    return LIB


def build_variant(name: str, defines: dict) -> str:
    """Tuning experiments only: the same sources with -D overrides, linked into
    lib/variants/<name>/libzonos_hip.so (select with ZK_LIB_PATH; the product uses LIB)."""
    d = os.path.join(LIBDIR, "variants", name)
    os.makedirs(d, exist_ok=True)
    extra = [f"-D{k}={v}" for k, v in defines.items()]
    with ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, d, extra), SOURCES))
    out = os.path.join(d, "libzonos_hip.so")
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    for o in objs:
        os.remove(o)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
