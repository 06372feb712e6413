"""Standalone launches for PMC collection of the c2 / c5 bench lines' dominant kernels:
    gemv : zk_gemv_fused fc1 + SwiGLU + LayerNorm prologue at M = 2 (B = 1), 4 rotating weight copies
    mamba: zk_mamba_step at the c5 shape (R = 128, d_inner 4096, 64 heads x 64, d_state 128), 3
           rotating SSM states
    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python3 tools/small_pmc.py gemv
"""
import sys

import torch

sys.path.insert(0, ".")
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402

dev = torch.device("cuda")
_lib.load()
s = _lib.stream_ptr()
mode = sys.argv[1]
if mode == "gemv":
    M, N, K = 2, 16384, 2048
    Ws = [torch.randn((N + 63) // 64 * 64, K, device=dev).to(torch.bfloat16) for _ in range(4)]
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    lw = torch.ones(K, device=dev).to(torch.bfloat16)
    lb = torch.zeros(K, device=dev).to(torch.bfloat16)
    h = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
    for i in range(16):
        call("zk_gemv_fused", ptr(x), K, ptr(Ws[i % 4]), M, N, K, 1, ptr(lw), ptr(lb), 1e-5, None, ptr(h), None, s)
    print("gemv fc1 M=2: algorithmic bytes/launch", N * K * 2 + M * K * 2 + 2 * K * 2 + M * N)
else:
    R, di, nh, hp, ds = 128, 4096, 64, 64, 128
    cdim, nin, gs = di + 2 * ds, 2 * di + 2 * ds + nh, 1
    part = torch.randn(gs * R * nin, device=dev) * 0.1
    cw = torch.randn(cdim, 4, device=dev) * 0.1
    cb = torch.zeros(cdim, device=dev)
    c0 = torch.zeros(R * cdim * 4, dtype=torch.bfloat16, device=dev)
    c1 = torch.zeros(R * cdim * 4, dtype=torch.bfloat16, device=dev)
    pos = torch.full((1,), 700, dtype=torch.int32, device=dev)
    ssms = [torch.randn(R * nh * hp * ds, device=dev).to(torch.bfloat16) for _ in range(3)]
    A = -torch.rand(nh, device=dev)
    dtb = torch.zeros(nh, device=dev)
    Dv = torch.ones(nh, device=dev)
    yz = torch.empty(R * di, device=dev)
    for i in range(12):
        call("zk_mamba_step", ptr(part), gs, R, di, nh, hp, ds, ptr(cw), ptr(cb), ptr(c0), ptr(c1), ptr(pos),
             ptr(ssms[i % 3]), None, ptr(A), ptr(dtb), ptr(Dv), ptr(yz), None, s)
    print("mamba_step R=128: algorithmic bytes/launch", R * di * ds * 2 * 2 + R * cdim * 8 * 2 + gs * R * nin * 4 + R * di * 4)
torch.cuda.synchronize()
