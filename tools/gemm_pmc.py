"""Standalone launches of the decode GEMMs at the c3 shapes (M=128) for PMC collection:

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/gpmc_f -o run --output-format csv -- python3 tools/gemm_pmc.py
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/gpmc_w -o run --output-format csv -- python3 tools/gemm_pmc.py
    python tools/pmc_summary.py gpurun_out/gpmc_f gpurun_out/gpmc_w --match k_gemm_ws
Each shape runs 10 times over 3 weight copies (> the 256 MB Infinity Cache for fc1/fc2)."""
import sys

import torch

sys.path.insert(0, ".")
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import _split_for  # noqa: E402

_lib.load()
dev = torch.device("cuda")
S = _lib.stream_ptr()
M = 128
for name, N, K, mode in (("qkv", 3072, 2048, 0), ("o", 2048, 2048, 0), ("fc1", 16384, 2048, 1),
                         ("fc2", 2048, 8192, 0)):
    ncopy = max(3, int(600e6 // (N * K * 2)) + 1)
    Ws = [torch.randn((N + 63) // 64 * 64, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    ns = 1 if mode == 1 else _split_for(N, K, M)
    part = torch.empty(ns * M * N, device=dev)
    out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
    for i in range(10):
        call("zk_gemm_bf16", ptr(A), K, ptr(Ws[i % ncopy]), M, N, K, ns, mode, ptr(part), ptr(out), None, S)
    torch.cuda.synchronize()
    print(name, N, K, ns, "weights MB", N * K * 2 / 1e6, "out MB", (ns * M * N * 4 if mode == 0 else M * N), flush=True)
    del Ws
