"""Does the Infinity Cache (MALL) speed up a B=1 weight-streaming GEMV? fc1 / out_proj shapes
(zk_gemv_fused, M=2) timed (a) rotating through weight copies larger than the MALL (cold), (b) the
same copy back to back (MALL-warm: 67 MB < 256 MB), (c) cold but with the first fraction of its
weights pre-read by zk_prefetch just before (the "tail prefetch" idea)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402

_lib.load()
dev = torch.device("cuda")
S = torch.cuda.current_stream().cuda_stream
M = 2
sink = torch.zeros(4, dtype=torch.int32, device=dev)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def ev_time(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for name, N, K, mode in (("fc1", 16384, 2048, 1), ("out", 2048, 2048, 2), ("fc2", 2048, 8192, 2)):
    nbytes = N * K * 2
    ncopy = max(3, int(600e6 // nbytes) + 1)
    Ws = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    lnw = torch.ones(K, device=dev).to(torch.bfloat16)
    lnb = torch.zeros(K, device=dev).to(torch.bfloat16)
    outb = torch.empty(M, max(N // 2, N), dtype=torch.bfloat16, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)

    def g(W):
        if mode == 1:
            call("zk_gemv_fused", ptr(x), K, ptr(W), M, N, K, 1, ptr(lnw), ptr(lnb), 1e-5, None, ptr(outb), None, S)
        else:
            call("zk_gemv_fused", ptr(x), K, ptr(W), M, N, K, 2, None, None, 1e-5, None, ptr(res), None, S)
    for _ in range(3):
        g(Ws[0])
    cold = ev_time(lambda i: g(Ws[i % ncopy]), 3 * ncopy)
    warm = ev_time(lambda i: g(Ws[0]), 30)
    print(f"{name}: cold (rotating {ncopy} copies) {cold:.2f} us = {nbytes / cold / 1e3:.0f} GB/s; "
          f"same copy back to back {warm:.2f} us = {nbytes / warm / 1e3:.0f} GB/s", flush=True)
    for frac in (0.1, 0.25, 1.0):
        pb = int(nbytes * frac) // 16 * 16
        ts = []
        for r in range(6):
            W = Ws[(r + 1) % ncopy]
            call("zk_prefetch", ptr(junk), 1 << 20, 1 << 20, 1024, 0, 512, ptr(sink), S)    # flush
            call("zk_prefetch", ptr(W), pb, pb, 1, 0, 256, ptr(sink), S)
            ts.append(ev_time(lambda i: g(W), 1))
        ts.sort()
        print(f"   after pre-reading the first {frac:.0%} of its weights: {ts[len(ts) // 2]:.2f} us", flush=True)
    del Ws
