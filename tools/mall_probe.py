"""Infinity Cache (MALL) warming probe for the c3 decode step: can the next layer's KV cache be
pulled on-die while the GEMM chain runs (HBM at ~3 TB/s there), so that the attention -- 51 % of
a c3 step at the HBM ceiling -- reads part of it from the MALL?
    python tools/mall_probe.py
Prints: attention time cold / after prefetching a fraction f of every (row, kv head) cache with
plain or non-temporal loads; prefetch kernel rate; a GEMM chain alone vs with a concurrent
prefetch on a second stream, and the attention after it."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import rope_table  # noqa: E402

_lib.load()
dev = torch.device("cuda")
S1 = torch.cuda.Stream()
S2 = torch.cuda.Stream()
R, H, Hk, hd = 128, 16, 4, 128
ctx, smax = 1705, 1792
ncopy = 3
kcs = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
vts = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
gs = 4
part = torch.randn(gs * R * (H + 2 * Hk) * hd, device=dev) * 0.1
freqs = rope_table(16384, hd).to(dev)
work = torch.empty(R * Hk * (8 + 4 * hd), device=dev)
out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
seg = smax * hd * 2                     # bytes of one (row, kv head) K (or V^T) block
M = 128
shapes = [("o", 2048, 2048, 4, 0), ("fc1", 16384, 2048, 1, 1), ("fc2", 2048, 8192, 8, 0), ("qkv", 3072, 2048, 4, 0)]
Ws = {n: torch.randn((N + 63) // 64 * 64, K, device=dev).to(torch.bfloat16) for n, N, K, _, _ in shapes}
A = torch.randn(M, 8192, device=dev).to(torch.bfloat16)
gpart = torch.empty(8 * M * 3072, device=dev)
gout = torch.empty(M, 8192, dtype=torch.bfloat16, device=dev)


def sp(s):
    return s.cuda_stream


def flush(s):
    call("zk_prefetch", ptr(junk), 1 << 20, 1 << 20, 1024, 0, 512, ptr(sink), sp(s))


def attn(i, s):
    call("zk_attn_decode_qkv", ptr(part), gs, ptr(freqs), ptr(kcs[i]), ptr(vts[i]), R, H, Hk, hd, smax, ctx, None,
         ptr(work), 1, ptr(out), 0, None, sp(s))


def prefetch(i, frac, mode, nblocks, s):
    nb = int(seg * frac) // 16 * 16
    if nb <= 0:
        return
    call("zk_prefetch", ptr(kcs[i]), seg, nb, R * Hk, mode, nblocks, ptr(sink), sp(s))
    call("zk_prefetch", ptr(vts[i]), seg, nb, R * Hk, mode, nblocks, ptr(sink), sp(s))


def chain(s):
    for n, N, K, ns, mode in shapes:
        call("zk_gemm_bf16", ptr(A), K, ptr(Ws[n]), M, N, K, ns, mode, ptr(gpart), ptr(gout), None, sp(s))


def timed(fn, s):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


kvb = R * ctx * Hk * hd * 2 * 2
with torch.cuda.stream(S1):
    for _ in range(3):
        attn(0, S1)
        chain(S1)
    torch.cuda.synchronize()
    cold = []
    for r in range(6):
        flush(S1)
        cold.append(timed(lambda: attn(r % ncopy, S1), S1))
    print(f"attention cold: {med(cold):.1f} us ({kvb / med(cold) / 1e3:.0f} GB/s on {kvb / 1e6:.0f} MB)", flush=True)
    warm = []
    for r in range(4):
        attn(r % ncopy, S1)
        warm.append(timed(lambda: attn(r % ncopy, S1), S1))
    print(f"attention right after itself: {med(warm):.1f} us", flush=True)
    for mode in (0, 1):
        for frac in (0.25, 0.5, 0.75):
            ts, tp = [], []
            for r in range(4):
                i = r % ncopy
                flush(S1)
                tp.append(timed(lambda: prefetch(i, frac, mode, 256, S1), S1))
                ts.append(timed(lambda: attn(i, S1), S1))
            pb = 2 * R * Hk * (int(seg * frac) // 16 * 16)
            print(f"prefetch mode {mode} frac {frac:.2f}: prefetch {med(tp):.1f} us ({pb / med(tp) / 1e3:.0f} GB/s, "
                  f"{pb / 1e6:.0f} MB) -> attention {med(ts):.1f} us", flush=True)
    for nbk in (32, 64, 128):
        tp = []
        for r in range(3):
            flush(S1)
            tp.append(timed(lambda: prefetch(0, 0.5, 0, nbk, S1), S1))
        pb = 2 * R * Hk * (int(seg * 0.5) // 16 * 16)
        print(f"prefetch 50 % with {nbk} workgroups: {med(tp):.1f} us ({pb / med(tp) / 1e3:.0f} GB/s)", flush=True)
    # GEMM chain alone vs beside a prefetch on a second stream, then the attention
    for frac, nbk in ((0.0, 0), (0.3, 32), (0.3, 64), (0.5, 64), (0.5, 128)):
        tc, ta = [], []
        for r in range(4):
            i = r % ncopy
            flush(S1)
            torch.cuda.synchronize()
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(S1)
            if frac > 0:
                S2.wait_event(e0)
                prefetch(i, frac, 0, nbk, S2)
            chain(S1)
            e1.record(S1)
            if frac > 0:
                S1.wait_stream(S2)
            attn(i, S1)
            e2.record(S1)
            torch.cuda.synchronize()
            tc.append(e0.elapsed_time(e1) * 1e3)
            ta.append(e1.elapsed_time(e2) * 1e3)
        print(f"chain {'alone' if frac == 0 else f'+ prefetch {frac:.1f} ({nbk} WGs)':>24s}: chain {med(tc):.1f} us, "
              f"then attention {med(ta):.1f} us, total {med(tc) + med(ta):.1f}", flush=True)
