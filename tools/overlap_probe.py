"""Feasibility probe: does the c3 decode attention (HBM-bound) overlap with the decode GEMMs
(per-CU intake bound) when the 128 rows are split into two independent halves on two streams?

    python tools/overlap_probe.py [ctx]

Per "layer": attention over the KV cache (zk_attn_decode, q given) + the four decode GEMMs
(in_proj, out_proj, fc1 + SwiGLU, fc2) at the c3 shapes, with distinct weights / caches per layer
(nothing served from L2 / MALL across layers). Three schedules, HIP-event timed:
  full     one stream, 128 rows (the product's launch shape)
  halves   one stream, two 64-row halves one after the other
  overlap  two streams, half A runs attention then GEMMs, half B GEMMs then attention
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import _split_for  # noqa: E402

_lib.load()
dev = torch.device("cuda")
H, Hk, hd, D, F = 16, 4, 128, 2048, 8192
NL = 8
ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 1705
smax = (ctx + 255) // 256 * 256
SHAPES = [((H + 2 * Hk) * hd, D, 0), (D, H * hd, 0), (2 * F, D, 1), (D, F, 0)]


def bf(n):
    return torch.randn(n, device=dev).to(torch.bfloat16)


Ws = [[bf((N + 63) // 64 * 64 * K) for (N, K, _) in SHAPES] for _ in range(NL)]


class Half:
    def __init__(self, R):
        self.R = R
        self.kc = [bf(R * Hk * smax * hd) for _ in range(NL)]
        self.vt = [bf(R * Hk * smax * hd) for _ in range(NL)]
        self.q = bf(R * H * hd)
        self.out = torch.empty(R * H * hd, dtype=torch.bfloat16, device=dev)
        self.A = bf(R * F)
        self.h = torch.empty(R * F, dtype=torch.bfloat16, device=dev)
        self.splits = [1 if m == 1 else _split_for(N, K, R, 256) for (N, K, m) in SHAPES]
        self.part = torch.empty(max(s * R * N for s, (N, _, _) in zip(self.splits, SHAPES)), device=dev)

    def attn(self, l, s):
        call("zk_attn_decode", ptr(self.q), ptr(self.kc[l]), ptr(self.vt[l]), self.R, H, Hk, hd, smax, ctx, None,
             None, 1, ptr(self.out), None, s)

    def gemms(self, l, s):
        for (N, K, m), W, ns in zip(SHAPES, Ws[l], self.splits):
            call("zk_gemm_bf16", ptr(self.A), K, ptr(W), self.R, N, K, ns, m, ptr(self.part), ptr(self.h), None, s)


full, a, b = Half(128), Half(64), Half(64)
main = torch.cuda.current_stream()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run_full():
    for l in range(NL):
        full.attn(l, main.cuda_stream)
        full.gemms(l, main.cuda_stream)


def run_halves():
    for l in range(NL):
        for hf in (a, b):
            hf.attn(l, main.cuda_stream)
            hf.gemms(l, main.cuda_stream)


def run_overlap():
    s1.wait_stream(main)
    s2.wait_stream(main)
    for l in range(NL):
        a.attn(l, s1.cuda_stream)
        a.gemms(l, s1.cuda_stream)
        b.gemms(l, s2.cuda_stream)
        b.attn(l, s2.cuda_stream)
    main.wait_stream(s1)
    main.wait_stream(s2)


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(reps):
        fn()
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / NL * 1e3   # us per layer


def parts():
    """attention alone and GEMMs alone, per layer"""
    def att():
        for l in range(NL):
            full.attn(l, main.cuda_stream)

    def gem():
        for l in range(NL):
            full.gemms(l, main.cuda_stream)
    return timed(att), timed(gem)


if __name__ == "__main__":
    at, ge = parts()
    print(f"ctx {ctx}: per layer attention {at:6.1f} us, 4 GEMMs {ge:6.1f} us (128 rows)", flush=True)
    for name, fn in (("full", run_full), ("halves", run_halves), ("overlap", run_overlap)) * 2:
        print(f"  {name:8s} {timed(fn):7.1f} us per layer", flush=True)
