"""Probe: do two half-batch decode pipelines on two HIP streams overlap well?
Times (a) one M=128 GEMM / attention launch, (b) two M=64 launches on two streams, same weights."""
import sys
import time

import torch

sys.path.insert(0, ".")
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import _split_for, pack_weights, rope_table  # noqa: E402

dev = torch.device("cuda")
_lib.load()
s0 = torch.cuda.Stream()
s1 = torch.cuda.Stream()


def tm(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


for name, N, K, mode in (("qkv", 3072, 2048, 0), ("o", 2048, 2048, 0), ("fc1", 16384, 2048, 1), ("fc2", 2048, 8192, 0)):
    W = pack_weights(torch.randn(N, K, device=dev).to(torch.bfloat16), _lib.stream_ptr())
    outs = {}
    for M in (128, 64):
        ns = 1 if mode else _split_for(N, K, M)
        A = [torch.randn(M, K, device=dev).to(torch.bfloat16) for _ in range(2)]
        P = [torch.empty(ns * M * N, device=dev) for _ in range(2)]
        O = [torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev) for _ in range(2)]
        outs[M] = (ns, A, P, O)

    def one128():
        ns, A, P, O = outs[128]
        call("zk_gemm_bf16", ptr(A[0]), K, ptr(W), 128, N, K, ns, mode, ptr(P[0]), ptr(O[0]), None,
             torch.cuda.current_stream().cuda_stream)

    def two64():
        ns, A, P, O = outs[64]
        for i, st in enumerate((s0, s1)):
            call("zk_gemm_bf16", ptr(A[i]), K, ptr(W), 64, N, K, ns, mode, ptr(P[i]), ptr(O[i]), None, st.cuda_stream)

    def seq64():
        ns, A, P, O = outs[64]
        for i in range(2):
            call("zk_gemm_bf16", ptr(A[i]), K, ptr(W), 64, N, K, ns, mode, ptr(P[i]), ptr(O[i]), None,
                 torch.cuda.current_stream().cuda_stream)

    print(f"gemm {name}: one M=128 {tm(one128):7.1f} us | two M=64 concurrent {tm(two64):7.1f} us | "
          f"two M=64 serial {tm(seq64):7.1f} us", flush=True)

# attention (R=64 per half) concurrent with fc1 GEMM of the other half
R, H, Hk, hd, ctx = 64, 16, 4, 128, 1705
smax = 1792
kc = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(2)]
vt = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(2)]
part = torch.randn(4 * R * (H + 2 * Hk) * hd, device=dev) * 0.1
fr = rope_table(16384, hd).to(dev)
y = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
work = torch.empty(R * Hk * 2 * (8 + 4 * hd), device=dev)
W1 = pack_weights(torch.randn(16384, 2048, device=dev).to(torch.bfloat16), _lib.stream_ptr())
A1 = torch.randn(64, 2048, device=dev).to(torch.bfloat16)
O1 = torch.empty(64, 8192, dtype=torch.bfloat16, device=dev)


def att(i, st):
    call("zk_attn_decode_qkv", ptr(part), 4, ptr(fr), ptr(kc[i]), ptr(vt[i]), R, H, Hk, hd, smax, ctx, None, ptr(work),
         2, ptr(y), 0, None, st.cuda_stream)


def g1(st):
    call("zk_gemm_bf16", ptr(A1), 2048, ptr(W1), 64, 16384, 2048, 1, 1, None, ptr(O1), None, st.cuda_stream)


print(f"attn R=64 alone {tm(lambda: att(0, s0)):7.1f} us | fc1 M=64 alone {tm(lambda: g1(s1)):7.1f} us | "
      f"concurrent {tm(lambda: (att(0, s0), g1(s1))):7.1f} us | two attn concurrent "
      f"{tm(lambda: (att(0, s0), att(1, s1))):7.1f} us", flush=True)
