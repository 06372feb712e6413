"""Reference point for the prefill GEMMs: torch.matmul (hipBLASLt) at the c3 prefill shapes,
bf16 in / fp32 accumulate, timed with HIP events -- the library's rate, not a product path."""
import torch

dev = torch.device("cuda")
M = 52608
for name, N, K in (("qkv", 3072, 2048), ("o", 2048, 2048), ("fc1", 16384, 2048), ("fc2", 2048, 8192)):
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"torch.matmul {name:4s} M={M} N={N:5d} K={K}: {ms:7.3f} ms  {2 * M * N * K / ms / 1e9:7.1f} TFLOP/s",
          flush=True)
    del a, w, c
