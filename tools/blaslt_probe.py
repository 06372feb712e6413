"""How fast would a library GEMM (torch.mm -> hipBLASLt) run the c3 prefill projections?
Informational only (the product prefill runs zk_gemm_bf16). Prints ms and TFLOP/s per shape."""
import torch

M = 128 * 411
dev = torch.device("cuda")
for name, N, K in (("qkv", 3072, 2048), ("o", 2048, 2048), ("fc1", 16384, 2048), ("fc2", 2048, 8192)):
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(3):
        torch.mm(A, W.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.mm(A, W.t())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"torch.mm {name:4s} M={M} N={N:5d} K={K:5d}: {ms:7.3f} ms {2.0 * M * N * K / (ms * 1e-3) / 1e12:7.1f} TFLOP/s",
          flush=True)
    del A, W
