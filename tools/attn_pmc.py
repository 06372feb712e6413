"""Standalone launches of the fused decode attention (zk_attn_decode_qkv) at the bench's
workload shape (R=128 rows, Hkv=4, ctx 1705) for PMC collection:

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run --output-format csv -- python3 tools/attn_pmc.py
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run --output-format csv -- python3 tools/attn_pmc.py
    python tools/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_w > profiles/<round>_attn_pmc.txt
"""
import sys

import torch

sys.path.insert(0, ".")
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import rope_table  # noqa: E402

R, H, Hk, hd, ctx, gsplit = 128, 16, 4, 128, int(sys.argv[1]) if len(sys.argv) > 1 else 1705, 4
smax = (ctx + 1 + 255) // 256 * 256
dev = torch.device("cuda")
_lib.load()
kc = torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16)
vt = torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16)
N = (H + 2 * Hk) * hd
part = torch.randn(gsplit * R * N, device=dev) * 0.1
freqs = rope_table(16384, hd).to(dev)
out = torch.empty(R * H * hd, dtype=torch.bfloat16, device=dev)
work = torch.empty(1, device=dev)
s = _lib.stream_ptr()
for _ in range(20):
    call("zk_attn_decode_qkv", ptr(part), gsplit, ptr(freqs), ptr(kc), ptr(vt), R, H, Hk, hd, smax, ctx, None,
         ptr(work), 1, ptr(out), 0, None, s)
torch.cuda.synchronize()
print(f"R={R} ctx={ctx} smax={smax}: 20 launches; algorithmic bytes/launch = "
      f"{R * ctx * Hk * hd * 4 + gsplit * R * N * 4 + R * H * hd * 2 + R * Hk * hd * 4}")
