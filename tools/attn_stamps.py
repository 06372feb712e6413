"""Where the B = 1 decode attention's time goes (profiling build with -DZK_ATT_PROF, loaded via
ZK_LIB_PATH): per-workgroup s_memrealtime stamps [entry, KV loads issued, prologue done, key loop
done, merged, end] of one launch, against the launch's HIP-event time."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import rope_table  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda")
S = _lib.stream_ptr()
R, H, Hk, hd, smax = 2, 16, 4, 128, 1280
prof = torch.zeros(512 * 8, dtype=torch.int64, device=dev)
cnt = torch.zeros(R * Hk, dtype=torch.int32, device=dev)
lib.zk_att_prof_set.argtypes = [C.c_void_p]
assert lib.zk_att_prof_set(prof.data_ptr()) == 0
nl = 26
kcs = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(nl)]
vts = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(nl)]
part = torch.randn(R * (H + 2 * Hk) * hd, device=dev) * 0.1
freqs = rope_table(16384, hd).to(dev)
out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
work = torch.empty(R * Hk * (8 + 4 * hd), device=dev)
for ctx in (300, 600, 1000):
    for i in range(60):
        call("zk_attn_decode_qkv", ptr(part), 1, ptr(freqs), ptr(kcs[i % nl]), ptr(vts[i % nl]), R, H, Hk, hd, smax,
             ctx, None, ptr(work), 1, ptr(out), 0, None, S)
    torch.cuda.synchronize()
    p = prof[: R * Hk * 8].view(R * Hk, 8).cpu().double() * 10.0 / 1000.0     # us (100 MHz)
    t0 = p[:, 0].min()
    d = p[:, :6] - t0
    print(f"ctx {ctx}: stamps relative to the first workgroup's entry (us), per workgroup:")
    names = ["entry", "issued", "prologue", "keyloop", "merged", "end"]
    print("   " + " ".join(f"{n:>9s}" for n in names))
    for wg in range(R * Hk):
        print("   " + " ".join(f"{float(x):9.2f}" for x in d[wg]))

for ctx, ns in ((600, 4), (600, 8), (1000, 4)):
    work = torch.empty(R * Hk * ns * (8 + 4 * hd), device=dev)
    prof.zero_()
    for i in range(60):
        call("zk_attn_decode_qkv_sc", ptr(part), 1, ptr(freqs), ptr(kcs[i % nl]), ptr(vts[i % nl]), R, H, Hk, hd,
             smax, ctx, None, ptr(work), ns, ptr(cnt), ptr(out), 0, None, S)
    torch.cuda.synchronize()
    n = R * Hk * ns
    p = prof[: n * 8].view(n, 8).cpu().double() * 10.0 / 1000.0
    t0 = p[:, 0].min()
    d = p - t0
    print(f"ctx {ctx}, {ns} splits merged in the launch: (us from the first entry)")
    names = ["entry", "issued", "prologue", "keyloop", "merged4w", "ticket", "mergebeg", "end"]
    print("   " + " ".join(f"{x:>9s}" for x in names))
    for wg in range(n):
        print("   " + " ".join(f"{float(x):9.2f}" if p[wg, k] > 0 else f"{'-':>9s}" for k, x in enumerate(d[wg])))
