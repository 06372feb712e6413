"""Per-step timing inside the channels-last DAC conv (diagnostic build -DZK_CL_PROF, GPU box):
    ZK_LIB_PATH=zonos_amd/lib/variants/clprof/libzonos_hip.so python tools/dac_conv_stamps.py [C] [dil]
Runs one plain k7 conv (C -> C channels, B = 4 x 165120 positions) and prints, over the first 64
workgroups, the median s_memtime cycles between the compute waves' barrier exits (one step), the
loader's wait before each barrier, and the main-loop / epilogue spans."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr, stream_ptr  # noqa: E402

lib = _lib.load()
Cc = int(sys.argv[1]) if len(sys.argv) > 1 else 192
dil = int(sys.argv[2]) if len(sys.argv) > 2 else 1
B, T, ks = 4, 165120, 7
dev = "cuda"
x = (torch.randn(B, T, Cc, device=dev) * 0.5).half()
w = (torch.randn(ks, Cc, Cc, device=dev) * 0.05).half()
bias = torch.zeros(Cc, device=dev)
alpha = torch.ones(Cc, device=dev)
s_out = torch.empty(B, T, Cc, dtype=torch.float16, device=dev)
S = stream_ptr()
for _ in range(3):
    call("zk_dac_conv_cl", ptr(x), B, Cc, T, ptr(w), 0, ptr(bias), Cc, ks, dil, 3 * dil, T, 1, 1, 0, T, None, None,
         ptr(alpha), ptr(s_out), 0, None, 1, 1, S)
torch.cuda.synchronize()
prof = np.zeros((64, 3, 64), dtype=np.uint64)
pend = np.zeros((64, 6), dtype=np.uint64)
lib.zk_cl_prof_read.argtypes = [C.c_void_p, C.c_void_p]
assert lib.zk_cl_prof_read(prof.ctypes.data, pend.ctypes.data) == 0
nstep = (Cc // 32) * ks
c = prof[:, 2, :nstep].astype(np.int64)                 # compute: after barrier s
l0 = prof[:, 0, :nstep].astype(np.int64)                # loader: before wait for step j
l1 = prof[:, 1, :nstep].astype(np.int64)                # loader: after barrier j
step = np.diff(c, axis=1)
print(f"C={Cc} dil={dil} steps/WG={nstep}: compute step (barrier exit to barrier exit) median {np.median(step):.0f} "
      f"cycles, p10 {np.percentile(step, 10):.0f}, p90 {np.percentile(step, 90):.0f}")
print(f"  loader wait+barrier (before wait -> after barrier) median {np.median(l1 - l0):.0f} cycles; "
      f"loader issue (after barrier j -> before wait j+1) median {np.median(l0[:, 1:] - l1[:, :-1]):.0f}")
rt = pend.astype(np.int64)
clk = np.median((rt[:, 5] - rt[:, 4]) / (rt[:, 3] - rt[:, 0]) * 100.0)      # MHz (memrealtime = 100 MHz)
us = lambda a: np.median(a) / 100.0
print(f"  per workgroup (us, median of 64): start -> first barrier {us(rt[:, 1] - rt[:, 0]):.2f}, main loop "
      f"{us(rt[:, 2] - rt[:, 1]):.2f}, epilogue {us(rt[:, 3] - rt[:, 2]):.2f}, total {us(rt[:, 3] - rt[:, 0]):.2f}; "
      f"clock {clk:.0f} MHz; start spread {np.ptp(rt[:, 0]) / 100:.2f} us")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    call("zk_dac_conv_cl", ptr(x), B, Cc, T, ptr(w), 0, ptr(bias), Cc, ks, dil, 3 * dil, T, 1, 1, 0, T, None, None,
         ptr(alpha), ptr(s_out), 0, None, 1, 1, S)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
fm = 3 if Cc % 96 == 0 and Cc // 32 % 4 else 4
wg = np.zeros((4096, 2), dtype=np.uint64)
lib.zk_cl_prof_read_wg.argtypes = [C.c_void_p]
assert lib.zk_cl_prof_read_wg(wg.ctypes.data) == 0
wg = wg.astype(np.int64)
nw = min(4096, int((wg[:, 0] > 0).sum()))
st, en = wg[:nw, 0], wg[:nw, 1]
t0 = st.min()
ev = sorted([(t, 1) for t in st] + [(t, -1) for t in en])
cur = best = 0
act = []
for t, d in ev:
    cur += d
    act.append((t, cur))
best = max(a for _, a in act)
tmid = t0 + (en.max() - t0) // 2
print(f"  workgroups 0..{nw - 1}: resident at once max {best}, at mid-run {max(a for t, a in act if t <= tmid)}; "
      f"median lifetime {np.median(en - st) / 100:.2f} us; first {nw} span {(en.max() - t0) / 100:.1f} us")
hw = np.zeros((4096, 8), dtype=np.uint32)
lib.zk_cl_prof_read_hw.argtypes = [C.c_void_p]
assert lib.zk_cl_prof_read_hw(hw.ctypes.data) == 0
hw = hw[:nw].astype(np.int64)
cu_key = (hw[:, 6] << 16) | (((hw[:, 0] >> 13) & 7) << 8) | (((hw[:, 0] >> 12) & 1) << 4) | ((hw[:, 0] >> 8) & 15)
from collections import Counter
per_cu = Counter(cu_key.tolist())
print(f"  CUs used {len(per_cu)}, workgroups per CU: {sorted(Counter(per_cu.values()).items())}")
simd = (hw[:, :6] >> 4) & 3
pat = Counter(tuple(np.bincount(simd[i], minlength=4).tolist()) for i in range(nw))
print(f"  waves per SIMD within a workgroup (waves 0-5): {pat.most_common(4)}")
# concurrent pairs on one CU: SIMD totals
tot = {}
for i in range(nw):
    tot.setdefault(int(cu_key[i]), np.zeros(4, dtype=int))
    tot[int(cu_key[i])] += np.bincount(simd[i], minlength=4)
print(f"  per-CU SIMD wave totals (all its workgroups): {Counter(tuple(v.tolist()) for v in tot.values()).most_common(5)}")
print(f"  launch {ms * 1e3:.1f} us, {2 * Cc * Cc * ks * B * T / ms / 1e9:.0f} TFLOP/s")
for s_ in (0, 1, 2, 6, 7, 8, 13, 14, 20, 21):
    if s_ + 1 < nstep:
        print(f"  step {s_:2d}: compute {np.median(c[:, s_ + 1] - c[:, s_]):6.0f}  loader wait {np.median(l1[:, s_] - l0[:, s_]):6.0f}")
