"""Where the c3 decode attention (k_attn_decode, B = 64: 128 rows x 4 kv heads = 512 workgroups, 2 per CU)
spends its time: per-workgroup s_memrealtime stamps (build variant -DZK_ATT_PROF=1) of the last attention
launch of a c3-shaped generate, at a few context lengths. Developer tool.
    ZK_LIB_PATH=zonos_amd/lib/variants/attprof/libzonos_hip.so python tools/attn_c3_stamps.py
Stamps: 0 entry, 1 step words tested, 2 prologue done (q / new key in LDS), 3 key loop done, 4 merged, 5 end."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib, synthetic  # noqa: E402
from zonos_amd.engine import EngineConfig, HipDecoder  # noqa: E402

lib = _lib.load()
lib.zk_att_prof_set.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
eng = HipDecoder(EngineConfig(**synthetic.ZONOS_V01), synthetic.backbone_weights(dev, seed=0), dev)
B = 64
cond = synthetic.conditioning(B, 400, 2048, seed=11, device=dev)
prefix = synthetic.prefix_codes(B, 10, seed=3, device=dev)
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)
prof = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
assert lib.zk_att_prof_set(prof.data_ptr()) == 0
names = ["entry", "words", "prologue", "loop", "merged", "end"]


def q(x, f):
    v = x.sort().values
    return float(v[min(len(v) - 1, int(f * (len(v) - 1)))])


for new in (300, 1300, 2500):
    prof.zero_()
    eng.generate(cond, prefix, new, 2.0, B, sp, seed=5, force_full_length=True, poll_every=64)
    torch.cuda.synchronize()
    p = prof.view(-1, 8)[:, :6].cpu()
    used = p[:, 0] > 0
    p = p[used].double()
    rel = (p - p[:, 0].min()) / 100.0          # s_memrealtime: 100 MHz -> us
    ctx = 400 + 10 + 1 + new
    print(f"ctx ~{ctx}: {int(used.sum())} workgroups (us from the first entry):", flush=True)
    for i, n in enumerate(names):
        x = rel[:, i]
        print(f"  {n:9s} p10 {q(x, .1):7.2f}  p50 {q(x, .5):7.2f}  p90 {q(x, .9):7.2f}  max {q(x, 1):7.2f}", flush=True)
    hw = prof.view(-1, 8)[used][:, 6:8].cpu()
    if int(hw[:, 1].max()) > 0 or int(hw[:, 0].max()) > 0:
        xcc = (hw[:, 1] & 0xF).long()
        cu = ((hw[:, 0] >> 8) & 0xF) + 16 * ((hw[:, 0] >> 13) & 0x3) + 64 * ((hw[:, 0] >> 12) & 0x1)
        loop_end = rel[:, 3]
        print("  loop end by XCC: " + "  ".join(f"{x}: p50 {q(loop_end[xcc == x], .5):.1f} max {q(loop_end[xcc == x], 1):.1f}"
                                                for x in range(8) if int((xcc == x).sum()) > 0), flush=True)
        key = xcc * 1024 + cu
        same, diff = [], []
        for k in key.unique():
            idx = (key == k).nonzero().flatten()
            if len(idx) == 2:
                same.append(abs(float(loop_end[idx[0]] - loop_end[idx[1]])))
        if same:
            same = torch.tensor(same)
            print(f"  workgroup pairs sharing a CU: {len(same)}; |loop end difference| p50 {q(same, .5):.1f} max {q(same, 1):.1f} us",
                  flush=True)
        cu_end = {}
        for k in key.unique():
            cu_end[int(k)] = float(loop_end[key == k].max())
        ce = torch.tensor(list(cu_end.values()))
        print(f"  per-CU last loop end ({len(ce)} CUs): p10 {q(ce, .1):.1f} p50 {q(ce, .5):.1f} p90 {q(ce, .9):.1f} max {q(ce, 1):.1f}",
              flush=True)
    dur = rel[:, 5] - rel[:, 0]
    print(f"  per-workgroup duration p10 {q(dur, .1):.2f} p50 {q(dur, .5):.2f} p90 {q(dur, .9):.2f} max {q(dur, 1):.2f}",
          flush=True)
