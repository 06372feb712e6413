"""Where the B = 1 decode attention (k_attn_decode_qs) spends its time inside the c2 step: per-workgroup
s_memrealtime stamps (build variant -DZK_ATT_PROF=1, zonos_amd.build.build_variant) of the last attention
launch of a c2 generate (graph replay, 26 layers), at a few context lengths.
    ZK_LIB_PATH=zonos_amd/lib/variants/attprof/libzonos_hip.so python tools/attn_b1_stamps.py
Stamps: 0 entry, 1 context known, 2 first slice multiplied, 3 key loop done, 4 4-wave merge done, 5 end."""
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
cond = synthetic.conditioning(1, 160, 2048, seed=11, device=dev)
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)
prof = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
assert lib.zk_att_prof_set(prof.data_ptr()) == 0
names = ["entry", "ctx", "slice1", "loop", "merged", "end"]
for new in (100, 400, 800):
    prof.zero_()
    eng.generate(cond, None, new, 2.0, 1, sp, seed=5, force_full_length=True, poll_every=64)
    torch.cuda.synchronize()
    p = prof.view(-1, 8)[:, :6].cpu()
    used = p[:, 0] > 0
    p = p[used].double()
    t0 = p[:, 0].min()
    rel = (p - t0) / 100.0          # s_memrealtime: 100 MHz -> us
    ctx = 160 + new + 9
    print(f"ctx ~{ctx}: {int(used.sum())} workgroups; stamps (us from the first entry): "
          + "  ".join(f"{n} {rel[:, i].mean():.2f} [{rel[:, i].min():.2f}..{rel[:, i].max():.2f}]"
                      for i, n in enumerate(names)), flush=True)
