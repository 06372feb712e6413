"""Anatomy of the B = 1 GEMV launches (k_gemv_f) inside the c2 step: per-workgroup s_memrealtime stamps
(build variant -DZK_GF_PROF=1) of the last launch of each kind in a c2 generate (graph replay).
    ZK_LIB_PATH=zonos_amd/lib/variants/gfprof/libzonos_hip.so python tools/gemv_b1_stamps.py
Stamps: 0 entry, 1 first k-step multiplied (its weights landed), 2 last k-step multiplied, 3 K-quarters
reduced (then the epilogue stores). Times in us from the launch's first workgroup entry."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib, synthetic  # noqa: E402
from zonos_amd.engine import EngineConfig, HipDecoder  # noqa: E402

lib = _lib.load()
lib.zk_gf_prof_set.argtypes = [C.c_void_p]
dev = torch.device("cuda", 0)
eng = HipDecoder(EngineConfig(**synthetic.ZONOS_V01), synthetic.backbone_weights(dev, seed=0), dev)
cond = synthetic.conditioning(1, 160, 2048, seed=11, device=dev)
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)
prof = torch.zeros(8 * 2048 * 4, dtype=torch.int64, device=dev)
assert lib.zk_gf_prof_set(prof.data_ptr()) == 0
kinds = {0: "heads (mode 0, LN)", 2: "fc1 (mode 1, LN, SwiGLU)", 4: "fc2 (mode 2)", 5: "out_proj (mode 2 + merge)",
         6: "in_proj (mode 3, LN, RoPE)"}
eng.generate(cond, None, 400, 2.0, 1, sp, seed=5, force_full_length=True, poll_every=64)
torch.cuda.synchronize()
P = prof.view(8, 2048, 4).cpu()
for slot, name in kinds.items():
    p = P[slot]
    used = p[:, 0] > 0
    p = p[used].double()
    if not len(p):
        continue
    rel = (p - p[:, 0].min()) / 100.0
    qs = lambda v: f"{v.mean():6.2f} [p10 {v.quantile(0.1):5.2f} p90 {v.quantile(0.9):5.2f} max {v.max():5.2f}]"
    print(f"{name:28s} {int(used.sum()):4d} WGs: entry {qs(rel[:, 0])}  first-mfma {qs(rel[:, 1])}  "
          f"last-mfma {qs(rel[:, 2])}  reduced {qs(rel[:, 3])}", flush=True)
    # per-XCD (blockIdx % 8) finish
    idx = torch.nonzero(used).flatten()
    fin = [rel[(idx % 8) == x, 3].max().item() for x in range(8)]
    print(f"{'':28s} last 'reduced' per blockIdx%8: " + " ".join(f"{v:5.2f}" for v in fin), flush=True)
