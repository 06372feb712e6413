"""A/B of the fused residual decode path (zk_gemm_resid + zk_gemm_ln, no k_resid_ln) against the
launch sequence with k_resid_ln, on one engine at the c3 shape (B = 64, Lc = 400, prefix 10):
decode ms per step (generate wall time / steps, graph replay), alternating, and the fp32 CFG logits
of a short teacher-free run compared between the two paths.

    python tools/fuse_ab.py [new_tokens] [reps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import synthetic  # noqa: E402
from zonos_amd.engine import EngineConfig, HipDecoder  # noqa: E402

new = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda")
mc = dict(synthetic.ZONOS_V01, n_layer=26)
W = synthetic.backbone_weights(dev, seed=0, **mc)
eng = HipDecoder(EngineConfig(**mc), W, dev)
del W
B = 64
cond = synthetic.conditioning(B, 400, mc["d_model"], seed=1, device=dev)
prefix = synthetic.prefix_codes(B, 10, seed=3, device=dev)
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)


def run(fuse, n, **kw):
    eng.fuse_resid = fuse
    eng._ws = None
    torch.cuda.synchronize()
    t = time.time()
    out = eng.generate(cond, prefix, n, 2.0, B, sp, seed=7, force_full_length=True, poll_every=64, **kw)
    torch.cuda.synchronize()
    return (time.time() - t) / (n + 8) * 1e3, out


for fuse in (True, False):
    eng.fuse_resid = fuse
    eng._ws = None
    ws = eng._alloc(B, 400, 10, 8)
    print("fuse", fuse, "->", ws.get("fuse"), flush=True)
# logits of the first steps, both paths (no graph: one step per poll)
logs = {}
for fuse in (True, False):
    tr = {}
    eng.fuse_resid = fuse
    eng._ws = None
    eng.generate(cond, prefix, 6, 2.0, B, sp, seed=7, force_full_length=True, trace=tr)
    logs[fuse] = torch.stack([t.float() for t in tr["logits"]])
fin = torch.isfinite(logs[False])
d = (logs[True] - logs[False])[fin].abs()
print(f"logits fused vs unfused over {logs[True].shape[0]} steps: max |d| {float(d.max()):.4f}, "
      f"mean {float(d.mean()):.5f}, mean |logit| {float(logs[False][fin].abs().mean()):.3f}", flush=True)
for r in range(reps):
    for fuse in (True, False):
        ms, _ = run(fuse, new)
        print(f"rep {r} fuse={fuse}: {ms:.4f} ms per decode step ({new} tokens)", flush=True)
