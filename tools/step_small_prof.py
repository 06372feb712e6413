"""Phase anatomy of the persistent small-batch step (zk_decode_small with the prof buffer):
runs a B=1 c2-like generate to warm up, then launches the step kernel at a fixed context with
timestamps and prints per-phase-kind averages of: seam wait (all CUs), staging, GEMM/attention
body, signal; plus the loader's free-slot wait. Usage: python tools/step_small_prof.py [ctx]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from oracle import zonos_ref  # noqa: E402  (synthetic weights only)
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call  # noqa: E402
from zonos_amd.engine import EngineConfig, HipDecoder  # noqa: E402

ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 600
cfgz = zonos_ref.ZONOS_V01_TRANSFORMER
W = zonos_ref.make_weights(cfgz, seed=0)
cfg = EngineConfig(d_model=cfgz.d_model, n_layer=cfgz.n_layer, n_heads=cfgz.n_heads, n_kv=cfgz.n_kv, d_ff=cfgz.d_ff,
                   eps=cfgz.eps)
eng = HipDecoder(cfg, W, "cuda")
del W
cond = zonos_ref.synthetic_conditioning(1, 160, cfgz.d_model, seed=1).cuda()
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)
eng.generate(cond, None, 861, 2.0, 1, sp, seed=1, force_full_length=True)
ws = eng._ws
src = ws["small"]["args"]
a = type(src).from_buffer_copy(src)
pos = torch.full((1,), ctx - 1, dtype=torch.int32, device="cuda")
a.pos_dev = pos.data_ptr()
a.skip = None
NL = cfg.n_layer
ncu = torch.cuda.get_device_properties(0).multi_processor_count
prof = torch.zeros(ncu, NL * 5 + 2, 4, dtype=torch.int64, device="cuda")
stream = _lib.stream_ptr()
for it in range(6):
    a.prof = prof.data_ptr() if it == 5 else None
    call("zk_decode_small", C.byref(a), stream)
torch.cuda.synchronize()
eng._check_small(ws)
p = prof.cpu().numpy().astype(np.float64) * 10.0 / 1000.0      # 100 MHz ticks -> us
t0 = p[:, 0, 0].min()
step_end = p[:, NL * 5, 3].max()
print(f"ctx {ctx}: step (first seam start -> last heads end) {step_end - t0:.1f} us over {ncu} CUs")
names = ["IN", "ATT", "OUT", "FC1", "FC2"]
rows = []
for k in range(5):
    idx = [l * 5 + k for l in range(NL)]
    seam = (p[:, idx, 1] - p[:, idx, 0])
    stage = (p[:, idx, 2] - p[:, idx, 1])
    body = (p[:, idx, 3] - p[:, idx, 2])
    span = (p[:, idx, 3].max(axis=0) - p[:, idx, 0].min(axis=0))     # per layer: first start -> last end
    rows.append((names[k], seam.mean(), seam.max(axis=0).mean(), stage.mean(), body.mean(), body.max(axis=0).mean(),
                 span.mean()))
print(f"{'phase':5s} {'seam avg':>9s} {'seam max':>9s} {'stage':>7s} {'body avg':>9s} {'body max':>9s} {'span':>7s}  (us, mean over layers)")
for r in rows:
    print(f"{r[0]:5s} {r[1]:9.2f} {r[2]:9.2f} {r[3]:7.2f} {r[4]:9.2f} {r[5]:9.2f} {r[6]:7.2f}")
h = NL * 5
print(f"heads: seam {np.mean(p[:, h, 1] - p[:, h, 0]):.2f} stage {np.mean(p[:, h, 2] - p[:, h, 1]):.2f} "
      f"body {np.mean(p[:, h, 3] - p[:, h, 2]):.2f}")
L = p[:, NL * 5 + 1]
print(f"loader: run {np.mean(L[:, 1] - L[:, 0]):.1f} us (max {np.max(L[:, 1] - L[:, 0]):.1f}), free-slot wait "
      f"{np.mean(L[:, 2]) * 1.0:.1f} us avg, slots {int(L[0, 3])}")
per_layer = [(p[:, l * 5 + 4, 3].max() - p[:, l * 5, 0].min()) for l in range(NL)]
print("layer spans (us):", " ".join(f"{x:.1f}" for x in per_layer))
