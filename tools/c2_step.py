"""c2 decode-step timing (B = 1, Lc 160, no prefix, 861 new tokens: BASELINE configs[1]) for A/Bs of
the B = 1 path: `python tools/c2_step.py [merge ...]` times generate() on the current library
(ZK_LIB_PATH) for each attention split count (engine.ATTN_MERGE_DEFAULT), interleaved, and prints the
decode ms per step of every run. Developer tool, not part of the product."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import engine, synthetic  # noqa: E402
from zonos_amd.engine import EngineConfig, HipDecoder  # noqa: E402

merges = [int(a) for a in sys.argv[1:]] or [engine.ATTN_MERGE_DEFAULT]
reps = int(os.environ.get("ZK_C2_REPS", "3"))
dev = torch.device("cuda", 0)
eng = HipDecoder(EngineConfig(**synthetic.ZONOS_V01), synthetic.backbone_weights(dev, seed=0), dev)
cond = synthetic.conditioning(1, 160, 2048, seed=11, device=dev)
sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
          repetition_penalty_window=8, temperature=1.0)
lib = os.environ.get("ZK_LIB_PATH", "product")
for r in range(reps + 1):
    for m in merges:
        engine.ATTN_MERGE_DEFAULT = m
        eng.release()
        torch.cuda.synchronize()
        t = time.time()
        eng.generate(cond, None, 861, 2.0, 1, sp, seed=5, force_full_length=True, poll_every=64)
        torch.cuda.synchronize()
        dt = time.time() - t
        if r:
            print(f"c2 {lib} merge={m}: {dt / 869 * 1e3:.4f} ms/step (incl. prefill) ws.merge={eng._ws['attn_merge']}",
                  flush=True)
