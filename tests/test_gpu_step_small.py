"""The persistent small-batch decode step (zk_decode_small, csrc/step_small.hip) against the
launch sequence it replaces, at the full Zonos-v0.1-transformer geometry.

zk_decode_small runs the arithmetic of the five-launch-per-block path (zk_gemv_fused with 4
K-quarter waves, i.e. ZK_GF_LAYOUT=1, + the unsplit fused decode attention), so for B = 1 and 2
(R = 2, 4 rows) its logits and codes must be BIT-IDENTICAL to that path. The comparison runs in a
child process because the GEMV layout knob is read once per process. Parity of the persistent path
against the reference itself is test_gpu_fullwidth.py (c1 free-running greedy codes, c2 logits),
which now runs through it (B = 1)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch, numpy as np
sys.path.insert(0, sys.argv[1])
from tests.golden_util import CLI_SP, FULL, full_weights
from oracle import zonos_ref
from zonos_amd.engine import EngineConfig, HipDecoder
cfg = EngineConfig(d_model=FULL.d_model, n_layer=FULL.n_layer, n_heads=FULL.n_heads, n_kv=FULL.n_kv,
                   d_ff=FULL.d_ff, eps=FULL.eps)
eng = HipDecoder(cfg, full_weights("random"), "cuda")
for B, T in ((1, 48), (2, 24)):
    cond = zonos_ref.synthetic_conditioning(B, 24, FULL.d_model, seed=1).cuda()
    res = {}
    for persist in (True, False):
        eng.release()
        eng.persistent_small = persist
        tr = {}
        out = eng.generate(cond, None, T, 2.0, B, CLI_SP, seed=5, trace=tr)          # eager
        out_g = eng.generate(cond, None, T, 2.0, B, CLI_SP, seed=5)                   # hipGraph replays
        assert all(torch.equal(a, b) for a, b in zip(out, out_g)), "graph != eager"
        assert ("small" in eng._ws) == persist
        res[persist] = (out, [t.cpu() for t in tr["logits"]])
    (o1, l1), (o0, l0) = res[True], res[False]
    assert len(l1) == len(l0)
    for s, (a, b) in enumerate(zip(l1, l0)):
        assert torch.equal(a, b), f"B={B}: step {s} logits differ (max {(a - b).abs().max().item()})"
    for a, b in zip(o1, o0):
        assert torch.equal(a, b), f"B={B}: codes differ"
    print(f"B={B}: {len(l1)} steps of logits and {sum(x.shape[1] for x in o1)} frames bit-identical")
print("OK")
'''


@pytest.mark.timeout(500)
@pytest.mark.parametrize("splits", ["1", "2"])
def test_persistent_step_bit_identical_to_launch_sequence(splits):
    """splits = attention key splits of both paths (ZK_ATTN_SPLITS): 1 = one unit per (row, kv
    head); 2 = partials merged inside the launch by the last split to arrive (the launch path's
    in-launch combine, k_attn_decode COMB)."""
    env = dict(os.environ, ZK_GF_LAYOUT="1", ZK_ATTN_SPLITS=splits)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=600,
                       cwd=REPO)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-4000:]
