"""TEST INFRASTRUCTURE ONLY -- the oracle's copy of the engine's sampling-noise stream.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module. The product path (zonos_amd) generates the same stream on the GPU inside
the sampler kernel (zonos_amd/csrc/sampler.hip) and never calls this file.

Why a counter-based stream: the reference draws the exponential race noise with
``torch.empty_like(probs).exponential_(1)`` (zonos/sampling.py:26-28), i.e. from
torch's global generator, whose stream differs between CPU and CUDA and cannot be
reproduced inside a graph-captured HIP sampler. The engine instead keys every
noise value by (seed, step, draw, utterance, codebook, token) with Philox4x32-10,
so the codes are independent of launch geometry and of how utterances are
sharded across GPUs. Parity with the reference is pinned by injecting this same
stream into the reference's ``multinomial`` when generating the golden fixtures
(tests/golden/make_golden.py).

Noise definition (identical in sampler.hip):
    ctr  = (token, utterance*16 + codebook, step, draw)      (4 x uint32)
    key  = (seed & 0xffffffff, seed >> 32)
    x    = Philox4x32_10(ctr, key)[0]
    u    = ((x >> 8) + 0.5) * 2**-24                          (exact in f64, 0<u<1)
    q    = float32(-log(float64(u)))                          (Exp(1) sample)
The reference's multinomial then picks argmax(probs / q)  (zonos/sampling.py:27-28).
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11). All inputs uint32 arrays/scalars."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (a.copy() for a in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    for r in range(10):
        p0 = c0.astype(np.uint64) * _M0
        p1 = c2.astype(np.uint64) * _M1
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & _MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & _MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if r != 9:
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def exp_noise(seed: int, step: int, draw: int, batch: int, n_cb: int, vocab: int,
              row_base: int = 0) -> np.ndarray:
    """Exp(1) noise of shape [batch, n_cb, vocab] float32 for one sampler call."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0, k1 = seed & 0xFFFFFFFF, seed >> 32
    v = np.arange(vocab, dtype=np.uint32)[None, None, :]
    b = np.arange(batch, dtype=np.uint32)[:, None, None] + np.uint32(row_base)
    cb = np.arange(n_cb, dtype=np.uint32)[None, :, None]
    x, _, _, _ = philox4x32_10(v, b * np.uint32(16) + cb, np.uint32(step), np.uint32(draw), k0, k1)
    u = ((x >> np.uint32(8)).astype(np.float64) + 0.5) * (2.0 ** -24)
    return (-np.log(u)).astype(np.float32)
