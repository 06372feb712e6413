"""TEST INFRASTRUCTURE ONLY -- restatement of torch's GPU `Tensor.exponential_(1)` stream.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product generates the same stream on the GPU (zonos_amd/csrc/sampler.hip, torch noise mode)
and never calls this file.

The reference draws the race noise of its sampler as
``torch.empty_like(probs).exponential_(1)`` (zonos/sampling.py:26-28) from torch's global
generator; on a ROCm GPU that call runs (torch 2.10, headers under torch/include):
  * ATen/native/hip/DistributionTemplates.h:52-63 calc_execution_policy: block 256, grid =
    min(multiProcessorCount * (maxThreadsPerMultiProcessor / 256), ceil(n / 256)); the call takes
    the generator's Philox (seed, offset) and advances the offset by
    ((n - 1) / (256 * grid * 4) + 1) * 4;
  * :66-91 distribution_elementwise_grid_stride_kernel: thread idx = hiprand_init(seed,
    subsequence = idx, offset); loop iteration j draws hiprand_uniform4 (one Philox4x32-10 block,
    counter (offset / 4 + j, idx), rocrand/rocrand_philox4x32_10.h) and element
    idx + (4 j + ii) * stride takes word ii;
  * rocrand/rocrand_uniform.h:66-68: u = 2^-32 + word * 2^-32 (float32, in (0, 1]);
  * ATen/core/TransformationHelper.h:129-146 exponential: log = u >= 1 - eps/2 ? -eps/2 :
    at::log(u) (device: __logf, ATen/NumericUtils.h:150-160); q = -1 / lambda * log.
The words and u are reproduced exactly here. The float32 log is the device's: torch's __logf is
the hardware log2 (v_log_f32, not correctly rounded) times ln2 in extended precision (ln2 = hi + lo
floats, one fma; tools/torch_noise_probe.py). `exp_noise` follows that formula with a correctly
rounded log2, so it lands within 2 ulp of torch's values (72 % exactly on the fixture); the GPU test
compares the product kernel, which uses the hardware log2, with torch's output bit for bit.
"""
from __future__ import annotations

import numpy as np

from .philox import philox4x32_10

EPS_HALF = np.float32(2.0 ** -24)          # numeric_limits<float>::epsilon() / 2
INV32 = np.float32(2.0 ** -32)             # ROCRAND_2POW32_INV


def policy(n: int, mp_count: int, max_threads_per_mp: int) -> tuple[int, int]:
    """(stride, offset increment) of one exponential_ call over n elements."""
    grid = min(mp_count * (max_threads_per_mp // 256), (n + 255) // 256)
    stride = 256 * grid
    return stride, ((n - 1) // (stride * 4) + 1) * 4


def words(n: int, seed: int, offset: int, stride: int) -> np.ndarray:
    """The uint32 Philox word each of the n elements takes (exact)."""
    e = np.arange(n, dtype=np.int64)
    t = e % stride
    q = e // stride
    ctr = np.uint64(offset // 4) + (q >> 2).astype(np.uint64)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c0 = (ctr & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    c1 = (ctr >> np.uint64(32)).astype(np.uint32)
    c2 = (t & 0xFFFFFFFF).astype(np.uint32)
    c3 = (t >> 32).astype(np.uint32)
    r = philox4x32_10(c0, c1, c2, c3, seed & 0xFFFFFFFF, seed >> 32)
    out = np.empty(n, dtype=np.uint32)
    for ii in range(4):
        m = (q & 3) == ii
        out[m] = r[ii][m]
    return out


def uniforms(w: np.ndarray) -> np.ndarray:
    """hiprand_uniform4's float32 u in (0, 1] (the product of a uint32 and 2^-32 is exact)."""
    return (INV32 + w.astype(np.float32) * INV32).astype(np.float32)


LN2_HI = np.array([0x3F317218], dtype=np.uint32).view(np.float32)[0]
LN2_LO = np.array([0xB102E308], dtype=np.uint32).view(np.float32)[0]


def exp_noise(n: int, seed: int, offset: int, stride: int) -> np.ndarray:
    """Exp(1) values of one call (float32; log = fma(y, ln2_hi, y * ln2_lo) with y = log2(u), see
    the header)."""
    u = uniforms(words(n, seed, offset, stride))
    y = np.log2(u.astype(np.float64)).astype(np.float32)
    lo = (y * LN2_LO).astype(np.float32)
    lg = (y.astype(np.longdouble) * np.longdouble(LN2_HI) + np.longdouble(lo)).astype(np.float32)
    lg = np.where(u >= np.float32(1.0) - EPS_HALF, -EPS_HALF, lg)
    return (-lg).astype(np.float32)
