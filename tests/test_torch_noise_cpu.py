"""CPU checks of the torch-noise restatement (oracle/torch_philox.py) against torch's own GPU
`exponential_` output (tests/golden/torch_exp_noise.npz, written on an MI355X by
tests/golden/make_torch_noise.py with torch alone), and of the host-side policy in the library."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import torch_philox

G = os.path.join(os.path.dirname(__file__), "golden", "torch_exp_noise.npz")


def _fixture():
    if not os.path.exists(G):
        pytest.skip("torch_exp_noise.npz not generated yet")
    return np.load(G)


def test_offset_increment_and_policy_match_torch():
    """The generator offset torch advanced by on the GPU == the policy's increment."""
    d = _fixture()
    mp, mt = int(d["mp_count"]), int(d["max_threads_per_mp"])
    for i in range(int(d["n_cases"])):
        n = int(d[f"c{i}_n"])
        _, incr = torch_philox.policy(n, mp, mt)
        assert int(d[f"c{i}_off_after"]) - int(d[f"c{i}_off"]) == incr, (i, n)


def test_restatement_matches_torch_gpu_values():
    """Philox words and uniforms are integer-exact by construction; the float32 log is the
    device's own (hardware log2 x ln2), which the restatement's correctly rounded log2 matches to
    within 2 ulp (>= 60 % exactly). This pins torch's element -> (thread, iteration, word) mapping and
    the offsets: a mapping error would put ~100 % of the values far off. (Bit-exactness of the product
    kernel against torch is tests/test_gpu_torch_noise.py.)"""
    d = _fixture()
    mp, mt = int(d["mp_count"]), int(d["max_threads_per_mp"])
    total = exact = 0
    for i in range(int(d["n_cases"])):
        n, seed, off = int(d[f"c{i}_n"]), int(d[f"c{i}_seed"]), int(d[f"c{i}_off"])
        stride, _ = torch_philox.policy(n, mp, mt)
        q = torch_philox.exp_noise(n, seed, off, stride)[d[f"c{i}_idx"]]
        ref = d[f"c{i}_q"]
        ulp = np.abs(q.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert ulp.max() <= 2, (i, n, int(ulp.max()))
        total += q.size
        exact += int((ulp == 0).sum())
    assert exact >= 0.6 * total, (exact, total)


def test_library_policy_matches_oracle():
    from zonos_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = C.CDLL(_lib.LIB_PATH)
    lib.zk_torch_noise_policy.restype = C.c_int
    lib.zk_torch_noise_policy.argtypes = [C.c_long, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_long)]
    for mp, mt in ((256, 2048), (304, 2048), (80, 1024)):
        for n in (1, 17, 256, 257, 9234, 590976, 2 ** 21, 2 ** 21 + 1, 2770200):
            s, inc = C.c_int(), C.c_long()
            assert lib.zk_torch_noise_policy(n, mp, mt, C.byref(s), C.byref(inc)) == 0
            assert (s.value, inc.value) == torch_philox.policy(n, mp, mt), (n, mp, mt)
