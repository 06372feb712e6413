"""CPU: the C-ABI library builds/loads and exports every symbol include/zonos_hip.h declares;
host-side logic that needs no GPU."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "zonos_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from zonos_amd import build
    path = build.build()
    return ctypes.CDLL(path)


def test_library_exports_header(lib):
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in zonos_hip.h but not exported"


def test_python_binding_covers_header():
    from zonos_amd import _lib
    assert set(header_symbols()) == set(_lib.exported_symbols())


def test_version_and_error_without_gpu(lib):
    lib.zk_version.restype = ctypes.c_int
    assert lib.zk_version() >= 1
    lib.zk_last_error.restype = ctypes.c_char_p
    assert isinstance(lib.zk_last_error(), bytes)


def test_argument_validation_without_gpu(lib):
    # shape checks run on the host before any launch
    rc = lib.zk_gemm_bf16(None, ctypes.c_long(100), None, 0, 10, 64, 1, 0, None, None, None, None)
    assert rc != 0
    lib.zk_last_error.restype = ctypes.c_char_p
    assert b"zk_gemm_bf16" in lib.zk_last_error()


def test_prefill_rejects_short_kv_cache_without_gpu(lib):
    """zk_prefill / zk_hybrid_prefill refuse a descriptor whose KV cache (smax keys) is shorter than
    the context of the last decode step (Lc + Ld), before any launch: the decode attention's context
    clamp is then only ever reached by no-op launches after the last step."""
    import ctypes as C

    from zonos_amd import _lib
    lays = (_lib.StepLayer * 1)()
    d = _lib.StepDesc()
    d.B, d.n_layer, d.d_model, d.smax, d.layers = 1, 1, 64, 256, C.cast(lays, C.c_void_p)
    d.st.Ld, d.st.K, d.st.V = 250, 9, 1026
    buf = C.create_string_buffer(16)
    lib.zk_last_error.restype = C.c_char_p
    assert lib.zk_prefill(C.byref(d), buf, 10, 0, buf, None) != 0      # 10 + 250 > 256
    assert b"KV cache" in lib.zk_last_error()


def test_gemm_warm_up_stays_inside_packed_image(lib):
    """The L2 warm-up a kernel issues for the next decode GEMM reads only tiles of that GEMM's packed
    weight image (the 48-column workgroups of the c5 Mamba in_proj -- N = 8512, 178 x 3 =
    534 tiles -- warmed 2 tiles past the 532-tile image). Every decode GEMM shape of c2-c5 at R = 128
    and R = 24, each split the engine may pick."""
    lib.zk_gemm_warm_tiles.restype = ctypes.c_int
    shapes = [(3072, 2048), (2048, 2048), (16384, 2048), (2048, 8192), (9234, 2048), (8512, 2048),
              (2048, 4096), (9280, 2048), (4400, 2048), (1000, 2048)]
    seen_narrow = False
    for M in (24, 72, 128):
        for N, K in shapes:
            for nsplit in (1, 2, 4, 8):
                if K % (nsplit * 64) or K // nsplit // 64 > 32:
                    continue
                for mode in (0, 1):
                    if mode == 1 and (nsplit != 1 or N % 16):
                        continue
                    t = lib.zk_gemm_warm_tiles(M, N, K, nsplit, mode, 2)
                    assert 0 <= t <= (N + 15) // 16, (M, N, K, nsplit, mode, t)
                    seen_narrow |= (N == 8512 and M == 128 and nsplit == 1 and t > 0)
    assert seen_narrow


def test_split_selection_batch_invariant():
    from zonos_amd.engine import _split_for
    for N, K in ((3072, 2048), (2048, 2048), (2048, 8192), (9234, 2048)):
        s = _split_for(N, K, 128)
        assert K % (s * 64) == 0
        assert all(_split_for(N, K, m) == s for m in (2, 8, 64, 128))
        assert ((N + 63) // 64) * s >= 128


def test_attention_split_rule():
    """Flash-decoding key splits: none at B=64 (512 workgroups already), and each split covers
    >= 2048 cached keys (a combine launch costs more than it saves below that)."""
    from zonos_amd.engine import attn_merge_for, attn_splits_for
    # B = 1: 4 splits of 32-key slices at every cache size (round-6 A/B, c2 decode step at
    # 2 / 4 / 8 splits: 0.975-0.978 / 0.959-0.962 / 0.977-0.980 ms, profiles/r6_c2_split_ab.txt)
    assert attn_merge_for(2, 1280) == 4 and attn_merge_for(2, 256) == 4 and attn_merge_for(1 * 2, 3328) == 4
    assert attn_merge_for(4, 1280) == 0 and attn_merge_for(128, 3072) == 0
    assert attn_splits_for(128, 4, 3072) == 1           # c3
    assert attn_splits_for(2, 4, 1280) == 1             # c2: B=1, 10 s
    assert attn_splits_for(2, 4, 3328) == 2             # B=1, 30 s
    for R in (2, 8, 16, 64, 128):
        for smax in (256, 1024, 3072, 8192):
            s = attn_splits_for(R, 4, smax)
            assert 1 <= s <= max(1, smax // 128) and (s == 1 or smax / s >= 1024)


def test_kv_layout_pack_roundtrip():
    """zonos_amd.kvlayout (host view of backbone.hip k_off / v_off): pack/unpack are inverse
    and element positions follow the documented fragment order."""
    import torch
    from zonos_amd.kvlayout import pack_k, pack_v, unpack_k, unpack_v
    R, Hk, S = 2, 3, 64
    k, v = torch.randn(R, Hk, S, 128), torch.randn(R, Hk, S, 128)
    kp, vp = pack_k(k), pack_v(v)
    assert torch.equal(unpack_k(kp, S), k) and torch.equal(unpack_v(vp, S), v)
    for key in (0, 5, 13, 31, 37, 63):
        o = key & 31
        ln = 4 * (o >> 3) + (o & 3)
        h = (o >> 2) & 1
        for c8 in (0, 3, 7, 15):
            off = (key >> 5) * 4096 + ((h * 4 + (c8 >> 2)) * 64 + (c8 & 3) * 16 + ln) * 8
            assert torch.equal(kp[1, 2, off:off + 8], k[1, 2, key, 8 * c8:8 * c8 + 8])
        for ch in (0, 17, 127):
            off = (key >> 5) * 4096 + ((ch >> 4) * 64 + (o >> 3) * 16 + (ch & 15)) * 8 + (o & 7)
            assert vp[1, 2, off] == v[1, 2, key, ch]


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the by-value/by-pointer structs (ZkCondPlan, sampling params, generation
    state) have the C compiler's size and field offsets."""
    import ctypes as C
    import shutil
    import subprocess

    from zonos_amd import _lib as zl
    from zonos_amd.conditioning import ZkCondPlan, ZkCondSeg
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "zonos_hip.h")
    src = tmp_path / "layout.c"
    src.write_text(f'#include "{hdr}"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(ZkCondSeg), sizeof(ZkCondPlan),'
                   ' offsetof(ZkCondPlan, seg), offsetof(ZkCondSeg, table), offsetof(ZkCondPlan, norm_w),'
                   ' sizeof(zk_sampling_params)); return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(ZkCondSeg), C.sizeof(ZkCondPlan), ZkCondPlan.seg.offset, ZkCondSeg.table.offset,
                   ZkCondPlan.norm_w.offset, C.sizeof(zl.SamplingParams)]


def test_ctypes_struct_layouts_match_the_c_abi(lib):
    """The by-value / by-pointer ABI structs the Python binding builds (SamplingParams, GenState,
    ZkCondSeg, ZkCondPlan, StepLayer, StepDesc, DacDesc) have the C compiler's size and field offsets."""
    import ctypes as C

    from zonos_amd import _lib
    from zonos_amd.conditioning import ZkCondPlan, ZkCondSeg
    lib.zk_abi_size.restype = C.c_long
    lib.zk_abi_size.argtypes = [C.c_int]
    for which, cls in [(0, _lib.SamplingParams), (1, _lib.GenState), (4, ZkCondSeg), (5, ZkCondPlan)]:
        assert lib.zk_abi_size(which) == C.sizeof(cls), (cls.__name__, lib.zk_abi_size(which), C.sizeof(cls))
    assert lib.zk_abi_size(12) == _lib.GenState.seed.offset
    assert lib.zk_abi_size(22) == _lib.GenState.noise_offset.offset
    assert lib.zk_abi_size(6) == C.sizeof(_lib.StepLayer) and lib.zk_abi_size(7) == C.sizeof(_lib.StepDesc)
    assert lib.zk_abi_size(13) == _lib.StepDesc.eps.offset
    assert lib.zk_abi_size(14) == _lib.StepDesc.st.offset and lib.zk_abi_size(15) == _lib.StepDesc.sp.offset
    assert lib.zk_abi_size(8) == C.sizeof(_lib.DacDesc) and lib.zk_abi_size(17) == C.sizeof(_lib.DacBlock)
    assert lib.zk_abi_size(16) == _lib.DacDesc.blocks.offset
    assert lib.zk_abi_size(18) == C.sizeof(_lib.HybridLayer) and lib.zk_abi_size(19) == C.sizeof(_lib.HybridDesc)
    assert lib.zk_abi_size(20) == _lib.HybridDesc.st.offset and lib.zk_abi_size(21) == _lib.HybridDesc.eps.offset


