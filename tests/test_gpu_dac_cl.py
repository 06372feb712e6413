"""Channels-last fp16 DAC kernels (dac_cl.hip) vs plain PyTorch fp32 references of the same op
on the same fp16-rounded operands: RVQ lookup, Conv1d / ConvTranspose1d with the fused
Snake/residual epilogue, and the tail conv."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from zonos_amd import _lib
    _lib.load()
    return _lib


def _snake(x, a):
    a = a.view(1, 1, -1)
    return x + (a + 1e-9).reciprocal() * torch.sin(a * x).pow(2)


def _prep(w, mode, s=1):
    """fp16 [phase][tap][Cout][Cin] via zk_dac_prep_w16 (as the decoder does)."""
    L = _lib()
    if mode == 0:
        co, ci, ks = w.shape
        n = ks * co * ci
    else:
        ci, co, _ = w.shape
        ks, n = 2, s * 2 * co * ci
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    L.call("zk_dac_prep_w16", L.ptr(w), co, ci, ks, s, mode, L.ptr(out), None, L.stream_ptr(w.device))
    return out


CONV_CASES = [  # Cin, Cout, ks, dil, T, resid
    (64, 128, 7, 1, 300, False),
    (96, 96, 7, 9, 517, True),
    (96, 96, 1, 1, 200, True),
    (192, 192, 7, 3, 260, False),
    (1024, 1536, 7, 1, 40, False),
    (384, 384, 1, 1, 129, True),
    (192, 192, 1, 1, 300, True),
]


# More tiles than resident workgroups (each persistent workgroup streams >= 2 tiles through its
# loader rings, dac_cl.hip:148-160): the fat 12-wave k7 form (96 / 192 channels, 512-position tiles,
# one workgroup per CU), the residual 1x1 form and the FM = 4 k7 form (two per CU, 128 positions).
MULTITILE_CASES = [
    (96, 96, 7, 3, 120000, False),
    (192, 192, 7, 1, 70000, False),
    (96, 96, 1, 1, 60000, True),
    (384, 384, 1, 1, 30000, True),
    (1024, 1536, 7, 1, 4000, False),
]


def _min_tiles_per_wg(B, T, Cout, resid):
    nco = Cout // 32
    FM = 4 if nco % 4 == 0 else 3 if nco % 3 == 0 else 2 if nco % 2 == 0 else 1
    fat = not resid and FM <= 3
    qt = 512 if fat else 128
    ntiles = B * (-(-T // qt)) * (Cout // (32 * FM))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    return ntiles // (ncu * (1 if fat else 2))


@pytest.mark.parametrize("Cin,Cout,ks,dil,T,use_resid", CONV_CASES + MULTITILE_CASES)
def test_conv_cl_vs_torch(Cin, Cout, ks, dil, T, use_resid):
    L = _lib()
    if T >= 4000:
        assert _min_tiles_per_wg(3, T, Cout, use_resid) >= 2
    torch.manual_seed(Cin + Cout + ks + dil)
    dev = "cuda"
    B = 3
    lens = torch.tensor([T, T // 2, 1], dtype=torch.int32, device=dev)
    x = torch.randn(B, T, Cin, device=dev).half()
    w = (torch.randn(Cout, Cin, ks, device=dev) / math.sqrt(Cin * ks)).float()
    bias = torch.randn(Cout, device=dev) * 0.1
    alpha = torch.rand(Cout, device=dev) + 0.5
    resid = torch.randn(B, T, Cout, device=dev) if use_resid else None
    w16 = _prep(w, 0)
    xo = torch.empty(B, T, Cout, device=dev)
    so = torch.full((B, T, Cout), 12345, dtype=torch.int16, device=dev)
    pad = (ks - 1) // 2 * dil
    L.call("zk_dac_conv_cl", L.ptr(x), B, Cin, T, L.ptr(w16), 0, L.ptr(bias), Cout, ks, dil, pad, T, 1, 1, 0, T,
           L.ptr(resid), L.ptr(xo), L.ptr(alpha), L.ptr(so), 0, L.ptr(lens), 1, 1, L.stream_ptr(torch.device(dev)))
    torch.cuda.synchronize()
    # reference: per row, inputs beyond the row's length are zero, outputs beyond it zero
    xin = x.float().clone()
    for b in range(B):
        xin[b, int(lens[b]):] = 0
    y = F.conv1d(xin.transpose(1, 2), w.half().float(), bias, padding=pad, dilation=dil).transpose(1, 2)
    if use_resid:
        y = y + resid
    for b in range(B):
        y[b, int(lens[b]):] = 0
    s_ref = _snake(y, alpha)
    err = (xo - y).abs().max().item()
    assert err < 2e-3 * max(1.0, y.abs().max().item()), err
    s_got = so.view(torch.float16).float()
    assert (s_got - s_ref).abs().max().item() < 1e-2 * max(1.0, s_ref.abs().max().item())
    assert torch.all(s_got[1, int(lens[1]):] == 0)
    # fp32 Snake output variant (feeds the tail)
    s32 = torch.empty(B, T, Cout, device=dev)
    L.call("zk_dac_conv_cl", L.ptr(x), B, Cin, T, L.ptr(w16), 0, L.ptr(bias), Cout, ks, dil, pad, T, 1, 1, 0, T,
           L.ptr(resid), None, L.ptr(alpha), L.ptr(s32), 1, L.ptr(lens), 1, 1, L.stream_ptr(torch.device(dev)))
    torch.cuda.synchronize()
    assert (s32 - s_ref).abs().max().item() < 2e-3 * max(1.0, s_ref.abs().max().item())


# the fused residual unit (zk_dac_resunit_cl): C = 96 in 512-position tiles, C = 192 in 256-position
# tiles, one workgroup per CU; the long cases give >= 2 tiles per persistent workgroup
@pytest.mark.parametrize("C,dil,T", [(96, 1, 300), (96, 3, 517), (96, 9, 1000), (96, 3, 120000),
                                     (192, 1, 300), (192, 9, 1000), (192, 3, 70000)])
def test_resunit_fused_vs_pair_and_torch(C, dil, T):
    L = _lib()
    B, dev = 3, "cuda"
    assert L.load().zk_dac_resunit_supported(384) == 0      # (96 / 192: the product fuses, variants may not)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if T >= 50000:
        assert B * (-(-T // (512 if C == 96 else 256))) >= 2 * ncu
    torch.manual_seed(C + dil * 1000 + T)
    st = L.stream_ptr(torch.device(dev))
    lens = torch.tensor([T, T // 2, 1], dtype=torch.int32, device=dev)
    s_in = torch.randn(B, T, C, device=dev).half()
    x0 = torch.randn(B, T, C, device=dev)
    w7 = (torch.randn(C, C, 7, device=dev) / math.sqrt(C * 7)).float()
    w1 = (torch.randn(C, C, 1, device=dev) / math.sqrt(C)).float()
    b7, b1 = torch.randn(C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    a2, an = torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) + 0.5
    w7h, w1h = _prep(w7, 0), _prep(w1, 0)
    # the unfused pair (k7 -> fp16 s2; 1x1 + residual -> x, next Snake)
    tmp = torch.empty(B, T, C, dtype=torch.int16, device=dev)
    x_pair, s_pair = x0.clone(), torch.empty(B, T, C, dtype=torch.int16, device=dev)
    L.call("zk_dac_conv_cl", L.ptr(s_in), B, C, T, L.ptr(w7h), 0, L.ptr(b7), C, 7, dil, 3 * dil, T, 1, 1, 0, T,
           None, None, L.ptr(a2), L.ptr(tmp), 0, L.ptr(lens), 1, 1, st)
    L.call("zk_dac_conv_cl", L.ptr(tmp), B, C, T, L.ptr(w1h), 0, L.ptr(b1), C, 1, 1, 0, T, 1, 1, 0, T,
           L.ptr(x_pair), L.ptr(x_pair), L.ptr(an), L.ptr(s_pair), 0, L.ptr(lens), 1, 1, st)
    # fused, fp16 and fp32 Snake outputs
    x_f, s_f = x0.clone(), torch.full((B, T, C), 12345, dtype=torch.int16, device=dev)
    L.call("zk_dac_resunit_cl", L.ptr(s_in), B, C, T, L.ptr(w7h), L.ptr(b7), dil, L.ptr(a2), L.ptr(w1h), L.ptr(b1),
           L.ptr(x_f), L.ptr(an), L.ptr(s_f), 0, L.ptr(lens), 1, st)
    x_f32, s_f32 = x0.clone(), torch.empty(B, T, C, device=dev)
    L.call("zk_dac_resunit_cl", L.ptr(s_in), B, C, T, L.ptr(w7h), L.ptr(b7), dil, L.ptr(a2), L.ptr(w1h), L.ptr(b1),
           L.ptr(x_f32), L.ptr(an), L.ptr(s_f32), 1, L.ptr(lens), 1, st)
    with pytest.raises(L.ZonosHipError, match="alias"):
        L.call("zk_dac_resunit_cl", L.ptr(s_in), B, C, T, L.ptr(w7h), L.ptr(b7), dil, L.ptr(a2), L.ptr(w1h),
               L.ptr(b1), L.ptr(x_f32), L.ptr(an), L.ptr(s_in), 0, L.ptr(lens), 1, st)
    torch.cuda.synchronize()
    # fused vs pair: the same k7 sums; the 1x1 sums grouped 16- instead of 32-deep (fp32 rounding only)
    scale = max(1.0, x_pair.abs().max().item())
    assert (x_f - x_pair).abs().max().item() < 1e-5 * scale
    assert torch.equal(x_f, x_f32)
    sp, sf = s_pair.view(torch.float16).float(), s_f.view(torch.float16).float()
    assert (sf - sp).abs().max().item() < 2e-3 * max(1.0, sp.abs().max().item())
    assert (sf != sp).float().mean().item() < 1e-3
    for b in range(B):
        assert torch.all(x_f[b, int(lens[b]):] == 0) and torch.all(sf[b, int(lens[b]):] == 0)
    # fp32 torch reference of the unit on the same fp16 operands
    xin = s_in.float().clone()
    for b in range(B):
        xin[b, int(lens[b]):] = 0
    y = F.conv1d(xin.transpose(1, 2), w7.half().float(), b7, padding=3 * dil, dilation=dil).transpose(1, 2)
    s2 = _snake(y, a2).half().float()
    v = x0 + (s2 @ w1[:, :, 0].half().float().t() + b1)
    for b in range(B):
        v[b, int(lens[b]):] = 0
    assert (x_f - v).abs().max().item() < 2e-3 * max(1.0, v.abs().max().item())
    s_ref = _snake(v, an)
    assert (s_f32 - s_ref).abs().max().item() < 2e-3 * max(1.0, s_ref.abs().max().item())


@pytest.mark.parametrize("Cin,Cout,st,T", [(192, 96, 2, 70), (1536, 768, 8, 12), (384, 192, 4, 33),
                                          (192, 96, 2, 40000), (768, 384, 4, 9000)])
def test_convt_cl_vs_torch(Cin, Cout, st, T):
    L = _lib()
    torch.manual_seed(st + T)
    dev = "cuda"
    B = 2
    lens = torch.tensor([T, T - 5], dtype=torch.int32, device=dev)
    x = torch.randn(B, T, Cin, device=dev).half()
    w = (torch.randn(Cin, Cout, 2 * st, device=dev) / math.sqrt(Cin * 2)).float()
    bias = torch.randn(Cout, device=dev) * 0.1
    alpha = torch.rand(Cout, device=dev) + 0.5
    w16 = _prep(w, 1, st)
    Lo = T * st
    xo = torch.empty(B, Lo, Cout, device=dev)
    so = torch.empty(B, Lo, Cout, dtype=torch.int16, device=dev)
    L.call("zk_dac_conv_cl", L.ptr(x), B, Cin, T, L.ptr(w16), 2 * Cout * Cin, L.ptr(bias), Cout, 2, 1, 1, T + 1, st, st,
           -((st + 1) // 2), Lo, None, L.ptr(xo), L.ptr(alpha), L.ptr(so), 0, L.ptr(lens), 1, st,
           L.stream_ptr(torch.device(dev)))
    torch.cuda.synchronize()
    ys = []
    for b in range(B):
        n = int(lens[b])
        xb = x[b:b + 1, :n].float().transpose(1, 2)
        yb = F.conv_transpose1d(xb, w.half().float(), bias, stride=st, padding=math.ceil(st / 2),
                                output_padding=st % 2).transpose(1, 2)[0]
        full = torch.zeros(Lo, Cout, device=dev)
        full[:n * st] = yb
        ys.append(full)
    y = torch.stack(ys)
    err = (xo - y).abs().max().item()
    assert err < 2e-3 * max(1.0, y.abs().max().item()), err
    s_ref = _snake(y, alpha)
    s_got = so.view(torch.float16).float()
    assert (s_got - s_ref).abs().max().item() < 1e-2 * max(1.0, s_ref.abs().max().item())


def test_rvq_and_tail_cl_vs_torch():
    L = _lib()
    torch.manual_seed(3)
    dev = "cuda"
    st = L.stream_ptr(torch.device(dev))
    B, K, T, V, H = 2, 9, 50, 1024, 64
    tables = torch.randn(K, V, H, device=dev)
    codes = torch.randint(0, V, (B, K, T), device=dev)
    lens = torch.tensor([T, 20], dtype=torch.int32, device=dev)
    z = torch.empty(B, T, 96, dtype=torch.int16, device=dev)
    L.call("zk_dac_rvq_decode_cl", L.ptr(codes), B, K, T, K * T, L.ptr(tables), V, H, 96, L.ptr(z), L.ptr(lens), st)
    torch.cuda.synchronize()
    ref = torch.zeros(B, T, 96, device=dev)
    for b in range(B):
        for k in range(K):
            ref[b, :, :H] += tables[k][codes[b, k]]
        ref[b, int(lens[b]):] = 0
    assert torch.allclose(z.view(torch.float16).float(), ref, atol=1e-2, rtol=1e-3)

    C, Tt = 96, 1000
    s = torch.randn(B, Tt, C, device=dev)
    w = torch.randn(C, 7, device=dev) * 0.05
    bias = torch.randn(1, device=dev)
    out = torch.empty(B, Tt, device=dev)
    lens2 = torch.tensor([Tt, 600], dtype=torch.int32, device=dev)
    L.call("zk_dac_tail_cl", L.ptr(s), B, C, Tt, L.ptr(w), L.ptr(bias), L.ptr(out), L.ptr(lens2), 1, st)
    torch.cuda.synchronize()
    sin = s.float().clone()
    sin[1, 600:] = 0
    y = torch.tanh(F.conv1d(sin.transpose(1, 2), w.unsqueeze(0), bias, padding=3))[:, 0]
    y[1, 600:] = 0
    assert (out - y).abs().max().item() < 1e-4
