"""GPU parity of the individual HIP kernels (through the C ABI) against the oracle /
golden vectors. Tolerances are written next to each comparison."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import zonos_ref
from oracle.philox import exp_noise

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from zonos_amd import _lib
    _lib.load()


def test_sampler_golden_exact():
    """Sampled tokens == reference tokens (reference run with the same Philox noise)."""
    from zonos_amd.sampling import sample_from_logits
    d = np.load(os.path.join(G, "sampler.npz"))
    mism = 0
    total = 0
    for ci in range(int(d["n_cases"])):
        sp = {k[len(f"sp_{ci}_"):]: float(d[k]) for k in d.files if k.startswith(f"sp_{ci}_")}
        sp["top_k"] = int(sp.get("top_k", 0))
        sp["repetition_penalty_window"] = int(sp["repetition_penalty_window"])
        sp.pop("repetition_penalty")
        logits = torch.from_numpy(d[f"logits_{ci}"]).to(DEV)
        tok = sample_from_logits(logits, generated_tokens=torch.from_numpy(d[f"gen_{ci}"].astype(np.int64)).to(DEV),
                                 repetition_penalty=torch.from_numpy(d[f"rp_{ci}"]), seed=int(d["seed"]), step=ci + 1,
                                 **sp)
        got = tok.squeeze(-1).cpu().numpy()
        exp = d[f"tok_{ci}"]
        mism += int((got != exp).sum())
        total += exp.size
        if sp.get("temperature", 1.0) == 0:
            assert np.array_equal(got, exp), f"greedy case {ci} must be bit-exact"
    # sampled cases: fp32 softmax/exp differ in the last ulp between CPU and GPU; a flip needs
    # an exact near-tie of probs/q. Allow at most 1 flipped token in all cases.
    assert mism <= 1, f"{mism}/{total} sampled tokens differ"


def test_noise_matches_oracle():
    """Exponential-race noise stream: one-hot logits expose argmax(p/q) = argmin over ties of q."""
    from zonos_amd.sampling import sample_from_logits
    B, K, V = 3, 9, 1026
    logits = torch.zeros(B, K, V, device=DEV)   # uniform probs -> token = argmin q
    for step in (0, 5):
        for draw in (0, 1):
            tok = sample_from_logits(logits, temperature=1.0, repetition_penalty=1.0, seed=99, step=step, draw=draw,
                                     row_base=7)
            q = exp_noise(99, step, draw, B, K, V, row_base=7)
            p = np.full((B, K, V), 1.0 / V, dtype=np.float32)
            exp = np.argmax(p / q, axis=-1)
            assert np.array_equal(tok.squeeze(-1).cpu().numpy(), exp)


def test_delay_pattern_golden():
    from zonos_amd.codebook_pattern import apply_delay_pattern, revert_delay_pattern
    d = np.load(os.path.join(G, "delay.npz"))
    codes = torch.from_numpy(d["codes"].astype(np.int64)).to(DEV)
    dl = apply_delay_pattern(codes, 1025)
    assert np.array_equal(dl.cpu().numpy(), d["delayed"])
    assert np.array_equal(revert_delay_pattern(dl).cpu().numpy(), d["reverted"])
    # empty time axis
    e = apply_delay_pattern(torch.zeros(2, 9, 0, dtype=torch.int64, device=DEV), 1025)
    assert e.shape == (2, 9, 9) and bool((e == 1025).all())


@pytest.mark.parametrize("M,N,K,nsplit", [(128, 3072, 2048, 8), (7, 1026 * 9, 256, 2), (300, 192, 512, 1),
                                          (128, 2048, 8192, 16), (2, 2048, 2048, 4), (20, 3072, 1024, 2),
                                          (64, 1168, 256, 4), (128, 3072, 2048, 1), (33, 1024, 8192, 1),
                                          # decode shapes (k_gemm_ws / k_gemv_rk)
                                          (128, 2048, 2048, 8), (128, 9234, 2048, 2), (128, 16384, 2048, 1),
                                          (128, 2048, 2048, 4), (100, 2048, 8192, 4), (1, 3072, 2048, 2),
                                          # < 192 tiles of 64 columns: 32-column workgroups (c5 Mamba in_proj)
                                          (128, 8512, 2048, 1), (72, 3000, 512, 1),
                                          # prefill shapes (k_gemm, M >= 1024)
                                          (1100, 256, 512, 1), (2048, 384, 2048, 1), (1024, 1152, 128, 1),
                                          # prefill shapes with >= 256 tiles of 256 x 256 (k_gemm_pf): ragged
                                          # last row block, N not a multiple of 256 (hybrid in_proj), K = 8192
                                          (16400, 4096, 1024, 1), (8300, 8512, 512, 1), (9000, 2048, 8192, 1)])
def test_gemm_vs_fp32(M, N, K, nsplit):
    from zonos_amd._lib import call, ptr, stream_ptr
    g = torch.Generator(device="cpu").manual_seed(M + N)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    from zonos_amd.engine import pack_weights
    Wpk = pack_weights(W, stream_ptr())
    part = torch.empty(nsplit, M, N, device=DEV)
    call("zk_gemm_bf16", ptr(A), K, ptr(Wpk), M, N, K, nsplit, 0, ptr(part), None, None, stream_ptr())
    got = part.sum(0)
    ref = A.float() @ W.float().t()
    # fp32 accumulation of bf16 products: error ~ K * eps32 * |a||w|
    assert torch.allclose(got, ref, atol=2e-3 * (K / 2048) ** 0.5, rtol=1e-3), (got - ref).abs().max()


@pytest.mark.parametrize("N,N2,nsplit", [(8512, 12288, 1), (9234, 10304, 2)])
def test_gemm_narrow_wide_workgroups_bit_identical(N, N2, nsplit):
    """k_gemm_ws workgroups of 3 waves (48 columns: slab GEMMs with < 192 64-column tiles, the c5 Mamba
    in_proj N = 8512) and of 5 waves (80 columns: > 256 tiles, the heads GEMM N = 9234 split 2) keep
    each column's K order: every split's columns equal, bit for bit, those of the 64-column form
    (forced by appending columns until neither grid rule applies)."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights
    M, K = 128, 2048
    g = torch.Generator(device="cpu").manual_seed(7)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    W2 = (torch.randn(N2, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    outs = []
    for n in (N, N2):
        Wpk = pack_weights(W2[:n].contiguous(), stream_ptr())
        part = torch.empty(nsplit, M, n, device=DEV)
        call("zk_gemm_bf16", ptr(A), K, ptr(Wpk), M, n, K, nsplit, 0, ptr(part), None, None, stream_ptr())
        outs.append(part[:, :, :N])
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K", [(16400, 4096, 1024), (8300, 2112, 512), (9000, 8256, 512)])
def test_prefill_gemm_epilogues_consistent(M, N, K):
    """k_gemm_pf's LDS-staged epilogues (whole-row stores, round 5): the SwiGLU output of mode 1 is
    the SwiGLU of mode 0's fp32 output over the same interleaved weights (both modes accumulate in one
    K order), computed here with torch: equal except where expf and torch.exp round the silu
    differently (<= 1 bf16 ulp of the product on a few elements); mode 0 against an fp32 reference.
    N = 8256: mode 1 on 256 x 384 tiles (N >= 8192, partial last column tile), mode 0 on 256 x 256."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights
    g = torch.Generator(device="cpu").manual_seed(M)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    s = stream_ptr()
    Wp = torch.empty_like(W)
    call("zk_permute_fc1", ptr(W), N // 2, K, ptr(Wp), s)
    Wpk = pack_weights(Wp, s)
    C = torch.empty(M, N, device=DEV)
    call("zk_gemm_bf16", ptr(A), K, ptr(Wpk), M, N, K, 1, 0, ptr(C), None, None, s)
    ref = A.float() @ Wp.float().t()
    assert torch.allclose(C, ref, atol=2e-3 * (K / 2048) ** 0.5, rtol=1e-3), (C - ref).abs().max()
    h = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
    call("zk_gemm_bf16", ptr(A), K, ptr(Wpk), M, N, K, 1, 1, None, ptr(h), None, s)
    Cq = C.view(M, N // 16, 2, 8)
    y, gt = Cq[:, :, 0].bfloat16().float(), Cq[:, :, 1].bfloat16().float()
    sl = (gt / (1.0 + torch.exp(-gt))).bfloat16().float()
    exp = (y * sl).bfloat16().reshape(M, N // 2)
    d = (h.float() - exp.float()).abs()
    ulp = exp.float().abs().clamp_min(1e-30) * 2 ** -7
    assert bool((d <= ulp * 1.01).all()), float((d / ulp).max())
    assert float((d > 0).float().mean()) < 1e-3


def test_pack_weights_layout():
    """Fragment-packed layout: block (nt, kc) lane l holds W[16nt + l%16][32kc + 8(l//16) .. +8]."""
    from zonos_amd._lib import stream_ptr
    from zonos_amd.engine import pack_weights
    N, K = 100, 128
    W = torch.arange(N * K, dtype=torch.float32).reshape(N, K).to(torch.bfloat16).to(DEV)
    P = pack_weights(W, stream_ptr()).cpu().reshape(-1, K // 32, 64, 8)
    assert P.shape[0] == 128 // 16
    Wc = W.cpu()
    for nt in range(P.shape[0]):
        for kc in range(K // 32):
            for lane in (0, 5, 17, 63):
                n, k = nt * 16 + lane % 16, kc * 32 + 8 * (lane // 16)
                exp = Wc[n, k:k + 8] if n < N else torch.zeros(8, dtype=torch.bfloat16)
                assert torch.equal(P[nt, kc, lane], exp)


@pytest.mark.parametrize("M,Fd,D", [(130, 256, 512), (2, 256, 512), (40, 256, 512), (128, 512, 2048),
                                    (3, 512, 2048), (1030, 256, 512), (8200, 4096, 1024)])
def test_gemm_swiglu(M, Fd, D):
    from zonos_amd._lib import call, ptr, stream_ptr
    g = torch.Generator(device="cpu").manual_seed(1)
    A = torch.randn(M, D, generator=g).to(torch.bfloat16)
    W1 = (torch.randn(2 * Fd, D, generator=g) / D ** 0.5).to(torch.bfloat16)
    if M * Fd * D < 2 ** 30:
        ref_y, ref_g = F.linear(A, W1).chunk(2, dim=-1)      # bf16 CPU like the reference
    else:                                                     # (the k_gemm_pf size: fp32 GEMM on the GPU, bf16-rounded)
        ref_y, ref_g = (A.to(DEV).float() @ W1.to(DEV).float().t()).bfloat16().cpu().chunk(2, dim=-1)
    ref = ref_y * F.silu(ref_g)
    Wp = torch.empty_like(W1).to(DEV)
    s = stream_ptr()
    call("zk_permute_fc1", ptr(W1.to(DEV)), Fd, D, ptr(Wp), s)
    from zonos_amd.engine import pack_weights
    Wp = pack_weights(Wp, s)
    A_d = A.to(DEV)
    out = torch.empty(M, Fd, dtype=torch.bfloat16, device=DEV)
    call("zk_gemm_bf16", ptr(A_d), D, ptr(Wp), M, 2 * Fd, D, 1, 1, None, ptr(out), None, s)
    err = (out.float().cpu() - ref.float()).abs()
    # one bf16 ulp of the product (|h| < 4 here) plus accumulation-order flips of y/gate
    assert err.max() < 0.05 and (err > 0).float().mean() < 0.05, err.max()


def test_layernorm_and_resid_ln():
    from zonos_amd._lib import call, ptr, stream_ptr
    for D in (256, 2048):
        rows = 33
        g = torch.Generator(device="cpu").manual_seed(D)
        x = torch.randn(rows, D, generator=g).to(torch.bfloat16)
        w = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
        b = (0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
        part = torch.randn(3, rows, D, generator=g)
        ref_ln = F.layer_norm(x, (D,), w, b, 1e-5)
        y = torch.empty(rows, D, dtype=torch.bfloat16, device=DEV)
        xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
        s = stream_ptr()
        call("zk_layernorm", ptr(xd), ptr(wd), ptr(bd), 1e-5, rows, D, ptr(y), s)
        assert (y.float().cpu() - ref_ln.float()).abs().max() < 0.04   # ~1 bf16 ulp at |y|<5
        ref_x = x + part.sum(0).to(torch.bfloat16)
        ref_xn = F.layer_norm(ref_x, (D,), w, b, 1e-5)
        xo = torch.empty_like(xd)
        xn = torch.empty_like(xd)
        pd = part.to(DEV)
        call("zk_resid_ln", ptr(pd), 3, ptr(xd), ptr(wd), ptr(bd), 1e-5, rows, D, ptr(xo), ptr(xn), 0, None, s)
        assert (xo.float().cpu() - ref_x.float()).abs().max() < 0.07
        assert (xn.float().cpu() - ref_xn.float()).abs().max() < 0.06
        # ln_on_sum (mamba_ssm layer_norm_fn prenorm): LN of the fp32 sum, residual stored bf16
        xo2, xn2 = torch.empty_like(xd), torch.empty_like(xd)
        call("zk_resid_ln", ptr(pd), 3, ptr(xd), ptr(wd), ptr(bd), 1e-5, rows, D, ptr(xo2), ptr(xn2), 1, None, s)
        ssum = x.float() + part.sum(0).to(torch.bfloat16).float()
        ref_xn2 = F.layer_norm(ssum, (D,), w.float(), b.float(), 1e-5)
        assert torch.equal(xo2.cpu(), xo.cpu())
        assert (xn2.float().cpu() - ref_xn2).abs().max() < 0.06


def _attn_setup(R, S_ctx, H, Hk, hd, smax, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    k = torch.randn(R, S_ctx, Hk, hd, generator=g).to(torch.bfloat16)
    v = torch.randn(R, S_ctx, Hk, hd, generator=g).to(torch.bfloat16)
    from zonos_amd.kvlayout import pack_k, pack_v
    kf = torch.zeros(R, Hk, smax, hd, dtype=torch.bfloat16)
    vf = torch.zeros(R, Hk, smax, hd, dtype=torch.bfloat16)
    kf[:, :, :S_ctx] = k.transpose(1, 2)
    vf[:, :, :S_ctx] = v.transpose(1, 2)
    return k, v, pack_k(kf), pack_v(vf)


@pytest.mark.parametrize("R,ctx,H,Hk,nsplit", [(4, 1, 16, 4, 1), (3, 300, 16, 4, 2), (2, 1000, 2, 1, 8),
                                                (128, 513, 16, 4, 1), (128, 1705, 16, 4, 2), (1, 2999, 16, 4, 24),
                                                (2, 129, 16, 4, 2)])
def test_attention_decode(R, ctx, H, Hk, nsplit):
    from zonos_amd._lib import call, ptr, stream_ptr
    hd = 128
    smax = ((ctx + 255) // 256) * 256
    k, v, kc, vt = _attn_setup(R, ctx, H, Hk, hd, smax)
    q = torch.randn(R, 1, H, hd).to(torch.bfloat16)
    ref = F.scaled_dot_product_attention(q.transpose(1, 2).float(), k.transpose(1, 2).float(),
                                         v.transpose(1, 2).float(), enable_gqa=True).transpose(1, 2).reshape(R, H * hd)
    nsplit = min(nsplit, smax // 128)
    work = torch.empty(R * Hk * nsplit * (8 + 4 * hd), device=DEV)
    out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    qd, kd, vd = q.to(DEV), kc.to(DEV), vt.to(DEV)
    call("zk_attn_decode", ptr(qd), ptr(kd), ptr(vd), R, H, Hk, hd, smax, ctx, None, ptr(work), nsplit, ptr(out),
         None, stream_ptr())
    # P is rounded to bf16 for the P.V MFMA (as the reference's CPU flash kernel does)
    assert (out.float().cpu() - ref).abs().max() < 2e-2


@pytest.mark.parametrize("R,ctx,H,Hk,nsplit,gs,neox", [(4, 1, 16, 4, 1, 4, 0), (6, 37, 2, 1, 2, 2, 0),
                                                        (128, 300, 16, 4, 1, 4, 0), (3, 700, 16, 4, 4, 8, 0),
                                                        (2, 129, 2, 1, 1, 1, 0), (5, 256, 16, 4, 2, 3, 0),
                                                        (6, 300, 16, 4, 2, 4, 1), (128, 77, 16, 4, 1, 4, 1)])
def test_attention_decode_fused_qkv_equals_separate(R, ctx, H, Hk, nsplit, gs, neox):
    """zk_attn_decode_qkv == zk_qkv_rope (at pos = ctx-1) + zk_attn_decode: bit-identical
    output and identical cache contents afterwards."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import rope_table
    hd = 128
    smax = ((ctx + 255) // 256) * 256
    nsplit = min(nsplit, smax // 128)
    g = torch.Generator(device="cpu").manual_seed(R * 1000 + ctx)
    N = (H + 2 * Hk) * hd
    part = (torch.randn(gs, R, N, generator=g) * 0.5).to(DEV)
    kc0 = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    vt0 = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    freqs = rope_table(16384, hd).to(DEV)
    s = stream_ptr()
    work = torch.empty(R * Hk * nsplit * (8 + 4 * hd), device=DEV)
    # separate kernels
    kc1, vt1 = kc0.clone(), vt0.clone()
    q = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    out1 = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    call("zk_qkv_rope", ptr(part), gs, R, 1, H, Hk, hd, ptr(freqs), ctx - 1, None, ptr(q), ptr(kc1), ptr(vt1), smax,
         None, neox, None, s)
    call("zk_attn_decode", ptr(q), ptr(kc1), ptr(vt1), R, H, Hk, hd, smax, ctx, None, ptr(work), nsplit, ptr(out1),
         None, s)
    # fused
    kc2, vt2 = kc0.clone(), vt0.clone()
    out2 = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    call("zk_attn_decode_qkv", ptr(part), gs, ptr(freqs), ptr(kc2), ptr(vt2), R, H, Hk, hd, smax, ctx, None,
         ptr(work), nsplit, ptr(out2), neox, None, s)
    torch.cuda.synchronize()
    assert torch.equal(kc1, kc2) and torch.equal(vt1, vt2)
    assert torch.equal(out1, out2), (out1.float() - out2.float()).abs().max()


@pytest.mark.parametrize("R,S,H,Hk", [(2, 1, 2, 1), (3, 70, 16, 4), (2, 200, 2, 1), (2, 411, 16, 4)])
def test_attention_prefill(R, S, H, Hk):
    from zonos_amd._lib import call, ptr, stream_ptr
    hd = 128
    smax = ((S + 255) // 256) * 256
    k, v, kc, vt = _attn_setup(R, S, H, Hk, hd, smax, seed=3)
    q = torch.randn(R, S, H, hd, generator=torch.Generator().manual_seed(4)).to(torch.bfloat16)
    ref = F.scaled_dot_product_attention(q.transpose(1, 2).float(), k.transpose(1, 2).float(),
                                         v.transpose(1, 2).float(), is_causal=S > 1, enable_gqa=True)
    ref = ref.transpose(1, 2).reshape(R * S, H * hd)
    out = torch.empty(R * S, H * hd, dtype=torch.bfloat16, device=DEV)
    qd, kd, vd = q.reshape(R * S, H * hd).to(DEV), kc.to(DEV), vt.to(DEV)
    call("zk_attn_prefill", ptr(qd), ptr(kd), ptr(vd), R, S, H, Hk, hd, smax, ptr(out), stream_ptr())
    # P is rounded to bf16 before P.V (as the reference's CPU flash kernel does) and the output is
    # bf16: vs an fp32 SDPA that is up to ~1 bf16 ulp of |out| <= ~2 per element, mean far below.
    err = (out.float().cpu() - ref).abs()
    assert err.max() < 2e-2 and err.mean() < 2e-3, (err.max(), err.mean())


def test_qkv_rope_matches_oracle():
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import rope_table
    R, S, H, Hk, hd, smax = 2, 5, 2, 1, 128, 256
    N = (H + 2 * Hk) * hd
    g = torch.Generator(device="cpu").manual_seed(7)
    part = torch.randn(2, R * S, N, generator=g)
    qkv = part.sum(0).to(torch.bfloat16).view(R, S, N)
    fr = rope_table(16384, hd)
    pos0 = 11
    fc = fr[torch.arange(S)[None, :] + pos0].expand(R, -1, -1, -1)
    qr, kr, vr = qkv.split([H * hd, Hk * hd, Hk * hd], dim=-1)
    q_ref = zonos_ref.rope(qr.reshape(R, S, H, hd), fc).reshape(R * S, H * hd)
    k_ref = zonos_ref.rope(kr.reshape(R, S, Hk, hd), fc)
    q = torch.empty(R * S, H * hd, dtype=torch.bfloat16, device=DEV)
    kc = torch.zeros(R, Hk, smax * hd, dtype=torch.bfloat16, device=DEV)
    vt = torch.zeros(R, Hk, smax * hd, dtype=torch.bfloat16, device=DEV)
    vrows = torch.zeros(R, Hk, S, hd, dtype=torch.bfloat16, device=DEV)
    pd, fd = part.to(DEV), fr.to(DEV)
    call("zk_qkv_rope", ptr(pd), 2, R, S, H, Hk, hd, ptr(fd), pos0, None, ptr(q), ptr(kc), ptr(vt), smax, ptr(vrows),
         0, None, stream_ptr())
    # slab sums in a different order can flip one bf16 rounding; then RoPE is exact fp32
    assert (q.float().cpu() - q_ref.float()).abs().max() < 0.05
    from zonos_amd.kvlayout import unpack_k, unpack_v
    kk, vv = unpack_k(kc.cpu(), smax), unpack_v(vt.cpu(), smax)
    assert (kk[:, :, pos0:pos0 + S].transpose(1, 2).float() - k_ref.float()).abs().max() < 0.05
    assert torch.equal(vv[:, :, pos0:pos0 + S].transpose(1, 2), vr.reshape(R, S, Hk, hd))
    assert kk[:, :, :pos0].abs().sum() == 0 and vv[:, :, pos0 + S:].abs().sum() == 0
    assert torch.equal(vrows.permute(0, 2, 1, 3).cpu(), vr.reshape(R, S, Hk, hd))


def test_embed_codes():
    from zonos_amd._lib import call, ptr, stream_ptr
    B, S, K, V, D = 3, 4, 9, 1026, 256
    g = torch.Generator(device="cpu").manual_seed(2)
    emb = torch.randn(K, V, D, generator=g).to(torch.bfloat16)
    ids = torch.randint(0, V, (B, K, S), generator=g)
    W = {f"embeddings.{k}.weight": emb[k] for k in range(K)}
    ref = zonos_ref.embed_codes(W, zonos_ref.BackboneCfg(d_model=D), ids).repeat(2, 1, 1)
    out = torch.zeros(2 * B, S + 2, D, dtype=torch.bfloat16, device=DEV)
    idd, ed = ids.to(DEV), emb.to(DEV)
    call("zk_embed_codes", ptr(idd), B, S, K, K * S, S, None, 0, ptr(ed), V, D, 2, ptr(out), S + 2, 2, None, None,
         1e-5, None, None, stream_ptr())
    assert torch.equal(out[:, 2:].cpu(), ref)          # bf16 sequential adds reproduced bit-exactly


@pytest.mark.parametrize("M,N,K,mode,ln", [(2, 3072, 2048, 0, True), (16, 3072, 2048, 0, True), (5, 9234, 2048, 0, True),
                                           (2, 2048, 2048, 2, False), (16, 2048, 8192, 2, False),
                                           (1, 2048, 4096, 2, False), (2, 16384, 2048, 1, True),
                                           (9, 16384, 2048, 1, True), (7, 4000, 2048, 0, False),
                                           (3, 5000, 2048, 0, True), (4, 5000, 8192, 2, False),
                                           # B = 1 (M <= 2): activation staged in LDS per wave (ZK_GF_XC) at
                                           # every K and layout, LayerNorm loads by the normalising waves only
                                           (2, 2048, 8192, 2, False), (1, 4000, 2048, 0, False),
                                           (2, 16384, 4096, 1, False), (2, 9234, 8192, 0, False),
                                           (1, 16384, 2048, 1, True)])
def test_gemv_fused(M, N, K, mode, ln):
    """Small-batch GEMV (zk_gemv_fused): LayerNorm prologue, fp32 / SwiGLU / residual epilogues,
    half-tile, one-tile and two-tile layouts, against torch on the CPU at the same rounding points."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + mode)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(K, generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(K, generator=g)).to(torch.bfloat16)
    s = stream_ptr()
    a = F.layer_norm(x, (K,), w, b, 1e-5) if ln else x          # bf16 LayerNorm (fp32 inside), CPU
    Wd = W.to(DEV)
    if mode == 1:
        Wp = torch.empty_like(Wd)
        call("zk_permute_fc1", ptr(Wd), N // 2, K, ptr(Wp), s)
        Wd = Wp
    Wpk = pack_weights(Wd, s)
    xd = x.to(DEV)
    keep = (w.to(DEV), b.to(DEV))            # LayerNorm weight / bias (held alive for the call)
    lw, lb = (ptr(keep[0]), ptr(keep[1])) if ln else (None, None)
    if mode == 0:
        out = torch.full((M, N), float("nan"), device=DEV)
        call("zk_gemv_fused", ptr(xd), K, ptr(Wpk), M, N, K, 0, lw, lb, 1e-5, ptr(out), None, None, s)
        ref = a.float() @ W.float().t()
        # the LayerNorm'd activation differs by <= 1 bf16 ulp from torch's in a few elements
        assert torch.allclose(out.cpu(), ref, atol=2e-2 if ln else 3e-3, rtol=1e-2), (out.cpu() - ref).abs().max()
    elif mode == 1:
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
        call("zk_gemv_fused", ptr(xd), K, ptr(Wpk), M, N, K, 1, lw, lb, 1e-5, None, ptr(out), None, s)
        ry, rg = F.linear(a, W).chunk(2, dim=-1)
        ref = ry * F.silu(rg)
        err = (out.float().cpu() - ref.float()).abs()
        assert err.max() < 0.06 and (err > 0).float().mean() < 0.06, err.max()
    else:
        res = torch.randn(M, N, generator=g).to(torch.bfloat16)
        xr = res.to(DEV)
        call("zk_gemv_fused", ptr(xd), K, ptr(Wpk), M, N, K, 2, None, None, 1e-5, None, ptr(xr), None, s)
        ref = res + F.linear(x, W)                               # bf16 + bf16(proj), like _torch.py:100-101
        err = (xr.float().cpu() - ref.float()).abs()
        assert err.max() < 0.07 and (err > 0).float().mean() < 0.05, err.max()


@pytest.mark.parametrize("R,ctx,nsplit", [(2, 600, 5), (2, 1000, 8), (16, 300, 3), (4, 129, 2)])
def test_attention_split_combine_in_launch(R, ctx, nsplit):
    """zk_attn_decode_qkv_sc (split partials merged inside the launch by the last workgroup of
    each (row, kv head)) == zk_attn_decode_qkv + k_attn_combine, bit for bit, over repeated
    launches (the ticket counters carry over from launch to launch)."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import rope_table
    H, Hk, hd = 16, 4, 128
    smax = ((ctx + 255) // 256) * 256
    g = torch.Generator(device="cpu").manual_seed(ctx)
    kc = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    vt = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    freqs = rope_table(16384, hd).to(DEV)
    work = torch.empty(R * Hk * nsplit * (8 + 4 * hd), device=DEV)
    cnt = torch.zeros(R * Hk, dtype=torch.int32, device=DEV)
    s = stream_ptr()
    for rep in range(3):
        part = (torch.randn(R * (H + 2 * Hk) * hd, generator=g) * 0.5).to(DEV)
        kc2, vt2 = kc.clone(), vt.clone()
        ref = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
        call("zk_attn_decode_qkv", ptr(part), 1, ptr(freqs), ptr(kc2), ptr(vt2), R, H, Hk, hd, smax, ctx + rep, None,
             ptr(work), nsplit, ptr(ref), 0, None, s)
        out = torch.full((R, H * hd), float("nan"), dtype=torch.bfloat16, device=DEV)
        call("zk_attn_decode_qkv_sc", ptr(part), 1, ptr(freqs), ptr(kc), ptr(vt), R, H, Hk, hd, smax, ctx + rep, None,
             ptr(work), nsplit, ptr(cnt), ptr(out), 0, None, s)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (rep, (out.float() - ref.float()).abs().max())
        assert torch.equal(kc, kc2) and torch.equal(vt, vt2)
    assert bool((cnt.cpu() % nsplit == 0).all()) and int(cnt.cpu()[0]) == 3 * nsplit


@pytest.mark.parametrize("R,ctx,nsplit", [(2, 300, 2), (2, 700, 4), (2, 1000, 8), (1, 129, 2), (2, 161, 8)])
def test_attention_out_proj_merge(R, ctx, nsplit):
    """zk_attn_decode_qkv_part + zk_gemv_attn_out (the split partials merged in the out_proj
    GEMV's prologue) == zk_attn_decode_qkv (+ k_attn_combine) + zk_gemv_fused mode 2, bit for
    bit: the residual stream after out_proj and the KV cache contents."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights, rope_table
    H, Hk, hd, D = 16, 4, 128, 2048
    smax = ((ctx + 255) // 256) * 256
    nsplit = min(nsplit, smax // 128)
    g = torch.Generator(device="cpu").manual_seed(ctx * 7 + nsplit)
    kc = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    vt = torch.randn(R * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    part = (torch.randn(R * (H + 2 * Hk) * hd, generator=g) * 0.5).to(DEV)
    freqs = rope_table(16384, hd).to(DEV)
    s = stream_ptr()
    Wo = pack_weights((torch.randn(D, H * hd, generator=g) * 0.02).to(torch.bfloat16).to(DEV), s)
    x0 = torch.randn(R, D, generator=g).to(torch.bfloat16).to(DEV)
    # reference sequence: attention output (split + combine launch), then out_proj + residual
    kc1, vt1, x1 = kc.clone(), vt.clone(), x0.clone()
    work1 = torch.empty(R * Hk * nsplit * (8 + 4 * hd), device=DEV)
    y = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    call("zk_attn_decode_qkv", ptr(part), 1, ptr(freqs), ptr(kc1), ptr(vt1), R, H, Hk, hd, smax, ctx, None,
         ptr(work1), nsplit, ptr(y), 0, None, s)
    call("zk_gemv_fused", ptr(y), H * hd, ptr(Wo), R, D, H * hd, 2, None, None, 1e-5, None, ptr(x1), None, s)
    # merged in the consumer
    kc2, vt2, x2 = kc.clone(), vt.clone(), x0.clone()
    work2 = torch.full((R * Hk * nsplit * (8 + 4 * hd),), float("nan"), device=DEV)
    call("zk_attn_decode_qkv_part", ptr(part), 1, ptr(freqs), ptr(kc2), ptr(vt2), R, H, Hk, hd, smax, ctx, None,
         ptr(work2), nsplit, 0, None, s)
    call("zk_gemv_attn_out", ptr(work2), nsplit, Hk, ptr(Wo), R, D, H * hd, ptr(x2), None, s)
    torch.cuda.synchronize()
    assert torch.equal(kc1, kc2) and torch.equal(vt1, vt2)
    assert torch.equal(x1.view(torch.int16), x2.view(torch.int16)), (x1.float() - x2.float()).abs().max()
    # and the result is the attention + projection of an fp32 reference within bf16 tolerance
    assert not torch.equal(x1, x0)


@pytest.mark.parametrize("M,pos,smax", [(2, 0, 256), (2, 31, 256), (2, 32, 512), (1, 600, 1280), (2, 1029, 1280),
                                        (2, 5000, 1280)])
def test_gemv_qkv_rope_equals_gemv_and_rope(M, pos, smax):
    """zk_gemv_qkv_rope (the B = 1 in_proj with the RoPE / KV-write epilogue) == zk_gemv_fused mode 0
    with the LayerNorm prologue + zk_qkv_rope at the same position, bit for bit: q and every cache
    byte (a position past the cache is clamped to Smax - 1, as the attention clamps its context)."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights, rope_table
    H, Hk, hd, D = 16, 4, 128, 2048
    N = (H + 2 * Hk) * hd
    g = torch.Generator(device="cpu").manual_seed(pos * 3 + M)
    s = stream_ptr()
    x = torch.randn(M, D, generator=g).to(torch.bfloat16).to(DEV)
    Wpk = pack_weights((torch.randn(N, D, generator=g) / D ** 0.5).to(torch.bfloat16).to(DEV), s)
    lw = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16).to(DEV)
    lb = (0.1 * torch.randn(D, generator=g)).to(torch.bfloat16).to(DEV)
    freqs = rope_table(16384, hd).to(DEV)
    kc0 = torch.randn(M * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    vt0 = torch.randn(M * Hk * smax * hd, generator=g).to(torch.bfloat16).to(DEV)
    p = min(pos, smax - 1)
    part = torch.empty(M, N, device=DEV)
    call("zk_gemv_fused", ptr(x), D, ptr(Wpk), M, N, D, 0, ptr(lw), ptr(lb), 1e-5, ptr(part), None, None, s)
    q1 = torch.empty(M, H * hd, dtype=torch.bfloat16, device=DEV)
    kc1, vt1 = kc0.clone(), vt0.clone()
    call("zk_qkv_rope", ptr(part), 1, M, 1, H, Hk, hd, ptr(freqs), p, None, ptr(q1), ptr(kc1), ptr(vt1), smax, None,
         0, None, s)
    q2 = torch.full((M, H * hd), float("nan"), dtype=torch.bfloat16, device=DEV)
    kc2, vt2 = kc0.clone(), vt0.clone()
    posd = torch.tensor([pos], dtype=torch.int32, device=DEV)
    call("zk_gemv_qkv_rope", ptr(x), ptr(Wpk), M, H, Hk, hd, ptr(lw), ptr(lb), 1e-5, ptr(q2), ptr(kc2), ptr(vt2), smax,
         ptr(posd), ptr(freqs), None, s)
    torch.cuda.synchronize()
    assert torch.equal(q1.view(torch.int16), q2.view(torch.int16))
    assert torch.equal(kc1, kc2) and torch.equal(vt1, vt2)
    assert not torch.equal(kc1, kc0) and not torch.equal(vt1, vt0)
    # skipped (done word set): nothing is written
    done = torch.ones(1, dtype=torch.int32, device=DEV)
    kc3, vt3 = kc0.clone(), vt0.clone()
    q3 = q2.clone()
    call("zk_gemv_qkv_rope", ptr(x), ptr(Wpk), M, H, Hk, hd, ptr(lw), ptr(lb), 1e-5, ptr(q3), ptr(kc3), ptr(vt3), smax,
         ptr(posd), ptr(freqs), ptr(done), s)
    torch.cuda.synchronize()
    assert torch.equal(kc3, kc0) and torch.equal(vt3, vt0) and torch.equal(q3.view(torch.int16), q2.view(torch.int16))


@pytest.mark.parametrize("R,ctx,nsplit", [(2, 1, 8), (2, 31, 4), (2, 33, 8), (2, 600, 4), (2, 600, 8), (1, 1000, 16),
                                          (2, 1030, 16), (2, 257, 2)])
def test_attention_q_part_out_proj_merge(R, ctx, nsplit):
    """zk_attn_decode_q_part (32-key slices interleaved over nsplit workgroups per (row, kv head)) +
    zk_gemv_attn_out == the unsplit zk_attn_decode + zk_gemv_fused mode 2 up to the fp32 summation
    order of the split merge (the residual stream after out_proj within 1 bf16 ulp; measured: up to 6 %
    of its elements one ulp apart),
    and the attention itself against an fp32 SDPA of the same cache."""
    from zonos_amd._lib import call, ptr, stream_ptr
    from zonos_amd.engine import pack_weights
    H, Hk, hd, D = 16, 4, 128, 2048
    smax = ((ctx + 255) // 256) * 256
    k, v, kc, vt = _attn_setup(R, ctx, H, Hk, hd, smax, seed=ctx + nsplit)
    g = torch.Generator(device="cpu").manual_seed(ctx * 5 + nsplit)
    q = torch.randn(R, H * hd, generator=g).to(torch.bfloat16)
    s = stream_ptr()
    Wo = pack_weights((torch.randn(D, H * hd, generator=g) * 0.02).to(torch.bfloat16).to(DEV), s)
    x0 = torch.randn(R, D, generator=g).to(torch.bfloat16).to(DEV)
    qd, kd, vd = q.to(DEV), kc.to(DEV), vt.to(DEV)
    ctxd = torch.tensor([ctx - 1], dtype=torch.int32, device=DEV)       # ctx = ctx0 (1) + *ctx_dev
    y = torch.empty(R, H * hd, dtype=torch.bfloat16, device=DEV)
    call("zk_attn_decode", ptr(qd), ptr(kd), ptr(vd), R, H, Hk, hd, smax, ctx, None, None, 1, ptr(y), None, s)
    x1 = x0.clone()
    call("zk_gemv_fused", ptr(y), H * hd, ptr(Wo), R, D, H * hd, 2, None, None, 1e-5, None, ptr(x1), None, s)
    work = torch.full((R * Hk * nsplit * (8 + 4 * hd),), float("nan"), device=DEV)
    call("zk_attn_decode_q_part", ptr(qd), ptr(kd), ptr(vd), R, H, Hk, hd, smax, 1, ptr(ctxd), ptr(work), nsplit,
         None, s)
    x2 = x0.clone()
    call("zk_gemv_attn_out", ptr(work), nsplit, Hk, ptr(Wo), R, D, H * hd, ptr(x2), None, s)
    torch.cuda.synchronize()
    assert torch.isfinite(x2.float()).all()
    err = (x2.float() - x1.float()).abs()
    assert err.max() < 0.07 and (err > 0).float().mean() < 0.15, (err.max(), (err > 0).float().mean())
    # the merged attention itself (from the partials) vs an fp32 SDPA
    wk = work.view(R, Hk, nsplit, 8 + 4 * hd).cpu()
    m, l, o = wk[..., :4], wk[..., 4:8], wk[..., 8:].view(R, Hk, nsplit, 4, hd)
    M_ = m.max(dim=2, keepdim=True).values
    c = torch.where(m == -float("inf"), torch.zeros_like(m), torch.exp(m - M_))
    att = (o * c[..., None]).sum(2) / (l * c).sum(2)[..., None]
    ref = F.scaled_dot_product_attention(q.view(R, 1, H, hd).transpose(1, 2).float(), k.transpose(1, 2).float(),
                                         v.transpose(1, 2).float(), enable_gqa=True).view(R, Hk, 4, hd)
    assert (att - ref).abs().max() < 2e-2
