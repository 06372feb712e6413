"""Per-kernel timing at the decode-step shapes of Zonos-v0.1 (B=64 -> 128 rows), HIP events.
    python tools/microbench.py [gemm|attn|dac|all]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib  # noqa: E402
from zonos_amd._lib import call, ptr  # noqa: E402
from zonos_amd.engine import _split_for  # noqa: E402

_lib.load()
dev = torch.device("cuda")
S = _lib.stream_ptr()


def timeit(fn, reps=50, warm=5):
    e0, e1 = _lib.P(), _lib.P()
    call("zk_event_create", C.byref(e0))
    call("zk_event_create", C.byref(e1))
    for _ in range(warm):
        fn()
    call("zk_event_record", e0.value, S)
    for _ in range(reps):
        fn()
    call("zk_event_record", e1.value, S)
    ms = C.c_float()
    call("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
    return ms.value / reps * 1e3   # us


def gemm():
    M = int(os.environ.get("ZK_MB_M", "128"))
    shapes = [("qkv", 3072, 2048, 0), ("o", 2048, 2048, 0), ("fc1", 16384, 2048, 1),
              ("fc2", 2048, 8192, 0), ("heads", 9234, 2048, 0)]
    # extra shapes "name:N:K:mode,..." (e.g. fc1 as a split-K slab GEMM: "fc1s:16384:2048:0")
    shapes += [(t[0], int(t[1]), int(t[2]), int(t[3])) for t in
               (x.split(":") for x in os.environ.get("ZK_MB_GEMM_EXTRA", "").split(",") if x)]
    for name, N, K, mode in shapes:
        # distinct weight buffers per rep set so L2/MALL does not serve them: rotate 8 copies (>256 MB total)
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        Npad = (N + 63) // 64 * 64        # packed layout reads whole 64-row tiles
        Ws = [torch.randn(Npad, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]   # packed-size buffers
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ns = 1 if mode == 1 else _split_for(N, K, M, int(os.environ.get("ZK_SPLIT_TARGET", "256")))
        ovr = dict(kv.split("=") for kv in os.environ.get("ZK_SPLITS", "").split(",") if kv)
        ns = int(ovr.get(name, ns))
        part = torch.empty(ns * M * N, device=dev)
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
        it = [0]

        def f():
            W = Ws[it[0] % ncopy]
            it[0] += 1
            call("zk_gemm_bf16", ptr(A), K, ptr(W), M, N, K, ns, mode, ptr(part), ptr(out), None, S)
        us = timeit(f)
        gb = N * K * 2 / 1e9
        print(f"gemm {name:6s} N={N:5d} K={K:5d} split={ns:2d}: {us:8.1f} us  weights {gb*1e3:6.1f} MB  "
              f"{gb / (us * 1e-6):7.0f} GB/s", flush=True)
        del Ws


def sweep():
    """Fixed cost vs streamed bytes of the decode GEMM family: k_gemm_ws (M = 128, split 4) and the
    B <= 8 GEMV (M = 2, split 1) at N = 2048 / 8192 over K = 512 .. 8192; fit t = t0 + bytes / rate."""
    import numpy as np
    for M, ns in ((128, 4), (2, 1)):
        for N in (2048, 8192):
            pts = []
            for K in (512, 1024, 2048, 4096, 8192):
                if M > 16 and K // ns // 64 > 32:
                    continue
                if M <= 16 and K > 2048:        # (the B <= 8 step runs K > 2048 through zk_gemv_fused)
                    continue
                ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
                Ws = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
                A = torch.randn(M, K, device=dev).to(torch.bfloat16)
                part = torch.empty(ns * M * N, device=dev)
                it = [0]

                def f():
                    W = Ws[it[0] % ncopy]
                    it[0] += 1
                    call("zk_gemm_bf16", ptr(A), K, ptr(W), M, N, K, ns, 0, ptr(part), None, None, S)
                us = timeit(f)
                pts.append((N * K * 2, us))
                print(f"sweep M={M:3d} N={N:5d} K={K:5d} split={ns}: {us:7.2f} us  {N * K * 2 / 1e6:6.1f} MB  "
                      f"{N * K * 2 / (us * 1e-6) / 1e9:6.0f} GB/s", flush=True)
                del Ws
            x = np.array([p[0] for p in pts], dtype=float)
            y = np.array([p[1] for p in pts])
            b, a = np.polyfit(x, y, 1)
            print(f"fit   M={M:3d} N={N:5d}: fixed {a:5.2f} us + bytes at {1e-6 / b:5.2f} TB/s", flush=True)


def warm():
    """Experiment: k_gemm_ws launches whose first weight chunks were just read into L2 by a small
    preceding kernel (zk_l2_warm_gemm) vs cold; time(pair) - time(warm kernel alone) vs time(cold)."""
    M = 128
    lib = _lib.load()
    lib.zk_l2_warm_gemm.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    for name, N, K, mode, ns in (("qkv", 3072, 2048, 0, 4), ("o", 2048, 2048, 0, 4), ("fc1", 16384, 2048, 1, 1),
                                 ("fc2", 2048, 8192, 0, 8)):
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        Npad = (N + 63) // 64 * 64
        Ws = [torch.randn(Npad, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        part = torch.empty(ns * M * N, device=dev)
        out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)
        for chunks in (2, 4):
            for nwg in (128, 256):
                it = [0]

                def g():
                    W = Ws[it[0] % ncopy]; it[0] += 1
                    call("zk_gemm_bf16", ptr(A), K, ptr(W), M, N, K, ns, mode, ptr(part), ptr(out), None, S)

                def wg():
                    W = Ws[it[0] % ncopy]; it[0] += 1
                    rc = lib.zk_l2_warm_gemm(ptr(W), N, K, ns, chunks, nwg, ptr(sink), S)
                    assert rc == 0

                def pair():
                    W = Ws[it[0] % ncopy]; it[0] += 1
                    rc = lib.zk_l2_warm_gemm(ptr(W), N, K, ns, chunks, nwg, ptr(sink), S)
                    assert rc == 0
                    call("zk_gemm_bf16", ptr(A), K, ptr(W), M, N, K, ns, mode, ptr(part), ptr(out), None, S)
                tc, tw, tp = timeit(g), timeit(wg), timeit(pair)
                print(f"warm {name:4s} split={ns} chunks={chunks} nwg={nwg}: cold {tc:6.2f} us, warm kernel {tw:5.2f}, "
                      f"pair {tp:6.2f} -> gemm after warm-up {tp - tw:6.2f} us", flush=True)
        del Ws


def prefill():
    """Prefill GEMMs at c3 (M = 2B x (Lc + P + 1) = 128 x 411 rows, split-K 1)."""
    M = 128 * 411
    for name, N, K, mode in (("qkv", 3072, 2048, 0), ("o", 2048, 2048, 0), ("fc1", 16384, 2048, 1),
                             ("fc2", 2048, 8192, 0)):
        Wp = torch.randn((N + 63) // 64 * 64, K, device=dev).to(torch.bfloat16)
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        part = torch.empty(M * N if mode == 0 else 1, device=dev)
        out = torch.empty(M, N // 2 if mode == 1 else 1, dtype=torch.bfloat16, device=dev)

        def f():
            call("zk_gemm_bf16", ptr(A), K, ptr(Wp), M, N, K, 1, mode, ptr(part), ptr(out), None, S)
        us = timeit(f, reps=10, warm=2)
        print(f"prefill {name:4s} M={M} N={N:5d} K={K:5d}: {us / 1e3:7.3f} ms  "
              f"{2.0 * M * N * K / (us * 1e-6) / 1e12:7.1f} TFLOP/s", flush=True)
        del Wp, A, part, out


def ln():
    R, D = 128, 2048
    for ns in (1, 4, 8):
        ncopy = 16
        parts = [torch.randn(ns * R * D, device=dev) for _ in range(ncopy)]
        x = torch.randn(R, D, device=dev).to(torch.bfloat16)
        w = torch.randn(D, device=dev).to(torch.bfloat16)
        b = torch.randn(D, device=dev).to(torch.bfloat16)
        xn = torch.empty_like(x)
        it = [0]

        def f():
            p = parts[it[0] % ncopy]
            it[0] += 1
            call("zk_resid_ln", ptr(p), ns, ptr(x), ptr(w), ptr(b), 1e-5, R, D, ptr(x), ptr(xn), 0, None, S)
        print(f"resid_ln rows={R} D={D} slabs={ns}: {timeit(f):6.2f} us", flush=True)


def attn():
    R, H, Hk, hd = 128, 16, 4, 128
    for ctx in (512, 1705, 2999):
        smax = ((ctx + 255) // 256) * 256
        ncopy = 3
        kcs = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        vts = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        q = torch.randn(R, H * hd, device=dev).to(torch.bfloat16)
        from zonos_amd.engine import attn_splits_for, rope_table
        for ms_ in sorted({attn_splits_for(R, Hk, smax), 1}):
            attn_one(R, H, Hk, hd, ctx, smax, kcs, vts, q, ms_, ncopy)
        # fused in_proj epilogue (the product path)
        gs = 4
        part = torch.randn(gs * R * (H + 2 * Hk) * hd, device=dev) * 0.1
        freqs = rope_table(16384, hd).to(dev)
        work = torch.empty(R * Hk * (8 + 4 * hd), device=dev)
        out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
        it = [0]

        def fq():
            i = it[0] % ncopy
            it[0] += 1
            call("zk_attn_decode_qkv", ptr(part), gs, ptr(freqs), ptr(kcs[i]), ptr(vts[i]), R, H, Hk, hd, smax, ctx,
                 None, ptr(work), 1, ptr(out), 0, None, S)
        us = timeit(fq)
        b = R * ctx * Hk * hd * 2 * 2 + gs * R * (H + 2 * Hk) * hd * 4
        print(f"attn+qkv ctx={ctx:5d} fused: {us:8.1f} us  {b/1e6:7.1f} MB  {b / (us * 1e-6) / 1e9:7.0f} GB/s",
              flush=True)
        qkv_out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)

        def fr():
            call("zk_qkv_rope", ptr(part), gs, R, 1, H, Hk, hd, ptr(freqs), ctx - 1, None, ptr(qkv_out), ptr(kcs[0]),
                 ptr(vts[0]), smax, None, 0, None, S)
        us = timeit(fr)
        print(f"qkv_rope alone ctx={ctx:5d}: {us:8.1f} us", flush=True)


def attn_small():
    """B = 1 decode attention (R = 2 rows) with the fused in_proj epilogue: one workgroup per
    (row, kv head) vs key splits merged by k_attn_combine (second launch) or in the launch
    (zk_attn_decode_qkv_sc). 26 rotating caches, as the 26 layers of a step."""
    from zonos_amd.engine import rope_table
    R, H, Hk, hd = int(os.environ.get("ZK_MB_R", "2")), 16, 4, 128
    smax = 1280
    nl = 26
    kcs = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(nl)]
    vts = [torch.randn(R * Hk * smax * hd, device=dev).to(torch.bfloat16) for _ in range(nl)]
    part = torch.randn(R * (H + 2 * Hk) * hd, device=dev) * 0.1
    freqs = rope_table(16384, hd).to(dev)
    out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
    cnt = torch.zeros(R * Hk, dtype=torch.int32, device=dev)
    q = torch.randn(R, H * hd, device=dev).to(torch.bfloat16)
    for ctx in (1, 300, 600):
        it = [0]

        def fu():
            i = it[0] % nl
            it[0] += 1
            call("zk_attn_decode", ptr(q), ptr(kcs[i]), ptr(vts[i]), R, H, Hk, hd, smax, ctx, None, None, 1, ptr(out),
                 None, S)
        print(f"attn R={R} ctx={ctx:5d} unfused (q given), unsplit: {timeit(fu, reps=104, warm=26):6.2f} us", flush=True)

        def fr():
            call("zk_qkv_rope", ptr(part), 1, R, 1, H, Hk, hd, ptr(freqs), ctx - 1, None, ptr(q), ptr(kcs[0]),
                 ptr(vts[0]), smax, None, 0, None, S)
        print(f"qkv_rope alone R={R}: {timeit(fr, reps=104, warm=26):6.2f} us", flush=True)
    for ctx in (ENV_CTX if (ENV_CTX := [int(c) for c in os.environ.get("ZK_MB_CTX", "").split(",") if c]) else
                (1, 300, 600, 1000)):
        for ns in (1, 2, 4, 8):
            work = torch.empty(R * Hk * ns * (8 + 4 * hd), device=dev)
            for sc in ((False, True) if ns > 1 else (False,)):
                it = [0]

                def f():
                    i = it[0] % nl
                    it[0] += 1
                    if sc:
                        call("zk_attn_decode_qkv_sc", ptr(part), 1, ptr(freqs), ptr(kcs[i]), ptr(vts[i]), R, H, Hk,
                             hd, smax, ctx, None, ptr(work), ns, ptr(cnt), ptr(out), 0, None, S)
                    else:
                        call("zk_attn_decode_qkv", ptr(part), 1, ptr(freqs), ptr(kcs[i]), ptr(vts[i]), R, H, Hk, hd,
                             smax, ctx, None, ptr(work), ns, ptr(out), 0, None, S)
                us = timeit(f, reps=104, warm=26)
                print(f"attn R={R} ctx={ctx:5d} splits={ns:2d} {'in-launch combine' if sc else 'combine launch  ' if ns > 1 else 'unsplit         '}: {us:6.2f} us", flush=True)


def mamba():
    """Hybrid decode SSM update (zk_mamba_step) at c5 shapes: R=128 rows, 64 heads x 64 x 128 state,
    in_proj unsplit (as the engine runs it at c5), rotating over 8 layers' states (1.1 GB: nothing stays in the MALL)."""
    R, hp, ds, nh, gs = 128, 64, 128, 64, 1
    di = nh * hp
    conv_dim = di + 2 * ds
    ncol = 2 * di + 2 * ds + nh
    nl = 8
    parts = torch.randn(gs, R, ncol, device=dev) * 0.5
    cw = torch.randn(conv_dim, 4, device=dev) * 0.3
    cb = torch.randn(conv_dim, device=dev) * 0.1
    convs = [(torch.randn(R, conv_dim, 4, device=dev).to(torch.bfloat16),
              torch.randn(R, conv_dim, 4, device=dev).to(torch.bfloat16)) for _ in range(nl)]
    # double-buffered state (as the engine runs it)
    ssms = [(0.5 * torch.randn(2, R, nh, hp, ds, device=dev)).to(torch.bfloat16) for _ in range(nl)]
    A = -torch.rand(nh, device=dev) * 4
    dtb = torch.randn(nh, device=dev) * 0.5
    Dv = torch.randn(nh, device=dev)
    posd = torch.tensor([3], dtype=torch.int32, device=dev)
    yz = torch.empty(R, di, device=dev)
    it = [0]

    def f():
        i = it[0] % nl
        it[0] += 1
        call("zk_mamba_step", ptr(parts), gs, R, di, nh, hp, ds, ptr(cw), ptr(cb), ptr(convs[i][0]), ptr(convs[i][1]),
             ptr(posd), ptr(ssms[i][0]), ptr(ssms[i][1]), ptr(A), ptr(dtb), ptr(Dv), ptr(yz), None, S)
    us = timeit(f, reps=40, warm=8)
    b = R * di * ds * 2 * 2 + R * conv_dim * 8 * 2 + gs * R * ncol * 4 + R * di * 4
    print(f"mamba_step R={R}: {us:7.2f} us  "
          f"{b / 1e6:6.1f} MB  {b / (us * 1e-6) / 1e9:6.0f} GB/s", flush=True)


def attn_one(R, H, Hk, hd, ctx, smax, kcs, vts, q, ms_, ncopy):
    if True:
        work = torch.empty(R * Hk * ms_ * (8 + 4 * hd), device=dev)
        out = torch.empty(R, H * hd, dtype=torch.bfloat16, device=dev)
        it = [0]

        def f():
            i = it[0] % ncopy
            it[0] += 1
            call("zk_attn_decode", ptr(q), ptr(kcs[i]), ptr(vts[i]), R, H, Hk, hd, smax, ctx, None, ptr(work), ms_,
                 ptr(out), None, S)
        us = timeit(f)
        b = R * ctx * Hk * hd * 2 * 2
        print(f"attn ctx={ctx:5d} splits={ms_}: {us:8.1f} us  {b/1e6:7.1f} MB  {b / (us * 1e-6) / 1e9:7.0f} GB/s", flush=True)


def gemv():
    """Small-batch (M <= 16) decode projections: zk_gemv_fused (LN prologue / residual epilogue)
    vs the split-K zk_gemm_bf16 + zk_resid_ln pair it replaces. Rotating weight copies."""
    M = int(os.environ.get("ZK_MB_M", "2"))
    D = 2048
    x = torch.randn(M, 8192, device=dev).to(torch.bfloat16)
    lw = torch.ones(D, device=dev, dtype=torch.bfloat16)
    lb = torch.zeros(D, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, D, device=dev).to(torch.bfloat16)
    outf = torch.empty(M * 16384, device=dev)
    outb = torch.empty(M * 16384, device=dev, dtype=torch.bfloat16)
    part = torch.empty(16 * M * 16384, device=dev)
    xo, xn = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    tot_new = tot_old = 0.0
    shapes = (("qkv", 3072, 2048, 0, True), ("o", 2048, 2048, 2, False), ("fc1", 16384, 2048, 1, True),
              ("fc2", 2048, 8192, 2, False), ("heads", 9234, 2048, 0, True))
    if os.environ.get("ZK_MB_SHAPES"):      # "name:N:K:mode:ln,..." (extra tuning shapes)
        shapes = [(a, int(b), int(c), int(d), e == "1") for a, b, c, d, e in
                  (t.split(":") for t in os.environ["ZK_MB_SHAPES"].split(","))]
    for name, N, K, mode, ln in shapes:
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        Npad = (N + 63) // 64 * 64
        Ws = [torch.randn(Npad, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def f():
            W = Ws[it[0] % ncopy]
            it[0] += 1
            call("zk_gemv_fused", ptr(x), K, ptr(W), M, N, K, mode, ptr(lw) if ln else None, ptr(lb) if ln else None,
                 1e-5, ptr(outf), ptr(res) if mode == 2 else ptr(outb), None, S)
        us = timeit(f)
        # the replaced pair: split-K GEMV (+ the k_resid_ln of a residual / LayerNorm edge)
        gm = 1 if mode == 1 else _split_for(N, K, 2 * 8, 256 if name != "o" else 128)
        gm = 1 if name == "heads" else gm

        def g():
            W = Ws[it[0] % ncopy]
            it[0] += 1
            call("zk_gemm_bf16", ptr(x), K, ptr(W), M, N, K, gm, mode if mode < 2 else 0, ptr(part), ptr(outb),
                 None, S)
            if mode == 2 or name == "fc1":
                call("zk_resid_ln", ptr(part), gm, ptr(res), ptr(lw), ptr(lb), 1e-5, M, D, ptr(xo), ptr(xn), 0,
                     None, S)
        us_old = timeit(g)
        tot_new += us
        tot_old += us_old
        gb = N * K * 2 / 1e9
        print(f"gemv {name:6s} M={M} N={N:5d} K={K:5d}: fused {us:6.2f} us ({gb / (us * 1e-6):5.0f} GB/s)   "
              f"split-K(+resid_ln) {us_old:6.2f} us", flush=True)
        del Ws
    print(f"gemv total per layer-ish: fused {tot_new:.1f} us, old {tot_old:.1f} us", flush=True)


def gemv_warm():
    """Experiment: B = 1 GEMV launches (zk_gemv_fused at M = 2, the c2 layouts) whose first weight
    loads per wave were just pre-read into L2 by zk_gemv_warm (same grid and addresses) vs cold; the
    GEMV after the warm-up = time(pair) - time(warm alone). Rotating weight copies (> MALL)."""
    lib = _lib.load()
    lib.zk_gemv_warm.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    M, D = 2, 2048
    x = torch.randn(M, 8192, device=dev).to(torch.bfloat16)
    lw = torch.ones(D, device=dev, dtype=torch.bfloat16)
    lb = torch.zeros(D, device=dev, dtype=torch.bfloat16)
    outf = torch.empty(M * 16384, device=dev)
    outb = torch.empty(M * 16384, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, D, device=dev).to(torch.bfloat16)
    # name, N, K, mode, LN, layout (zk_gemv_fused: lay 0 half tiles / 1 one tile / 2 two tiles), loads per wave
    for name, N, K, mode, ln, lay, nl in (("qkv", 3072, 2048, 0, True, 1, 16), ("o", 2048, 2048, 2, False, 0, 4),
                                          ("fc1", 16384, 2048, 1, True, 2, 16), ("fc2", 2048, 8192, 2, False, 0, 16)):
        ncopy = max(2, int(600e6 // (N * K * 2)) + 1)
        Npad = (N + 63) // 64 * 64
        Ws = [torch.randn(Npad, K, device=dev).to(torch.bfloat16) for _ in range(ncopy)]
        it = [0]

        def g():
            W = Ws[it[0] % ncopy]; it[0] += 1
            call("zk_gemv_fused", ptr(x), K, ptr(W), M, N, K, mode, ptr(lw) if ln else None, ptr(lb) if ln else None,
                 1e-5, ptr(outf), ptr(res) if mode == 2 else ptr(outb), None, S)
        tc = timeit(g)
        for steps in sorted({2, 4, 8, nl}):
            if steps > nl:
                continue

            def wg():
                W = Ws[it[0] % ncopy]; it[0] += 1
                assert lib.zk_gemv_warm(ptr(W), N, K, lay, steps, S) == 0

            def pair():
                W = Ws[it[0] % ncopy]; it[0] += 1
                assert lib.zk_gemv_warm(ptr(W), N, K, lay, steps, S) == 0
                call("zk_gemv_fused", ptr(x), K, ptr(W), M, N, K, mode, ptr(lw) if ln else None,
                     ptr(lb) if ln else None, 1e-5, ptr(outf), ptr(res) if mode == 2 else ptr(outb), None, S)
            tw, tp = timeit(wg), timeit(pair)
            print(f"gemv_warm {name:4s} steps {steps:2d}/{nl}: cold {tc:6.2f} us, warm kernel {tw:5.2f}, pair {tp:6.2f}"
                  f" -> gemv after warm-up {tp - tw:6.2f} us", flush=True)
        del Ws


def dac():
    from zonos_amd import synthetic
    from zonos_amd.autoencoder import DacSpec, HipDacDecoder
    W = synthetic.dac_weights(dev)
    for prec in os.environ.get("ZK_MB_DAC_PREC", "fp16").split(","):
        d = HipDacDecoder(DacSpec(), W, dev, precision=prec)
        for B, T in ((8, 256), (16, 2580)):
            codes = torch.randint(0, 1024, (B, 9, T), device=dev)
            us = timeit(lambda: d.decode_padded(codes), reps=3, warm=1)
            fl = 1.6083e9 * B * T
            print(f"dac {prec:6s} B={B} T={T}: {us/1e3:8.1f} ms  {fl / (us * 1e-6) / 1e12:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "warm":
        warm()
    if what in ("gemm", "all"):
        gemm()
    if what == "sweep":
        sweep()
    if what in ("mamba",):
        mamba()
    if what in ("attn_small",):
        attn_small()
    if what in ("gemv",):
        gemv()
    if what == "gemv_warm":
        gemv_warm()
    if what in ("prefill", "all"):
        prefill()
    if what in ("ln", "all"):
        ln()
    if what in ("attn", "all"):
        attn()
    if what in ("dac", "all"):
        dac()
