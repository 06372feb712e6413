"""Benchmark: DAC codes/s + real-time factor of the Zonos hot path on MI355X.

Workload (BASELINE.json configs[2]): Zonos-v0.1-transformer
(D=2048, 26 layers, 16/4 heads, FFN 8192, 1.62 B params, seeded random bf16 weights --
no checkpoint is available offline), batch 64 utterances per GPU, synthetic LayerNorm'd
conditioning Lc=400, 10 prefix frames, 2580 new tokens (30 s of audio) with EOS
acceptance disabled so every row runs the full length, CLI sampling defaults; then the
DAC decoder (descript/dac_44khz geometry, seeded fp32 weights; fp16 conv operands with fp32
accumulation = the reference's own GPU numerics, torch.autocast fp16 at autoencoder.py:46)
turns all codes into waveforms. One "step" = generate() + DAC decode of the whole per-GPU
batch. Other configs: --batch 1 --lc 160 --prefix 0 --new-tokens 861 (c2), --model hybrid (c5).

Multi-GPU: one process per GPU. `python bench.py --gpus N` starts torchrun itself (N ranks,
127.0.0.1) before touching the GPU; under torchrun WORLD_SIZE must equal --gpus. Utterances
are sharded by rank (row_base = rank * B keys the sampling noise), each rank runs its own
engine with no data-path collective (zonos_amd.distributed.generate_sharded, the library
path), and one RCCL all_gather of the int32 codes closes each generate. Codes are shard-invariant as long as every shard has the same per-GPU batch (the GEMM
reduction order depends on the M regime). value = codes of all ranks /
max-over-ranks wall time ("scaling": "weak").

Prints ONE JSON line on rank 0. `--stub` replaces the GPU workload by a CPU stand-in (gloo) so
the launcher and the reporting path can be tested without a GPU (tests/test_bench_cpu.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FRAME_RATE = 44100 / 512          # DAC frames per second of audio (86.13)
HBM_PEAK_GBS = 8000.0             # MI355X spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", 1)))
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lc", type=int, default=400)
    ap.add_argument("--prefix", type=int, default=10)
    ap.add_argument("--new-tokens", type=int, default=2580)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--model", choices=["transformer", "hybrid"], default="transformer",
                    help="hybrid = Zonos-v0.1-hybrid geometry as assumed in synthetic.ZONOS_V01_HYBRID (config 5)")
    ap.add_argument("--no-dac", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-steps", type=int, default=1)
    ap.add_argument("--stub", action="store_true", help="CPU stand-in workload (launcher/reporting tests)")
    ap.add_argument("--graph-steps", type=int, default=None,
                    help="decode steps per hipGraph replay (default: the engine's graph_steps)")
    ap.add_argument("--dac-overlap", type=int, default=0,
                    help="1: decode each step's codes to waveforms on a side stream while the next step's generate "
                         "runs (the DAC's MFMA-bound convs beside the HBM-bound decode); 0: serial")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary measurements after a 1-GPU c3 run (c2, c5, c3 through Zonos.generate)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int | None:
    """--gpus N > 1 without a torchrun environment: run this script under torchrun (one rank per
    GPU) as a CHILD process -- nothing here has touched the GPU yet -- and return its exit code."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}")
        return None
    if args.gpus <= 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------ rooflines
def _time_launches(launches, reps=2):
    """Average duration of the given launch closures (each called with the stream) with HIP
    events on the engine's stream, after one warm pass. Returns seconds per launch."""
    import ctypes as C

    from zonos_amd import _lib
    from zonos_amd._lib import call
    stream = _lib.stream_ptr()
    e0, e1 = _lib.P(), _lib.P()
    call("zk_event_create", C.byref(e0))
    call("zk_event_create", C.byref(e1))
    for f in launches:
        f(stream)
    call("zk_event_record", e0.value, stream)
    for _ in range(reps):
        for f in launches:
            f(stream)
    call("zk_event_record", e1.value, stream)
    ms = C.c_float()
    call("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
    call("zk_event_destroy", e0.value)
    call("zk_event_destroy", e1.value)
    return ms.value / 1e3 / (reps * len(launches))


def _pmc_traffic(kernel_prefix: str, **shape):
    """HBM bytes per launch from the committed rocprofv3 PMC summaries (profiles/*pmc*.json,
    written by tools/attn_pmc.py / tools/gemm_pmc.py), matching kernel name prefix and shape."""
    import glob
    found = None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        for e in (d if isinstance(d, list) else [d]):
            if str(e.get("kernel", "")).startswith(kernel_prefix) and all(e.get(k) == v for k, v in shape.items()):
                found = e["hbm_bytes_per_launch"]
    return found


def _roof(bytes_per_launch, per_launch_s, **extra):
    ach = bytes_per_launch / per_launch_s / 1e9
    return dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                bytes_per_launch=int(bytes_per_launch), us_per_launch=round(per_launch_s * 1e6, 2), **extra)


def attn_roofline(eng, ctx):
    """Decode attention with the fused in_proj epilogue (zk_attn_decode_qkv), launched as the
    generate loop launches it, over the 26 layers' own KV caches in turn at the workload's mean
    context. Algorithmic bytes per launch = K+V rows read (R*ctx*Hkv*hd*2*2) + in_proj slabs read
    (nsplit*R*(H+2Hkv)*hd*4) + output write + new K/V write."""
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R, Hk, hd, H = ws["R"], c.n_kv, c.head_dim, c.n_heads
    gs = ws["splits"]["qkv"]

    def launch(layer):
        kc, vt = eng._kv(ws, layer)
        return lambda st: call("zk_attn_decode_qkv", ptr(ws["part"]), gs, ptr(eng.freqs), ptr(kc), ptr(vt), R, H, Hk,
                               hd, ws["smax"], ctx, None, ptr(ws["attn_work"]), ws["attn_splits"], ptr(ws["y"]),
                               eng.rope_neox, None, st)
    layers = getattr(eng, "attn_ids", range(c.n_layer))
    per = _time_launches([launch(i) for i in layers], reps=4)
    Nq = (H + 2 * Hk) * hd
    b = R * ctx * Hk * hd * 2 * 2 + gs * R * Nq * 4 + R * H * hd * 2 + R * Hk * hd * 2 * 2
    return _roof(b, per, traffic=_pmc_traffic("k_attn_decode<true", R=R, ctx=ctx),
                 kernel="k_attn_decode<true> (zk_attn_decode_qkv)" + ("+k_attn_combine" if ws["attn_splits"] > 1 else ""),
                 ctx=ctx, attn_splits=ws["attn_splits"], layers="rotating over all attention layers' caches")


def gemm_roofline(eng):
    """The decode step's weight GEMMs (k_gemm_ws, 16 < R <= 128) and split-K slab reduces (k_resid_ln),
    each launched as the step launches it (same shapes, splits and kernels) over the 26 layers'
    weights in turn, timed with HIP events; algorithmic bytes = weights + activation + output once
    (tools/gemm_pmc.py alg_bytes / reduce_bytes); traffic = PMC HBM bytes per launch of the same
    kernel at the same shape (profiles/*gemm_pmc*.json: FETCH_SIZE x2 + WRITE_SIZE). Isolated
    launches: inside the step the L2 warm-up by the kernel before each GEMM shortens it further."""
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R, D, H, Hk, hd, Fd = ws["R"], c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
    sp = ws["splits"]
    Nq = (H + 2 * Hk) * hd
    part, h, xn, x, y = ws["part"], ws["h"], ws["xn"], ws["x"], ws["y"]
    gemms = [("in_proj", "wqkv", xn, Nq, D, sp["qkv"], 0), ("out_proj", "wo", y, D, H * hd, sp["o"], 0),
             ("fc1", "fc1", xn, 2 * Fd, D, 1, 1), ("fc2", "fc2", h, D, Fd, sp["fc2"], 0)]
    out = {}
    for name, key, A, N, K, ns, mode in gemms:
        def launch(L, A=A, N=N, K=K, ns=ns, mode=mode, key=key):
            return lambda st: call("zk_gemm_bf16", ptr(A), K, ptr(L[key]), R, N, K, ns, mode, ptr(part), ptr(h), None,
                                   st)
        per = _time_launches([launch(L) for L in eng.layers], reps=2)
        b = N * K * 2 + R * K * 2 + (R * N * 4 * ns if mode == 0 else R * (N // 2) * 2)
        out[name] = dict(M=R, N=N, K=K, nsplit=ns, bytes=int(b), us=round(per * 1e6, 2),
                         frac=round(b / per / 1e9 / HBM_PEAK_GBS, 4),
                         traffic_ratio=_pmc_field("k_gemm_ws", "traffic_ratio", name=name, M=R))
    Nh = 9 * 1026
    per = _time_launches([lambda st: call("zk_gemm_bf16", ptr(xn), D, ptr(eng.heads), R, Nh, D, sp["heads"], 0,
                                          ptr(part), None, None, st)], reps=8)
    b = Nh * D * 2 + R * D * 2 + R * Nh * 4 * sp["heads"]
    out["heads"] = dict(M=R, N=Nh, K=D, nsplit=sp["heads"], bytes=int(b), us=round(per * 1e6, 2),
                        frac=round(b / per / 1e9 / HBM_PEAK_GBS, 4),
                        traffic_ratio=_pmc_field("k_gemm_ws", "traffic_ratio", name="heads", M=R))
    for ns in sorted({sp["o"], sp["fc2"]}):
        def launch(L, ns=ns):
            return lambda st: call("zk_resid_ln", ptr(part), ns, ptr(x), ptr(L["ln2_w"]), ptr(L["ln2_b"]), c.eps, R, D,
                                   ptr(x), ptr(xn), 0, None, st)
        per = _time_launches([launch(L) for L in eng.layers], reps=2)
        b = ns * R * D * 4 + R * D * 2 + 2 * D * 2 + 2 * R * D * 2
        out[f"resid_ln{ns}"] = dict(M=R, nsplit=ns, bytes=int(b), us=round(per * 1e6, 2),
                                    frac=round(b / per / 1e9 / HBM_PEAK_GBS, 4),
                                    traffic_ratio=_pmc_field("k_resid_ln", "traffic_ratio", name=f"resid_ln{ns}", M=R))
    per_step = 26 * sum(v["us"] for k, v in out.items() if k != "heads") + out["heads"]["us"]
    return dict(unit="us / launch (isolated)", peak_gbs=HBM_PEAK_GBS, per_step_us=round(per_step, 1), **out)


def hybrid_gemm_roofline(eng):
    """c5: the Mamba2 layers' weight GEMMs (in_proj 2048 -> 8512 unsplit, out_proj 4096 -> 2048 split-K) and
    the slab reduce after out_proj, launched as the hybrid step launches them over the Mamba layers' weights
    in turn, HIP events; bytes = weights + activation + output once. (The SSM update itself: `roofline`.)"""
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R, D, di = ws["R"], c.d_model, c.d_inner
    sp = ws["splits"]
    nin = c.d_in_proj
    part, xn = ws["part"], ws["xn"]
    Ls = [eng.layers[j] for j in eng.mamba_ids]
    out = {}
    for name, key, A, N, K, ns in (("mamba_in_proj", "w_in", xn, nin, D, sp["inp"]),
                                   ("mamba_out_proj", "w_out", ws["ym"], D, di, sp["out"])):
        def launch(L, A=A, N=N, K=K, ns=ns, key=key):
            return lambda st: call("zk_gemm_bf16", ptr(A), K, ptr(L[key]), R, N, K, ns, 0, ptr(part), None, None, st)
        per = _time_launches([launch(L) for L in Ls], reps=2)
        b = N * K * 2 + R * K * 2 + R * N * 4 * ns
        out[name] = dict(M=R, N=N, K=K, nsplit=ns, bytes=int(b), us=round(per * 1e6, 2),
                         frac=round(b / per / 1e9 / HBM_PEAK_GBS, 4))
    return dict(unit="us / launch (isolated)", peak_gbs=HBM_PEAK_GBS, **out)


def _pmc_field(kernel_prefix: str, field: str, **shape):
    """A field of the committed PMC summary entry matching the kernel prefix and shape (or None)."""
    import glob
    found = None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except ValueError:
            continue
        for e in (d if isinstance(d, list) else [d]):
            if str(e.get("kernel", "")).startswith(kernel_prefix) and all(e.get(k) == v for k, v in shape.items()):
                found = e.get(field)
    return found


def gemv_roofline(eng):
    """B <= 8 (c2): the largest launch of the small-batch step -- fc1 with the norm2 LayerNorm
    prologue and the SwiGLU epilogue (zk_gemv_fused -> k_gemv_f), launched as _layers_small
    launches it, over the 26 layers' fc1 weights in turn (67 MB each: nothing stays in L2/MALL
    between launches, as in the real step). Bytes = weights + residual rows + LN w/b + output."""
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R, D, Fd = ws["R"], c.d_model, c.d_ff

    def launch(L):
        return lambda st: call("zk_gemv_fused", ptr(ws["x"]), D, ptr(L["fc1"]), R, 2 * Fd, D, 1, ptr(L["ln2_w"]),
                               ptr(L["ln2_b"]), c.eps, None, ptr(ws["h"]), None, st)
    per = _time_launches([launch(L) for L in eng.layers if "fc1" in L], reps=4)
    b = 2 * Fd * D * 2 + R * D * 2 + 2 * D * 2 + R * Fd * 2
    return _roof(b, per, traffic=_pmc_traffic("k_gemv_f<1, true", R=R, N=2 * Fd, K=D),
                 kernel="k_gemv_f<1,true,2> (zk_gemv_fused: norm2 LayerNorm + fc1 + SwiGLU)", M=R, N=2 * Fd, K=D,
                 layers="rotating over all layers' fc1 weights")


def mamba_roofline(eng):
    """Hybrid (c5): zk_mamba_step (the SSM state update, HBM-bound) over every Mamba layer's state
    in turn; algorithmic bytes = SSM state read + write (R*d_inner*d_state*2 B each) + conv state
    read + write + in_proj slabs read + yz write."""
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R = ws["R"]
    gs = ws["splits"]["inp"]

    def launch(j):
        L = eng.layers[eng.mamba_ids[j]]
        return lambda st: call("zk_mamba_step", ptr(ws["part"]), gs, R, c.d_inner, c.nheads_ssm, c.headdim,
                               c.d_state, ptr(L["conv_w"]), ptr(L["conv_b"]), ptr(ws["conv"][j][0]),
                               ptr(ws["conv"][j][1]), ptr(ws["scal"][1:2]), ptr(ws["ssm"][j][0]), ptr(ws["ssm"][j][1]),
                               ptr(L["A"]), ptr(L["dt_bias"]), ptr(L["D"]), ptr(ws["yz"]), None, st)
    per = _time_launches([launch(j) for j in range(len(eng.mamba_ids))], reps=4)
    b = R * c.d_inner * c.d_state * 2 * 2 + R * c.conv_dim * 8 * 2 + gs * R * c.d_in_proj * 4 + R * c.d_inner * 4
    return _roof(b, per, traffic=_pmc_traffic("k_mamba_step", R=R), kernel="k_mamba_step",
                 layers="rotating over all Mamba layers' states")


def step_bytes(eng, R: int, ctx: float) -> float:
    """Algorithmic HBM bytes of one decode step at context ctx: every weight once
    (bf16 GEMM weights, LayerNorms, heads) + the KV cache read (R*ctx rows) and written (R rows);
    hybrid: + every Mamba layer's SSM state read and written and conv state."""
    c = eng.cfg
    D, H, Hk, hd = c.d_model, c.n_heads, c.n_kv, c.head_dim
    attn_layer = (H + 2 * Hk) * hd * D + D * H * hd + 3 * c.d_ff * D + 4 * D
    kv_row = 2 * Hk * hd * 2
    n_attn = len(getattr(eng, "attn_ids", range(c.n_layer)))
    b = 2 * (n_attn * attn_layer + 2 * D + 9 * 1026 * D) + n_attn * kv_row * R * (ctx + 1)
    if hasattr(eng, "mamba_ids"):
        nm = len(eng.mamba_ids)
        b += 2 * nm * (c.d_in_proj * D + D * c.d_inner + c.d_inner + 2 * D + c.conv_dim * 5 + 3 * c.nheads_ssm)
        b += nm * R * (2 * c.d_inner * c.d_state * 2 + 2 * c.conv_dim * 4 * 2)
    return b


# ------------------------------------------------------------------------------ CPU baseline
def cpu_baseline(args):
    """Oracle (CPU restatement, validated against the reference) timed on this host: decode
    steps at B=64 at 3 context lengths (KV cache pre-filled) + a 43-frame DAC decode; scaled
    to codes/s of the same workload (prefill excluded, <1% of the GPU time). Threads = the
    box's CPU share (16 per GPU)."""
    import torch

    from oracle import dac_ref, zonos_ref
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", 16)), 16)
    torch.set_num_threads(threads)
    cfg = zonos_ref.ZONOS_V01_TRANSFORMER
    W = zonos_ref.pad_heads(zonos_ref.make_weights(cfg, seed=0), cfg)
    B = args.batch
    N = args.new_tokens + 8
    ctx0 = args.lc + args.prefix + 1
    freqs = zonos_ref.rope_table(16384, cfg.head_dim)
    times = []
    t_begin = time.time()
    ctxs = [int(ctx0 + frac * N) for frac in (0.1, 0.5, 0.9)]
    # one cache sized for the longest context, filled once (cache contents do not change the
    # work; random fill of ~19 GB would dominate the sample)
    kv = zonos_ref.KVCache(cfg, 2 * B, max(ctxs) + 1)
    for layer in kv.kv:
        layer.fill_(0.01)
    t_setup = time.time() - t_begin
    for ctx in ctxs:
        ids = torch.randint(0, 1024, (2 * B, 9, 1))
        for _ in range(args.cpu_sample_steps):
            kv.seqlen_offset = ctx
            kv.lengths[:] = ctx
            t = time.time()
            with torch.no_grad():
                zonos_ref.compute_logits(W, cfg, zonos_ref.embed_codes(W, cfg, ids), kv, freqs, 2.0)
            times.append(time.time() - t)
    step_s = sum(times) / len(times)
    dW = dac_ref.make_dac_weights(dac_ref.DAC_44KHZ, seed=0)
    T = 43
    codes = torch.randint(0, 1024, (1, 9, T))
    t = time.time()
    dac_ref.decode(dW, dac_ref.DAC_44KHZ, codes)
    dac_s_per_frame = (time.time() - t) / T
    total_s = N * step_s + B * args.new_tokens * dac_s_per_frame
    codes_total = B * args.new_tokens * 9
    return dict(value=round(codes_total / total_s, 2), unit="codes/s", cores=threads, kind="port",
                sample=f"oracle decode step B={B} at ctx {ctxs[0]}/{ctxs[1]}/{ctxs[2]} x{args.cpu_sample_steps} "
                       f"(mean {step_s:.3f} s/step) + DAC 43 frames ({dac_s_per_frame * 1e3:.1f} ms/frame); scaled to "
                       f"{N} steps + {B * args.new_tokens} frames; {time.time() - t_begin - t_setup:.1f} s of timed "
                       f"CPU work (+{t_setup:.1f} s setup)",
                step_s=round(step_s, 4), dac_ms_per_frame=round(dac_s_per_frame * 1e3, 2))


# ------------------------------------------------------------------------------ workloads
class StubWorkload:
    """CPU stand-in with the real workload's interface: 'generates' B utterances of new_tokens
    frames per step (a short sleep) and gathers them over gloo like the codes gather."""

    def __init__(self, args, rank, world, dist):
        import torch
        self.args, self.rank, self.dist, self.torch = args, rank, dist, torch
        self.stats = {"gen_s": 0.0, "dac_s": 0.0}
        self.model_name = "stub"

    def step(self, i, timed):
        torch = self.torch
        B, T = self.args.batch, self.args.new_tokens
        time.sleep(0.01 * (1 + self.rank))
        codes = [torch.full((9, T), self.rank * B + b, dtype=torch.int64) for b in range(B)]
        if self.dist is not None:
            from zonos_amd.distributed import gather_codes
            allc = gather_codes(codes)
            assert len(allc) == B * self.dist.get_world_size()
        return B * T

    def sync(self):
        pass

    def report(self, elapsed, args):
        return {}


class GpuWorkload:
    def __init__(self, args, rank, world, dist, dev):
        import torch

        from zonos_amd import synthetic
        from zonos_amd.autoencoder import DacSpec, HipDacDecoder
        from zonos_amd.engine import EngineConfig, HipDecoder
        self.torch, self.args, self.rank, self.world, self.dist, self.dev = torch, args, rank, world, dist, dev
        if args.model == "hybrid":
            from zonos_amd.hybrid import HybridDecoder, HybridEngineConfig
            mc = dict(synthetic.ZONOS_V01_HYBRID)
            if args.layers:
                mc["n_layer"] = args.layers
                mc["attn_layer_idx"] = tuple(i for i in mc["attn_layer_idx"] if i < args.layers)
            W = synthetic.hybrid_weights(dev, seed=0, **mc)
            self.eng = HybridDecoder(HybridEngineConfig(**mc), W, dev)
        else:
            mc = dict(synthetic.ZONOS_V01, n_layer=args.layers or 26)
            W = synthetic.backbone_weights(dev, seed=0, **mc)
            self.eng = HipDecoder(EngineConfig(**mc), W, dev)
        del W
        if args.graph_steps:
            self.eng.graph_steps = args.graph_steps
        self.mc = mc
        self.dac = None if args.no_dac else HipDacDecoder(DacSpec(), synthetic.dac_weights(dev), dev)
        B = args.batch
        self.cond = synthetic.conditioning(B, args.lc, mc["d_model"], seed=1 + rank, device=dev)
        self.prefix = synthetic.prefix_codes(B, args.prefix, seed=3 + rank, device=dev) if args.prefix else None
        self.sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
                       repetition_penalty_window=8, temperature=1.0)
        self.stats = {"gen_s": 0.0, "dac_s": 0.0}
        self.model_name = ("Zonos-v0.1-transformer" if args.model == "transformer"
                           else "Zonos-v0.1-hybrid (assumed geometry)")
        self.side = torch.cuda.Stream(dev) if args.dac_overlap else None
        self.dac_events = []

    def step(self, i, timed):
        torch, args = self.torch, self.args
        if self.side is not None:
            return self._step_overlap(i, timed)
        t0 = time.time()
        from zonos_amd.distributed import generate_sharded
        # the library's sharded generate: this rank's B utterances of the global B x world batch
        # (row_base = rank * B keys the noise), then one all_gather of the int32 codes
        codes, allc = generate_sharded(self.eng, self.cond, self.prefix, args.new_tokens, 2.0,
                                       args.batch * self.world, self.sp, seed=1000 + i, local_input=True,
                                       coll_device=self.coll_dev, return_local=True, force_full_length=True,
                                       poll_every=64)
        assert len(codes) == args.batch and len(allc) == args.batch * self.world
        torch.cuda.synchronize(self.dev)
        t1 = time.time()
        if self.dac is not None:
            self.dac.decode_list(codes)
        torch.cuda.synchronize(self.dev)
        t2 = time.time()
        if timed:
            self.stats["gen_s"] += t1 - t0
            self.stats["dac_s"] += t2 - t1
        return sum(int(c.shape[1]) for c in codes)

    def _step_overlap(self, i, timed):
        """--dac-overlap 1: generate on the engine's stream, then this batch's DAC decode enqueued on a side
        stream, so it runs while the next step's generate does (the last step's DAC is waited for by sync()
        inside the timed region). DAC time = HIP events on the side stream (its own duration, overlapped)."""
        torch, args = self.torch, self.args
        from zonos_amd.distributed import generate_sharded
        t0 = time.time()
        codes, allc = generate_sharded(self.eng, self.cond, self.prefix, args.new_tokens, 2.0,
                                       args.batch * self.world, self.sp, seed=1000 + i, local_input=True,
                                       coll_device=self.coll_dev, return_local=True, force_full_length=True,
                                       poll_every=64)
        assert len(codes) == args.batch and len(allc) == args.batch * self.world
        main = torch.cuda.current_stream(self.dev)
        main.synchronize()
        t1 = time.time()
        if timed:
            self.stats["gen_s"] += t1 - t0
        if self.dac is not None:
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                for c in codes:
                    c.record_stream(self.side)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(self.side)
                self.dac.decode_list(codes)
                e1.record(self.side)
            if timed:
                self.dac_events.append((e0, e1))
        return sum(int(c.shape[1]) for c in codes)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def report(self, elapsed, args):
        if self.dac_events:
            self.stats["dac_s"] = sum(a.elapsed_time(b) for a, b in self.dac_events) / 1e3
        eng = self.eng
        R = 2 * args.batch
        n_dec = args.new_tokens + 8                       # decode steps per generate (max_steps)
        ctx_mean = args.lc + args.prefix + 1 + n_dec // 2
        if args.model == "hybrid":
            roof = mamba_roofline(eng)
        elif eng._small(R):
            roof = gemv_roofline(eng)
        else:
            roof = attn_roofline(eng, ctx_mean)
        gen_step_s = self.stats["gen_s"] / args.steps
        dec_ms = gen_step_s / n_dec * 1e3
        sb = step_bytes(eng, R, ctx_mean)
        step_roof = dict(bytes_per_step=int(sb), ctx_mean=ctx_mean, ms_per_decode_step=round(dec_ms, 4),
                         achieved=round(sb / (dec_ms / 1e3) / 1e9, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                         frac=round(sb / (dec_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         note="algorithmic bytes per decode step at the mean context / (generate wall time / decode "
                              "steps, prefill included)")
        extra = {}
        if args.model != "hybrid" and not eng._small(R) and R <= 128:
            extra["gemm_roofline"] = gemm_roofline(eng)
        return dict(roofline=roof, step_roofline=step_roof, **extra,
                    breakdown={"generate_s_per_step": round(gen_step_s, 3),
                               "dac_s_per_step": round(self.stats["dac_s"] / args.steps, 3),
                               "dac_overlap": bool(args.dac_overlap),
                               "dac_exposed_s_per_step": round(max(0.0, elapsed / args.steps - gen_step_s), 3),
                               "dac_precision": self.dac.precision if self.dac is not None else None,
                               "decode_ms_per_token_step": round(dec_ms, 3)})


# ------------------------------------------------------------------------------ secondary configs
SECONDARY_SP = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
                    repetition_penalty_window=8, temperature=1.0)


def _timed_config(torch, dev, generate, dac, B, lc, P, new, reps, warmup, roofline=None, eng=None):
    """Time `generate(i)` (-> list of [9, T] codes) + the DAC decode of its codes, warmup + reps times,
    and report the config's codes/s, RTF, decode step time and step roofline like the headline line."""
    gen_s = dac_s = 0.0
    frames = 0
    for i in range(warmup + reps):
        print(f"[bench] secondary rep {i + 1}/{warmup + reps} (B={B}, {new} tokens)", file=sys.stderr, flush=True)
        torch.cuda.synchronize(dev)
        t0 = time.time()
        codes = generate(i)
        torch.cuda.synchronize(dev)
        t1 = time.time()
        if dac is not None:
            dac.decode_list(codes)
        torch.cuda.synchronize(dev)
        t2 = time.time()
        if i >= warmup:
            gen_s += t1 - t0
            dac_s += t2 - t1
            frames += sum(int(c.shape[1]) for c in codes)
    elapsed = gen_s + dac_s
    n_dec = new + 8
    ctx_mean = lc + P + 1 + n_dec // 2
    dec_ms = gen_s / reps / n_dec * 1e3
    out = dict(value=round(frames * 9 / elapsed, 1), unit="codes/s", rtf=round(frames / FRAME_RATE / elapsed, 2),
               reps=reps, warmup=warmup, ms_per_rep=round(elapsed / reps * 1e3, 1),
               breakdown={"generate_s_per_rep": round(gen_s / reps, 4), "dac_s_per_rep": round(dac_s / reps, 4),
                          "decode_ms_per_token_step": round(dec_ms, 4)})
    if eng is not None:
        sb = step_bytes(eng, 2 * B, ctx_mean)
        out["step_roofline"] = dict(bytes_per_step=int(sb), ctx_mean=ctx_mean, ms_per_decode_step=round(dec_ms, 4),
                                    achieved=round(sb / (dec_ms / 1e3) / 1e9, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                                    frac=round(sb / (dec_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4))
    if roofline is not None:
        out["roofline"] = roofline()
    return out


def secondary_runs(args, wl, headline_value):
    """after the headline c3 line, on the same box and in the same run,
    * c2 (BASELINE configs[1]: B = 1, Lc 160, 861 tokens) on the same engine and weights;
    * c3 through the API callers use -- ``zonos.model.Zonos.generate`` with ``seed=None`` (the
      reference's torch noise stream), the default poll interval and the tqdm progress bar, DAC via
      ``model.autoencoder`` -- beside the keyed-engine headline (``generate_sharded``, poll 64);
    * c5 (configs[4]: the hybrid at B = 64, c3 lengths).
    Each as codes/s + RTF (generate + DAC decode of all codes, EOS disabled as in the headline),
    whole-step roofline and the dominant kernel's roofline (HIP events)."""
    import torch

    from zonos_amd import synthetic
    from zonos_amd.distributed import generate_sharded
    dev = wl.dev
    out = {}
    t_all = time.time()
    # --- c2 on the headline engine
    eng = wl.eng
    cond2 = synthetic.conditioning(1, 160, 2048, seed=11, device=dev)
    out["c2"] = dict(workload="c2: B=1, Lc=160, no prefix, 861 new tokens (10 s), EOS disabled, CLI sampling, "
                              "DAC decode; same engine and weights as the headline",
                     **_timed_config(torch, dev, lambda i: generate_sharded(
                         eng, cond2, None, 861, 2.0, 1, wl.sp, seed=2000 + i, force_full_length=True, poll_every=64),
                         wl.dac, 1, 160, 0, 861, reps=3, warmup=1, roofline=lambda: gemv_roofline(eng), eng=eng))
    eng.release()
    wl.eng = None
    del eng
    torch.cuda.empty_cache()
    # --- c3 through Zonos.generate (seed=None: torch's generator stream, poll 16, tqdm)
    from zonos_amd.autoencoder import DACAutoencoder
    from zonos_amd.config import BackboneConfig, PrefixConditionerConfig, ZonosConfig
    from zonos_amd.model import Zonos
    mc = wl.mc
    zc = ZonosConfig(BackboneConfig(d_model=mc["d_model"], attn_mlp_d_intermediate=mc["d_ff"], n_layer=mc["n_layer"],
                                    attn_cfg={"num_heads": mc["n_heads"], "num_heads_kv": mc["n_kv"]}),
                     PrefixConditionerConfig([], "none"))
    model = Zonos(zc, synthetic.backbone_weights(dev, seed=0, **mc), dev,
                  autoencoder=DACAutoencoder(state_dict=synthetic.dac_weights(dev), device=dev))
    torch.manual_seed(1234)
    B = args.batch
    dac = model.autoencoder if wl.dac is not None else None
    r = _timed_config(torch, dev, lambda i: model.generate(wl.cond, wl.prefix, args.new_tokens, 2.0, B, wl.sp,
                                                           force_full_length=True),
                      dac, B, args.lc, args.prefix, args.new_tokens, reps=1, warmup=1, eng=model.engine)
    out["c3_zonos_generate"] = dict(
        workload="c3 through zonos.model.Zonos.generate(seed=None): torch's CUDA generator noise (the reference's "
                 "exponential_ stream), poll every 16 steps, tqdm progress bar; DAC via model.autoencoder.decode_list; "
                 "force_full_length (EOS disabled) as in the headline",
        ratio_to_headline=round(r["value"] / headline_value, 4), **r)
    model.engine.release()
    del model
    torch.cuda.empty_cache()
    # --- c5: the hybrid at B = 64, c3 lengths
    from zonos_amd.hybrid import HybridDecoder, HybridEngineConfig
    hc = dict(synthetic.ZONOS_V01_HYBRID)
    heng = HybridDecoder(HybridEngineConfig(**hc), synthetic.hybrid_weights(dev, seed=0, **hc), dev)
    out["c5"] = dict(workload="c5: Zonos-v0.1-hybrid (assumed geometry: 46 layers, attention at 9/18/27/36/45, Mamba2 "
                              "defaults), B=64, Lc=400, prefix 10, 2580 new tokens, EOS disabled, DAC decode",
                     **_timed_config(torch, dev, lambda i: generate_sharded(
                         heng, wl.cond, wl.prefix, args.new_tokens, 2.0, B, wl.sp, seed=3000 + i,
                         force_full_length=True, poll_every=64),
                         wl.dac, B, args.lc, args.prefix, args.new_tokens, reps=2, warmup=1,
                         roofline=lambda: mamba_roofline(heng), eng=heng),
                     gemm_roofline=hybrid_gemm_roofline(heng))
    heng.release()
    del heng
    torch.cuda.empty_cache()
    out["wall_s"] = round(time.time() - t_all, 1)
    return out


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if args.stub:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        wl = StubWorkload(args, rank, world, dist)
    else:
        # ZK_BENCH_SHARE_GPU=1: rehearsal of the N-rank path on a one-GPU box -- every rank on
        # cuda:0 and the collectives over gloo on host tensors (RCCL refuses two ranks on one GPU)
        share = os.environ.get("ZK_BENCH_SHARE_GPU") == "1"
        torch.cuda.set_device(0 if share else local)
        dev = torch.device("cuda", 0 if share else local)
        if world > 1:
            import torch.distributed as dist
            if share:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=dev)
        wl = GpuWorkload(args, rank, world, dist, dev)
        wl.coll_dev = torch.device("cpu") if share else dev

    def progress(msg):      # stderr, rank 0: long runs show they are alive (stdout keeps the one JSON line)
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    for i in range(args.warmup):
        wl.step(i, False)
        progress(f"warm-up step {i + 1}/{args.warmup}")
    if dist is not None:
        dist.barrier()
    wl.sync()
    t0 = time.time()
    frames = 0
    for i in range(args.steps):
        frames += wl.step(args.warmup + i, True)
        progress(f"timed step {i + 1}/{args.steps}")
    wl.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    if dist is not None:
        dev_ = "cpu" if args.stub else wl.coll_dev
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        fr = torch.tensor([frames], dtype=torch.float64, device=dev_)
        dist.all_reduce(fr)
        frames = int(fr.item())

    if rank == 0:
        codes_s = frames * 9 / elapsed
        audio_s = frames / FRAME_RATE
        B = args.batch
        cfg_name = {(64, 400, 10, 2580): "c3", (1, 160, 0, 861): "c2"}.get(
            (args.batch, args.lc, args.prefix, args.new_tokens), "custom")
        if args.model == "hybrid" and cfg_name == "c3":
            cfg_name = "c5"
        if cfg_name == "c3" and world > 1:
            cfg_name = "c4" if world == 8 else f"c3x{world}"
        workload = (f"{cfg_name}: B={B}/GPU, Lc={args.lc}, prefix {args.prefix}, {args.new_tokens} new tokens "
                    f"({args.new_tokens / FRAME_RATE:.0f} s), EOS disabled, CLI sampling (linear .65 conf .4 rep "
                    f"2.5/8), DAC decode of all codes")
        out = {
            "metric": f"DAC codes/sec (end-to-end generate + DAC decode), {wl.model_name} batch={B}/GPU",
            "value": round(codes_s, 1), "unit": "codes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded random weights + LayerNorm'd random conditioning; no checkpoint offline)",
            "config": {"workload": workload, "model": wl.model_name, "global_batch": B * world,
                       "seq_len": args.lc + args.prefix + args.new_tokens + 9, "parallelism": f"dp{world}"},
            "rtf": round(audio_s / elapsed, 2),
        }
        out.update(wl.report(elapsed, args))
        if not args.stub and not args.no_cpu_baseline and world == 1 and args.model == "transformer":
            out["cpu_baseline"] = cpu_baseline(args)
        if (not args.stub and not args.no_secondary and world == 1 and cfg_name == "c3"
                and args.model == "transformer" and not args.layers):
            out["secondary"] = secondary_runs(args, wl, out["value"])
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
