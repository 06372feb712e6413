"""Benchmark: DAC codes/s + real-time factor of the Zonos hot path on MI355X.

Workload (BASELINE.json configs[2]): Zonos-v0.1-transformer
(D=2048, 26 layers, 16/4 heads, FFN 8192, 1.62 B params, seeded random bf16 weights --
no checkpoint is available offline), batch 64 utterances per GPU, synthetic LayerNorm'd
conditioning Lc=400, 10 prefix frames, 2580 new tokens (30 s of audio) with EOS
acceptance disabled so every row runs the full length, CLI sampling defaults; then the
DAC decoder (descript/dac_44khz geometry, seeded fp32 weights; fp16 conv operands with fp32
accumulation = the reference's own GPU numerics, torch.autocast fp16 at autoencoder.py:46)
turns all codes into waveforms. One "step" = generate() + DAC decode of the whole per-GPU
batch.

Multi-GPU: one process per GPU (torchrun), utterances sharded by rank (row_base keys the
noise, so codes equal a single big batch), RCCL all_gather of the int32 codes at the end
of each step; value = codes of all ranks / max-over-ranks wall time ("scaling": "weak").

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

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
    return ap.parse_args()


def attn_roofline(eng, ctx, reps=50):
    """Time the dominant kernel -- the decode attention with the fused in_proj epilogue
    (zk_attn_decode_qkv), as the generate loop launches it -- with HIP events on its stream at
    the workload's mean context. Algorithmic bytes per launch = K+V rows read (R*ctx*Hkv*hd*2*2)
    + in_proj slabs read (nsplit*R*(H+2Hkv)*hd*4) + out write + new K/V write. traffic: the
    PMC-measured HBM bytes per launch of the same kernel and shape, from the committed
    rocprofv3 summary (profiles/*attn_pmc.json, tools/attn_pmc.py), or null."""
    import ctypes as C

    from zonos_amd import _lib
    from zonos_amd._lib import call, ptr
    ws = eng._ws
    c = eng.cfg
    R, Hk, hd, H = ws["R"], c.n_kv, c.head_dim, c.n_heads
    gs = ws["splits"]["qkv"]
    kc, vt = eng._kv(ws, c.n_layer // 2)
    stream = _lib.stream_ptr()
    e0, e1 = _lib.P(), _lib.P()
    call("zk_event_create", C.byref(e0))
    call("zk_event_create", C.byref(e1))
    args = (ptr(ws["part"]), gs, ptr(eng.freqs), ptr(kc), ptr(vt), R, H, Hk, hd, ws["smax"], ctx, None,
            ptr(ws["attn_work"]), ws["attn_splits"], ptr(ws["y"]), 0, None, stream)
    for _ in range(5):
        call("zk_attn_decode_qkv", *args)
    call("zk_event_record", e0.value, stream)
    for _ in range(reps):
        call("zk_attn_decode_qkv", *args)
    call("zk_event_record", e1.value, stream)
    ms = C.c_float()
    call("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
    call("zk_event_destroy", e0.value)
    call("zk_event_destroy", e1.value)
    per_launch_s = ms.value / 1e3 / reps
    Nq = (H + 2 * Hk) * hd
    bytes_per_launch = R * ctx * Hk * hd * 2 * 2 + gs * R * Nq * 4 + R * H * hd * 2 + R * Hk * hd * 2 * 2
    ach = bytes_per_launch / per_launch_s / 1e9
    traffic = None
    import glob
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*attn*pmc*.json"))):
        d = json.load(open(f))
        if d.get("R") == R and d.get("ctx") == ctx and d.get("kernel") == "k_attn_decode<true>":
            traffic = d["hbm_bytes_per_launch"]
    return dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                traffic=traffic, kernel="k_attn_decode<true> (zk_attn_decode_qkv)" +
                ("+k_attn_combine" if ws["attn_splits"] > 1 else ""),
                ctx=ctx, attn_splits=ws["attn_splits"],
                bytes_per_launch=bytes_per_launch, us_per_launch=round(per_launch_s * 1e6, 2))


def mamba_roofline(eng, reps=50):
    """Hybrid: time zk_mamba_step (the SSM state update, HBM-bound) of one Mamba layer with HIP
    events; algorithmic bytes = SSM state read + write (R*d_inner*d_state*2 B each) + conv
    state read + write + in_proj slabs read + yz write."""
    import ctypes as C

    from zonos_amd import _lib
    from zonos_amd._lib import call, ptr
    ws, c = eng._ws, eng.cfg
    R = ws["R"]
    j = len(eng.mamba_ids) // 2
    L = eng.layers[eng.mamba_ids[j]]
    stream = _lib.stream_ptr()
    e0, e1 = _lib.P(), _lib.P()
    call("zk_event_create", C.byref(e0))
    call("zk_event_create", C.byref(e1))
    gs = ws["splits"]["inp"]
    args = (ptr(ws["part"]), gs, R, c.d_inner, c.nheads_ssm, c.headdim, c.d_state, ptr(L["conv_w"]),
            ptr(L["conv_b"]), ptr(ws["conv"][j][0]), ptr(ws["conv"][j][1]), ptr(ws["scal"][1:2]), ptr(ws["ssm"][j]),
            ptr(L["A"]), ptr(L["dt_bias"]), ptr(L["D"]), ptr(ws["yz"]), None, stream)
    for _ in range(5):
        call("zk_mamba_step", *args)
    call("zk_event_record", e0.value, stream)
    for _ in range(reps):
        call("zk_mamba_step", *args)
    call("zk_event_record", e1.value, stream)
    ms = C.c_float()
    call("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
    call("zk_event_destroy", e0.value)
    call("zk_event_destroy", e1.value)
    per = ms.value / 1e3 / reps
    b = (R * c.d_inner * c.d_state * 2 * 2 + R * c.conv_dim * 8 * 2 + gs * R * c.d_in_proj * 4 + R * c.d_inner * 4)
    ach = b / per / 1e9
    return dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                traffic=None, kernel="k_mamba_step", bytes_per_launch=b, us_per_launch=round(per * 1e6, 2))


def cpu_baseline(args):
    """Oracle (CPU restatement, validated against the reference) timed on this host: decode
    steps at B=64 at 3 context lengths (KV cache pre-filled) + a 43-frame DAC decode; scaled
    to codes/s of the same workload (prefill excluded, <1% of the GPU time)."""
    from oracle import dac_ref, zonos_ref
    cores = os.cpu_count() or 1
    threads = min(cores, 64)
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
                sample=f"oracle decode step B={B} at ctx {ctx0 + int(0.1 * N)}/{ctx0 + int(0.5 * N)}/"
                       f"{ctx0 + int(0.9 * N)} x{args.cpu_sample_steps} (mean {step_s:.3f} s/step) + DAC 43 frames "
                       f"({dac_s_per_frame * 1e3:.1f} ms/frame); scaled to {N} steps + {B * args.new_tokens} frames; "
                       f"{time.time() - t_begin - t_setup:.1f} s of timed CPU work (+{t_setup:.1f} s setup)",
                step_s=round(step_s, 4), dac_ms_per_frame=round(dac_s_per_frame * 1e3, 2))


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from zonos_amd import synthetic
    from zonos_amd.autoencoder import DacSpec, HipDacDecoder
    from zonos_amd.engine import EngineConfig, HipDecoder

    if args.model == "hybrid":
        from zonos_amd.hybrid import HybridDecoder, HybridEngineConfig
        mc = dict(synthetic.ZONOS_V01_HYBRID)
        if args.layers:
            mc["n_layer"] = args.layers
            mc["attn_layer_idx"] = tuple(i for i in mc["attn_layer_idx"] if i < args.layers)
        W = synthetic.hybrid_weights(dev, seed=0, **mc)
        eng = HybridDecoder(HybridEngineConfig(**mc), W, dev)
    else:
        mc = dict(synthetic.ZONOS_V01, n_layer=args.layers or 26)
        W = synthetic.backbone_weights(dev, seed=0, **mc)
        eng = HipDecoder(EngineConfig(**mc), W, dev)
    del W
    dac = None if args.no_dac else HipDacDecoder(DacSpec(), synthetic.dac_weights(dev), dev)
    B = args.batch
    cond = synthetic.conditioning(B, args.lc, mc["d_model"], seed=1 + rank, device=dev)
    prefix = synthetic.prefix_codes(B, args.prefix, seed=3 + rank, device=dev) if args.prefix else None
    sp = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
              repetition_penalty_window=8, temperature=1.0)
    stats = {"gen_s": 0.0, "dac_s": 0.0}

    def step(i, timed):
        t0 = time.time()
        codes = eng.generate(cond, prefix, args.new_tokens, 2.0, B, sp, seed=1000 + i, row_base=rank * B,
                             force_full_length=True, poll_every=64)
        torch.cuda.synchronize(dev)
        t1 = time.time()
        if dac is not None:
            dac.decode_list(codes)
        torch.cuda.synchronize(dev)
        t2 = time.time()
        if dist is not None:
            from zonos_amd.distributed import gather_codes
            gather_codes(codes, device=dev)
        if timed:
            stats["gen_s"] += t1 - t0
            stats["dac_s"] += t2 - t1
        return sum(int(c.shape[1]) for c in codes)

    for i in range(args.warmup):
        step(i, False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.time()
    frames = 0
    for i in range(args.steps):
        frames += step(args.warmup + i, True)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        fr = torch.tensor([frames], device=dev, dtype=torch.float64)
        dist.all_reduce(fr)
        frames = int(fr.item())

    if rank == 0:
        codes_s = frames * 9 / elapsed
        audio_s = frames / FRAME_RATE
        ctx_mean = args.lc + args.prefix + 1 + (args.new_tokens + 8) // 2
        roof = attn_roofline(eng, ctx_mean) if args.model == "transformer" else mamba_roofline(eng)
        model = "Zonos-v0.1-transformer" if args.model == "transformer" else "Zonos-v0.1-hybrid (assumed geometry)"
        cfg_name = {(64, 400, 10, 2580): "c3", (1, 160, 0, 861): "c2"}.get(
            (args.batch, args.lc, args.prefix, args.new_tokens), "custom")
        if args.model == "hybrid" and cfg_name == "c3":
            cfg_name = "c5"
        workload = (f"{cfg_name}: B={B}/GPU, Lc={args.lc}, prefix {args.prefix}, {args.new_tokens} new tokens "
                    f"({args.new_tokens / FRAME_RATE:.0f} s), EOS disabled, CLI sampling (linear .65 conf .4 rep "
                    f"2.5/8), DAC decode of all codes")
        out = {
            "metric": f"DAC codes/sec (end-to-end generate + DAC decode), {model} batch={B}/GPU",
            "value": round(codes_s, 1), "unit": "codes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded random weights + LayerNorm'd random conditioning; no checkpoint offline)",
            "config": {"workload": workload, "model": model, "global_batch": B * world,
                       "seq_len": args.lc + args.prefix + args.new_tokens + 9, "parallelism": f"dp{world}"},
            "rtf": round(audio_s / elapsed, 2),
            "breakdown": {"generate_s_per_step": round(stats["gen_s"] / args.steps, 3),
                          "dac_s_per_step": round(stats["dac_s"] / args.steps, 3),
                          "dac_precision": dac.precision if dac is not None else None,
                          "generate_codes_s": round(frames / world * 9 / max(stats["gen_s"], 1e-9) * world, 1),
                          "decode_ms_per_token_step": round(stats["gen_s"] / args.steps / (args.new_tokens + 8) * 1e3,
                                                            3)},
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1 and args.model == "transformer":
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
