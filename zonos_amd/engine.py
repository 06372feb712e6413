"""The MI355X decode engine: Zonos.generate()'s hot loop on hand-written HIP kernels.

Restates zonos/model.py:224-457 (generate) with the transformer backbone of
zonos/backbone/_torch.py, the heads/CFG of model.py:100-116, the sampler of
zonos/sampling.py and the delay pattern of zonos/codebook_pattern.py.

Design (MI355X-first):
  * All per-step state (offset, position, EOS protocol, repetition penalty, delayed
    codes) lives on the device; one decode step = a fixed launch sequence with no host
    synchronisation, captured once into a hipGraph and replayed in chunks of
    `poll_every` steps. The host polls a `done` word between chunks; steps after
    completion are no-ops (every kernel checks the word).
  * Weights are bf16 in HBM in the engine's layouts: 9 embedding tables stacked
    [9][1026][D], the 9 heads stacked [9*1026][D], fc1 rows interleaved for the fused
    SwiGLU epilogue, GEMM weights fragment-packed (zk_pack_weights). The KV cache stores
    per (row, kv head) 32-key slices in MFMA-fragment order (zonos_amd.kvlayout).
  * torch is plumbing only: it allocates device memory and provides the stream.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass

import torch

from . import _lib
from . import sampling as zsampling
from ._lib import GenState, SamplingParams, call, ptr

EOS, MASK, UNKNOWN = 1024, 1025, -1
N_CB = 9
VOCAB = 1026
ATTN_CHUNK = 256


@dataclass
class EngineConfig:
    d_model: int
    n_layer: int
    n_heads: int
    n_kv: int
    d_ff: int
    eps: float = 1e-5

    @property
    def head_dim(self):
        return self.d_model // self.n_heads

    @classmethod
    def from_backbone_config(cls, bc) -> "EngineConfig":
        return cls(d_model=bc.d_model, n_layer=bc.n_layer, n_heads=bc.attn_cfg["num_heads"],
                   n_kv=bc.attn_cfg["num_heads_kv"], d_ff=bc.attn_mlp_d_intermediate, eps=bc.norm_epsilon)


def rope_table(seq_len: int, head_dim: int, base: float = 10000.0) -> torch.Tensor:
    """precompute_freqs_cis (_torch.py:9-15), computed on the host CPU exactly as the
    reference does, then uploaded: [seq_len][hd/2][2] fp32 (cos, sin)."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2)[: head_dim // 2].float() / head_dim))
    ang = torch.outer(torch.arange(seq_len, device=inv.device), inv)
    z = torch.polar(torch.ones_like(ang), ang)
    return torch.stack([z.real, z.imag], dim=-1).contiguous()


def pack_weights(w: torch.Tensor, stream) -> torch.Tensor:
    """nn.Linear bf16 [N][K] -> the GEMM's fragment-packed layout (zk_pack_weights)."""
    N, K = w.shape
    out = torch.empty((N + 63) // 64 * 64, K, dtype=w.dtype, device=w.device)
    call("zk_pack_weights", ptr(w), N, K, ptr(out), stream)
    return out


def _split_for(N: int, K: int, M: int, target_blocks: int = 256) -> int:
    """Split-K count for the 128x64-tile GEMM: enough workgroups to cover the CUs.
    Depends on (N, K) only for M <= 128 so the reduction order is batch-invariant."""
    if M > 128:
        return 1
    tiles = (N + 63) // 64
    want = max(1, math.ceil(target_blocks / tiles))
    s = 1
    for cand in range(1, want + 1):
        if K % (cand * 64) == 0:
            s = cand
    return s


def attn_splits_for(R: int, Hkv: int, smax: int, target_blocks: int = 512) -> int:
    """Workgroups per (row, kv head) for flash-decoding. Measured at R=128 (B=64): one
    workgroup per (row, kv head) (512 workgroups, no combine pass) reads 5.4-5.7 TB/s at
    ctx 1.7-3k vs 4.5-4.7 with 2 splits. Small batches split the keys to fill the CUs, but
    each split must cover >= 2048 keys of the cache: the combine launch costs ~6 us, more than
    it saves below that (B=1, 10 s: 1.294 ms per decode step unsplit vs 1.353 with 10 splits,
    tools/c2_attn_ab.sh)."""
    want = -(-target_blocks // (R * Hkv))
    cap = max(1, -(-smax // 2048))
    return max(1, min(want, cap, smax // 128))


def attn_merge_for(R: int, smax: int) -> int:
    """B = 1 (R = 2 rows): key splits of the decode attention whose partials the out_proj GEMV
    merges in its prologue (zk_attn_decode_q_part + zk_gemv_attn_out) -- more CUs stream the
    small KV cache without a combine launch or in-launch tickets. 0 = unsplit attention. The
    splits take 32-key slices in turn (4 waves per split), so any count covers any context."""
    if R > 2:
        return 0
    for v in (16, 8, 4, 2):
        if ATTN_MERGE_DEFAULT >= v and smax >= 128:
            return v
    return 0


# c2 (B=1, Lc=160, 861 tokens) decode step: 1.13 ms unsplit, 1.09 / 1.07 / 1.085 ms with 2 / 4 / 8
# merged splits (profiles/r2_s4_attn_merge_ab.txt)
ATTN_MERGE_DEFAULT = 4


class HipBackbone:
    """The 26 transformer blocks + final LayerNorm on the device (zonos/backbone/_torch.py:52-152):
    bf16 weights in the engine's layouts and the layer launch sequence. Shared by the generate()
    engine (HipDecoder) and the backbone plugin (zonos_amd.backbone.HipZonosBackbone)."""

    def __init__(self, cfg: EngineConfig, weights: dict, device="cuda", prefix: str = "backbone."):
        _lib.load()
        self.cfg = cfg
        self.fuse_qkv = True      # in_proj epilogue inside the decode attention launch (False: separate kernel)
        self.rope_neox = 0        # transformer: interleaved RoPE pairs (_torch.py:18-30)
        self.device = torch.device(device)
        c = cfg
        bf = torch.bfloat16
        dev = self.device

        def w(name):
            t = weights[prefix + name]
            return t.to(device=dev, dtype=bf).contiguous()

        stream = _lib.stream_ptr(dev)
        self.layers = []
        for i in range(c.n_layer):
            p = f"layers.{i}."
            fc1 = w(p + "mlp.fc1.weight")
            fc1p = torch.empty_like(fc1)
            call("zk_permute_fc1", ptr(fc1), c.d_ff, c.d_model, ptr(fc1p), stream)
            del fc1
            self.layers.append(dict(
                ln1_w=w(p + "norm.weight"), ln1_b=w(p + "norm.bias"),
                wqkv=pack_weights(w(p + "mixer.in_proj.weight"), stream),
                wo=pack_weights(w(p + "mixer.out_proj.weight"), stream),
                ln2_w=w(p + "norm2.weight"), ln2_b=w(p + "norm2.bias"),
                fc1=pack_weights(fc1p, stream), fc2=pack_weights(w(p + "mlp.fc2.weight"), stream)))
        self.lnf_w = w("norm_f.weight")
        self.lnf_b = w("norm_f.bias")
        self.freqs = rope_table(16384, c.head_dim).to(dev)

    def _layers_small(self, ws, R: int, stream, skip):
        """Decode step of the 26 blocks for R <= 16 rows (B <= 8), five launches per block:
        [norm -> in_proj] -> attention (RoPE, KV write) -> [out_proj -> x += .] ->
        [norm2 -> fc1 -> SwiGLU] -> [fc2 -> x += .] (_torch.py:99-102, 117-152). Leaves the
        residual stream in ws['x'] (norm_f runs in the heads GEMV's prologue)."""
        c = self.cfg
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        Nqkv = (H + 2 * Hk) * hd
        x, y, h, part, scal = ws["x"], ws["y"], ws["h"], ws["part"], ws["scal"]
        merge = ws.get("attn_merge", 0)
        for i, L in enumerate(self.layers):
            kc, vt = self._kv(ws, i)
            if merge and not self.rope_neox:
                # B = 1: RoPE + KV write in the in_proj epilogue (q -> y), prologue-free attention over
                # 32-key slices, partials merged by the out_proj GEMV
                call("zk_gemv_qkv_rope", ptr(x), ptr(L["wqkv"]), R, H, Hk, hd, ptr(L["ln1_w"]), ptr(L["ln1_b"]),
                     c.eps, ptr(y), ptr(kc), ptr(vt), ws["smax"], ptr(scal[1:2]), ptr(self.freqs), skip, stream)
                call("zk_attn_decode_q_part", ptr(y), ptr(kc), ptr(vt), R, H, Hk, hd, ws["smax"], 1, ptr(scal[1:2]),
                     ptr(ws["attn_work"]), merge, skip, stream)
                call("zk_gemv_attn_out", ptr(ws["attn_work"]), merge, Hk, ptr(L["wo"]), R, D, H * hd, ptr(x), skip,
                     stream)
                call("zk_gemv_fused", ptr(x), D, ptr(L["fc1"]), R, 2 * Fd, D, 1, ptr(L["ln2_w"]), ptr(L["ln2_b"]),
                     c.eps, None, ptr(h), skip, stream)
                call("zk_gemv_fused", ptr(h), Fd, ptr(L["fc2"]), R, D, Fd, 2, None, None, c.eps, None, ptr(x), skip,
                     stream)
                continue
            call("zk_gemv_fused", ptr(x), D, ptr(L["wqkv"]), R, Nqkv, D, 0, ptr(L["ln1_w"]), ptr(L["ln1_b"]), c.eps,
                 ptr(part), None, skip, stream)
            if merge:
                call("zk_attn_decode_qkv_part", ptr(part), 1, ptr(self.freqs), ptr(kc), ptr(vt), R, H, Hk, hd,
                     ws["smax"], 1, ptr(scal[1:2]), ptr(ws["attn_work"]), merge, self.rope_neox, skip, stream)
                call("zk_gemv_attn_out", ptr(ws["attn_work"]), merge, Hk, ptr(L["wo"]), R, D, H * hd, ptr(x), skip,
                     stream)
            else:
                call("zk_attn_decode_qkv_sc", ptr(part), 1, ptr(self.freqs), ptr(kc), ptr(vt), R, H, Hk, hd,
                     ws["smax"], 1, ptr(scal[1:2]), ptr(ws["attn_work"]), ws["attn_splits"], ptr(ws["attn_cnt"]),
                     ptr(y), self.rope_neox, skip, stream)
                call("zk_gemv_fused", ptr(y), H * hd, ptr(L["wo"]), R, D, H * hd, 2, None, None, c.eps, None,
                     ptr(x), skip, stream)
            call("zk_gemv_fused", ptr(x), D, ptr(L["fc1"]), R, 2 * Fd, D, 1, ptr(L["ln2_w"]), ptr(L["ln2_b"]),
                 c.eps, None, ptr(h), skip, stream)
            call("zk_gemv_fused", ptr(h), Fd, ptr(L["fc2"]), R, D, Fd, 2, None, None, c.eps, None, ptr(x), skip,
                 stream)

    def _kv(self, ws, layer):
        if "kv_layers" in ws:            # caches handed out per layer (backbone plugin)
            kv = ws["kv_layers"][layer]
            return kv[0], kv[1]
        return ws["kv"][layer, 0], ws["kv"][layer, 1]

    # ------------------------------------------------------------------ transformer passes
    def _layers(self, ws, M: int, R: int, S: int, prefill: bool, stream, skip):
        """Run the 26 blocks on xn/x (rows = R*S). Leaves norm_f(x) in ws['xn']."""
        c = self.cfg
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        Nqkv = (H + 2 * Hk) * hd
        sp = ws["splits"] if not prefill else dict(qkv=1, o=1, fc2=1)
        x, xn, q, y, h, part = ws["x"], ws["xn"], ws["q"], ws["y"], ws["h"], ws["part"]
        scal = ws["scal"]
        pos_dev = None if prefill else ptr(scal[1:2])
        for i, L in enumerate(self.layers):
            kc, vt = self._kv(ws, i)
            call("zk_gemm_bf16", ptr(xn), D, ptr(L["wqkv"]), M, Nqkv, D, sp["qkv"], 0, ptr(part), None, skip, stream)
            if prefill:
                call("zk_qkv_rope", ptr(part), sp["qkv"], R, S, H, Hk, hd, ptr(self.freqs), 0, pos_dev, ptr(q),
                     ptr(kc), ptr(vt), ws["smax"], None, self.rope_neox, skip, stream)
                call("zk_attn_prefill", ptr(q), ptr(kc), ptr(vt), R, S, H, Hk, hd, ws["smax"], ptr(y), stream)
            elif self.fuse_qkv:
                # in_proj epilogue fused into the attention launch (position = ctx - 1 = scal[1])
                # split partials (long contexts at small batch) merged inside the launch
                call("zk_attn_decode_qkv_sc", ptr(part), sp["qkv"], ptr(self.freqs), ptr(kc), ptr(vt), R, H, Hk, hd,
                     ws["smax"], 1, ptr(scal[1:2]), ptr(ws["attn_work"]), ws["attn_splits"],
                     ptr(ws["attn_cnt"]) if "attn_cnt" in ws else None, ptr(y), self.rope_neox, skip, stream)
            else:
                call("zk_qkv_rope", ptr(part), sp["qkv"], R, S, H, Hk, hd, ptr(self.freqs), 0, pos_dev, ptr(q),
                     ptr(kc), ptr(vt), ws["smax"], None, self.rope_neox, skip, stream)
                call("zk_attn_decode", ptr(q), ptr(kc), ptr(vt), R, H, Hk, hd, ws["smax"], 1, ptr(scal[1:2]),
                     ptr(ws["attn_work"]), ws["attn_splits"], ptr(y), skip, stream)
            call("zk_gemm_bf16", ptr(y), H * hd, ptr(L["wo"]), M, D, H * hd, sp["o"], 0, ptr(part), None, skip, stream)
            call("zk_resid_ln", ptr(part), sp["o"], ptr(x), ptr(L["ln2_w"]), ptr(L["ln2_b"]), c.eps, M, D, ptr(x),
                 ptr(xn), 0, skip, stream)
            call("zk_gemm_bf16", ptr(xn), D, ptr(L["fc1"]), M, 2 * Fd, D, 1, 1, None, ptr(h), skip, stream)
            call("zk_gemm_bf16", ptr(h), Fd, ptr(L["fc2"]), M, D, Fd, sp["fc2"], 0, ptr(part), None, skip, stream)
            if i + 1 < len(self.layers):
                nw, nb = self.layers[i + 1]["ln1_w"], self.layers[i + 1]["ln1_b"]
            else:
                nw, nb = self.lnf_w, self.lnf_b
            call("zk_resid_ln", ptr(part), sp["fc2"], ptr(x), ptr(nw), ptr(nb), c.eps, M, D, ptr(x), ptr(xn), 0, skip,
                 stream)


class HipDecoder(HipBackbone):
    """Owns device weights in engine layout and runs generate() on the GPU."""

    # B <= 8 decode (R <= 16 rows) runs each block as five launches (zk_gemv_fused: LayerNorm
    # prologues, residual epilogues, no split-K slabs) instead of seven
    small_batch_path = True
    graph_steps = 1                 # decode steps captured per hipGraph replay (generate's G; 8 measured no faster)
    # layer 0's norm is fused into the embedding kernel (decode) / a zk_layernorm (prefill); False:
    # the subclass runs it as _prenorm (the hybrid backbone's RMS-norm / fp32-residual variants)
    embed_norm = True

    def __init__(self, cfg: EngineConfig, weights: dict, device="cuda"):
        super().__init__(cfg, weights, device)
        c = cfg
        dev = self.device

        def w(name):
            return weights[name].to(device=dev, dtype=torch.bfloat16).contiguous()

        self.emb = torch.stack([w(f"embeddings.{k}.weight") for k in range(N_CB)]).contiguous()
        assert self.emb.shape == (N_CB, VOCAB, c.d_model), self.emb.shape
        heads = []
        for k in range(N_CB):
            h = w(f"heads.{k}.weight")
            if h.shape[0] < VOCAB:      # pad_weight_ (utils.py:22-37): 1025 -> 1026 rows
                h = torch.cat([h, h.new_zeros(VOCAB - h.shape[0], h.shape[1])])
            heads.append(h)
        self.heads = pack_weights(torch.cat(heads).contiguous(), _lib.stream_ptr(dev))  # [9*1026 -> 9280][D] packed
        self._ws = None
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------ workspace
    def _alloc(self, B: int, Lc: int, P: int, max_new: int):
        c = self.cfg
        dev = self.device
        R = 2 * B
        T = P + max_new
        Ld = T + N_CB
        seq_len = Lc + T + N_CB
        smax = -(-seq_len // ATTN_CHUNK) * ATTN_CHUNK
        S_pre = Lc + P + 1
        key = (B, Lc, P, max_new)
        if self._ws is not None and self._ws["key"] == key:
            ws = self._ws
            ws["kv"].zero_()
            ws["attn_cnt"].zero_()
            return ws
        self.release()
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        Nqkv = (H + 2 * Hk) * hd
        Nh = N_CB * VOCAB
        Mp = R * S_pre
        f32, bf, i32 = torch.float32, torch.bfloat16, torch.int32
        # heads: no split-K (145 workgroups of 64 columns stream 37.8 MB in 15.6 us vs 19.8 us
        # with 2 splits, tools/microbench.py gemm; the sampler then reads one slab)
        # out_proj: 4-way split-K (128 workgroups) is as fast as 8-way (6.6 vs 6.5 us) and halves
        # the fp32 slabs it writes and k_resid_ln reads (4.2 vs 8.4 MB; resid_ln 4.3 vs 4.8 us)
        splits = dict(qkv=_split_for(Nqkv, D, R), o=_split_for(D, H * hd, R, target_blocks=128),
                      fc2=_split_for(D, Fd, R), heads=1)
        part_n = max(Mp * Nqkv, Mp * D, splits["qkv"] * R * Nqkv, splits["o"] * R * D, splits["fc2"] * R * D,
                     splits["heads"] * R * Nh)
        attn_splits = attn_splits_for(R, Hk, smax)
        attn_merge = attn_merge_for(R, smax)
        ws = dict(
            key=key, R=R, T=T, Ld=Ld, smax=smax, S_pre=S_pre, splits=splits, attn_splits=attn_splits,
            attn_merge=attn_merge,
            kv=torch.zeros(c.n_layer, 2, R * Hk * smax * hd, dtype=bf, device=dev),
            x=torch.empty(Mp, D, dtype=bf, device=dev), xn=torch.empty(Mp, D, dtype=bf, device=dev),
            q=torch.empty(Mp, H * hd, dtype=bf, device=dev), y=torch.empty(Mp, H * hd, dtype=bf, device=dev),
            h=torch.empty(Mp, Fd, dtype=bf, device=dev), part=torch.empty(part_n, dtype=f32, device=dev),
            attn_work=torch.empty(max(1, R * Hk * max(attn_splits, attn_merge) * (8 + 4 * hd)), dtype=f32,
                                  device=dev),
            attn_cnt=torch.zeros(R * Hk, dtype=i32, device=dev),     # in-launch split-combine tickets
            scal=torch.zeros(16, dtype=i32, device=dev),
            eos_mode=torch.zeros(B, dtype=i32, device=dev), steps_after=torch.zeros(B, dtype=i32, device=dev),
            remaining=torch.zeros(B, dtype=i32, device=dev), stopping=torch.zeros(B, dtype=i32, device=dev),
            act=torch.zeros(B, dtype=i32, device=dev), rp=torch.ones(B, dtype=f32, device=dev),
            tok0=torch.zeros(B * N_CB, dtype=i32, device=dev), tok1=torch.zeros(B * N_CB, dtype=i32, device=dev),
            delayed=torch.empty(B, N_CB, Ld, dtype=torch.int64, device=dev),
            dbg=torch.empty(B, N_CB, VOCAB, dtype=f32, device=dev),
            graph=None,
        )
        self._ws = ws
        return ws

    def release(self):
        if self._ws is not None and self._ws.get("graph"):
            call("zk_graph_destroy", self._ws["graph"])
        self._ws = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def _heads(self, ws, R: int, S: int, stream, skip):
        """Heads GEMM on the last position of every row -> split-K slabs in ws['part']."""
        D = self.cfg.d_model
        last = ws["xn"][S - 1:]           # rows r*S + S-1 via lda = S*D
        call("zk_gemm_bf16", ptr(last), S * D, ptr(self.heads), R, N_CB * VOCAB, D, ws["splits"]["heads"], 0,
             ptr(ws["part"]), None, skip, stream)

    def _gen_state(self, ws, B, seed, row_base, noise=(0, 0, 0, 0)) -> GenState:
        """noise = (mode, Philox offset, grid-stride, offset per call): zk_gen_state's noise words."""
        return GenState(ptr(ws["scal"]), ptr(ws["eos_mode"]), ptr(ws["steps_after"]), ptr(ws["remaining"]),
                        ptr(ws["stopping"]), ptr(ws["act"]), ptr(ws["rp"]), ptr(ws["tok0"]), ptr(ws["tok1"]),
                        ptr(ws["delayed"]), B, N_CB, ws["Ld"], VOCAB, seed & 0xFFFFFFFFFFFFFFFF, row_base, *noise)

    # the step's launch sequence is enqueued by the C ABI (zk_decode_step); False runs the same
    # sequence from Python (bit-identical; kept as the reference for the test)
    c_step = True

    def _step_desc(self, ws, B, st, sp):
        """zk_step_desc of this workspace: per-layer weights + KV caches, buffers, state, params."""
        c = self.cfg
        if "step_layers" not in ws:
            arr = (_lib.StepLayer * c.n_layer)()
            for i, L in enumerate(self.layers):
                kc, vt = self._kv(ws, i)
                arr[i] = _lib.StepLayer(ptr(L["ln1_w"]), ptr(L["ln1_b"]), ptr(L["wqkv"]), ptr(L["wo"]),
                                        ptr(L["ln2_w"]), ptr(L["ln2_b"]), ptr(L["fc1"]), ptr(L["fc2"]), ptr(kc), ptr(vt))
            ws["step_layers"] = arr
        sps = ws["splits"]
        return _lib.StepDesc(B, c.n_layer, c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff, ws["smax"],
                             sps["qkv"], sps["o"], sps["fc2"], sps["heads"], ws["attn_splits"],
                             ws.get("attn_merge", 0), self.rope_neox, int(self._small(2 * B)), c.eps,
                             C.cast(ws["step_layers"], C.c_void_p), ptr(self.emb), ptr(self.heads), ptr(self.lnf_w),
                             ptr(self.lnf_b), ptr(self.freqs), ptr(ws["x"]), ptr(ws["xn"]), ptr(ws["y"]), ptr(ws["h"]),
                             ptr(ws["part"]), ptr(ws["attn_work"]), ptr(ws["attn_cnt"]), ptr(ws["dbg"]), st, sp)

    def _c_decode(self, ws, B, st, sp, stream):
        call("zk_decode_step", C.byref(self._step_desc(ws, B, st, sp)), stream)

    def _c_prefill(self, ws, B, st, sp, cond, Lc, P, stream):
        call("zk_prefill", C.byref(self._step_desc(ws, B, st, sp)), ptr(cond), Lc, P, ptr(ws["q"]), stream)

    def _decode_step(self, ws, B, st, sp, stream):
        c = self.cfg
        R = 2 * B
        if self.c_step:
            self._c_decode(ws, B, st, sp, stream)
            return
        scal = ws["scal"]
        skip = ptr(scal[3:4])
        L0 = self.layers[0]
        small = self._small(R)                       # layer 0's LayerNorm runs in the in_proj prologue
        own = small or not self.embed_norm           # ... or its own launch (hybrid config variants)
        call("zk_embed_codes", ptr(ws["delayed"]), B, 1, N_CB, ws["Ld"] * N_CB, ws["Ld"], ptr(scal[0:1]), -1,
             ptr(self.emb), VOCAB, c.d_model, 2, ptr(ws["x"]), 1, 0, None if own else ptr(L0["ln1_w"]),
             None if own else ptr(L0["ln1_b"]), c.eps, None if own else ptr(ws["xn"]), skip, stream)
        if not self.embed_norm:
            self._prenorm(ws, R, stream, skip)
        logits, nsp = ws["part"], ws["splits"]["heads"]
        if small:
            self._layers_small(ws, R, stream, skip)
            # heads with the final LayerNorm (norm_f) as the GEMV prologue: one fp32 slab
            call("zk_gemv_fused", ptr(ws["x"]), c.d_model, ptr(self.heads), R, N_CB * VOCAB, c.d_model, 0,
                 ptr(self.lnf_w), ptr(self.lnf_b), c.eps, ptr(ws["part"]), None, skip, stream)
        else:
            self._layers(ws, R, R, 1, False, stream, skip)
            self._heads(ws, R, 1, stream, skip)
        call("zk_sample_heads", ptr(logits), nsp, C_ref(st), C_ref(sp), 0, 0, ptr(ws["dbg"]), stream)
        call("zk_sample_heads", ptr(logits), nsp, C_ref(st), C_ref(sp), 0, 1, None, stream)
        call("zk_eos_step", C_ref(st), 0, 0, stream)

    def _small(self, R: int) -> bool:
        return self.small_batch_path and R <= 16 and self.cfg.d_model == 2048

    # ------------------------------------------------------------------ generate
    @torch.inference_mode()
    def generate(self, prefix_conditioning: torch.Tensor, audio_prefix_codes=None, max_new_tokens: int = 86 * 30,
                 cfg_scale: float = 2.0, batch_size: int = 1, sampling_params: dict | None = None,
                 seed: int = 0, row_base: int = 0, force_full_length: bool = False, callback=None,
                 progress=None, poll_every: int = 16, trace: dict | None = None, use_graph: bool = True,
                 _after_prefill=None, noise: str = "keyed", generator: torch.Generator | None = None,
                 pad_rows: int = 0):
        """Zonos.generate (model.py:224-457). Returns the list of int64 [9, T_i] code tensors.

        ``noise`` picks the race noise of the sampler: "keyed" = the engine's stream keyed by
        (seed, step, draw, row_base + b, codebook, token), independent of batch sharding; "torch" =
        torch's own GPU stream, the values the reference's `exponential_` draws from ``generator``
        (default: torch's CUDA generator of the device) -- the generator is read at the start and
        advanced by the Philox offset the reference's sampler calls would have consumed, so
        ``torch.manual_seed(s)`` followed by this call leaves torch's RNG where the reference leaves it.

        ``trace`` (optional dict) receives per-step fp32 CFG logits (before bias) and the
        sampled frames -- test instrumentation, forces one step per poll and no graph.

        ``pad_rows``: the last ``pad_rows`` utterances are padding (generate_sharded's uniform shards)
        whose codes the caller drops. They run through the GEMMs like any row but stay out of the
        batch-wide EOS protocol (model.py:376-393): they start in EOS mode with no hold-off and no
        remaining steps, so an EOS they sample never triggers the resample draw of the real rows and
        never keeps the loop running after the real rows have stopped."""
        assert cfg_scale != 1, "TODO: add support for cfg_scale=1"                     # model.py:247
        if batch_size * 2 != prefix_conditioning.shape[0]:                            # model.py:249-250
            raise ValueError(f"Batch size mismatch: {batch_size} * 2 != {prefix_conditioning.shape[0]}")
        if not 0 <= pad_rows < batch_size:
            raise ValueError(f"pad_rows={pad_rows} must leave at least one real utterance of {batch_size}")
        _lib.require_gpu(prefix_conditioning, "prefix_conditioning")
        if prefix_conditioning.dim() != 3 or prefix_conditioning.shape[2] != self.cfg.d_model:
            # zk_prefill copies rows of Lc * d_model bf16: a wrong width would read out of bounds
            raise ValueError(f"prefix_conditioning must be [2B, Lc, {self.cfg.d_model}], "
                             f"got {tuple(prefix_conditioning.shape)}")
        spd = dict(top_p=0, top_k=0, min_p=0, linear=0.55, conf=0.4, quad=0.0, repetition_penalty=3.0,
                   repetition_penalty_window=2, temperature=1.0)
        spd.update(sampling_params or {})
        c = self.cfg
        B = batch_size
        R = 2 * B
        P = 0 if audio_prefix_codes is None else int(audio_prefix_codes.shape[2])
        Lc = int(prefix_conditioning.shape[1])
        ws = self._alloc(B, Lc, P, max_new_tokens)
        stream = _lib.stream_ptr(self.device)
        T, Ld, S = ws["T"], ws["Ld"], ws["S_pre"]
        D = c.d_model

        # codes -> delayed codes on device (model.py:288-295)
        codes = torch.full((B, N_CB, T), UNKNOWN, dtype=torch.int64, device=self.device)
        if audio_prefix_codes is not None:
            codes[..., :P] = audio_prefix_codes.to(self.device)
        call("zk_delay_apply", ptr(codes), B, N_CB, T, MASK, ptr(ws["delayed"]), stream)

        sp = SamplingParams(float(spd["temperature"]), float(spd["top_p"]), float(spd["min_p"]),
                            float(spd["linear"]), float(spd["conf"]), float(spd["quad"]), int(spd["top_k"]),
                            int(spd["repetition_penalty_window"]), float(cfg_scale), int(force_full_length))
        gen = None
        if noise == "torch":
            if row_base:
                raise ValueError("noise='torch' is one process's stream (row_base must be 0)")
            gen = generator if generator is not None else \
                torch.cuda.default_generators[_lib.device_index(self.device)]
            seed, off0 = int(gen.initial_seed()), int(gen.get_offset())
            stride, incr = zsampling.torch_noise_policy(B * N_CB * VOCAB, self.device)
            st = self._gen_state(ws, B, seed, 0, (1, off0, stride, incr))
        elif noise == "keyed":
            st = self._gen_state(ws, B, seed, row_base)
        else:
            raise ValueError(f"noise must be 'keyed' or 'torch', not {noise!r}")
        ws["scal"].zero_()

        # ---- prefill (model.py:297-319, _prefill 181-202)
        if self.c_step:        # the same sequence enqueued by the C ABI
            condb = ws["cond_keep"] = prefix_conditioning.to(torch.bfloat16).contiguous()   # alive until copied
            self._c_prefill(ws, B, st, sp, condb, Lc, P, stream)
        else:
            x = ws["x"][: R * S].view(R, S, D)
            x[:, :Lc].copy_(prefix_conditioning.to(torch.bfloat16))
            call("zk_embed_codes", ptr(ws["delayed"]), B, P + 1, N_CB, Ld * N_CB, Ld, None, 0, ptr(self.emb), VOCAB,
                 D, 2, ptr(ws["x"]), S, Lc, None, None, c.eps, None, None, stream)
            L0 = self.layers[0]
            if self.embed_norm:
                call("zk_layernorm", ptr(ws["x"]), ptr(L0["ln1_w"]), ptr(L0["ln1_b"]), c.eps, R * S, D,
                     ptr(ws["xn"]), stream)
            else:
                self._prenorm(ws, R * S, stream, None)
            self._layers(ws, R * S, R, S, True, stream, None)
            self._heads(ws, R, S, stream, None)
            call("zk_sample_heads", ptr(ws["part"]), ws["splits"]["heads"], C_ref(st), C_ref(sp), 1, 0,
                 ptr(ws["dbg"]), stream)
            call("zk_eos_step", C_ref(st), 1, P + 1, stream)
        if _after_prefill is not None:      # test hook (teacher forcing of the first frame)
            _after_prefill(ws["delayed"][..., P + 1:P + 2])
        # Debug logging. The sampler statistics need the logits of every step (one step per poll);
        # model.py:381's EOS message on the root logger only needs the steps where a row entered EOS
        # mode, which are recovered at poll boundaries from the eos_mode / steps_after words
        # (`_log_new_eos`), so a root logger at DEBUG level keeps multi-step polls (<= 6 steps, the
        # EOS hold-off, so the detection offset is exact).
        logdbg = zsampling.debug_enabled()
        eosdbg = not logdbg and logging.getLogger().isEnabledFor(logging.DEBUG)
        if zsampling.debug_enabled():       # the reference's sampler statistics (sampling.py:287-322)
            zsampling.log_sampling_stats(
                zsampling.engine_logits_row(ws["dbg"][0, 0], True, False, EOS, force_full_length), spd, None, 1.0, EOS)
        if trace is not None:
            trace.setdefault("logits", []).append(ws["dbg"].clone())
            trace.setdefault("tokens", []).append(ws["tok0"].view(B, N_CB, 1).long().clone())

        # ---- state for the loop (model.py:316-342)
        max_steps = Ld - (P + 1)
        ws["scal"].copy_(torch.tensor([P + 2, S, 1, 0, 0, max_steps] + [0] * 10, dtype=torch.int32))
        ws["eos_mode"].zero_()
        ws["steps_after"].fill_(6)
        ws["remaining"].fill_(max_steps)
        ws["stopping"].zero_()
        ws["act"].zero_()
        ws["rp"].fill_(float(spd["repetition_penalty"]))
        if pad_rows:                        # padding rows: out of the EOS protocol (docstring)
            ws["eos_mode"][B - pad_rows:] = 1
            ws["steps_after"][B - pad_rows:] = 0
            ws["remaining"][B - pad_rows:] = 0

        # ---- decode loop (model.py:345-432)
        per_poll = 1 if (callback is not None or trace is not None or logdbg) else max(1, poll_every)
        if eosdbg:
            per_poll = min(per_poll, 6)
            eos_prev = ws["eos_mode"].cpu()
        graph = None
        # steps per graph replay: a replay boundary leaves the GPU idle for 11-13 us (rocprofv3 kernel
        # trace, profiles/r5_trace_gaps_c{2,3}.txt: the gap before every step's first kernel), a kernel
        # boundary inside the graph ~1 us. G divides the poll length; the steps after the last one are
        # no-ops (every kernel tests the done word), so the final poll may run up to G - 1 of them
        G = max(g for g in range(1, min(self.graph_steps, per_poll) + 1) if per_poll % g == 0)
        if use_graph and trace is None:
            graph = self._capture(ws, B, st, sp, stream, G)
        done_steps = 0
        while True:
            n = min(per_poll, max_steps - done_steps)
            if n <= 0:
                break
            if logdbg:                      # state the step starts from (debug logging only)
                pre = (ws["scal"].cpu(), ws["act"][0].item(), ws["rp"][0].item(), ws["eos_mode"].cpu())
            if graph is not None:
                call("zk_graph_launch", graph, -(-n // G), stream)
            else:
                for _ in range(n):
                    self._decode_step(ws, B, st, sp, stream)
            done_steps += n
            if logdbg:
                self._log_step(ws, spd, pre, force_full_length)
            if trace is not None:
                trace["logits"].append(ws["dbg"].clone())
            scal = ws["scal"].cpu()
            if eosdbg:
                eos_prev = self._log_new_eos(ws, eos_prev, int(scal[0]) - 1)
            if progress is not None:
                progress.update(n)
            if callback is not None:
                off = int(scal[0]) - 1
                frame = ws["delayed"][..., off:off + 1]
                if not callback(frame, done_steps, max_steps):
                    break
            if trace is not None:
                off = int(scal[0]) - 1
                trace["tokens"].append(ws["delayed"][..., off:off + 1].clone())
            if int(scal[3]):
                break
        scal = ws["scal"].cpu()
        offset = int(scal[0]) - 1
        if gen is not None and float(spd["temperature"]) > 0:
            # sampler calls the reference made: the prefill sample, one per loop iteration
            # (scal[2] counts from 1) and one per EOS resample (scal[4]); greedy draws nothing
            gen.set_offset(off0 + (int(scal[2]) + int(scal[4])) * incr)
        if trace is not None:
            trace["delayed"] = ws["delayed"].clone()
            trace["offset"] = offset
        return finalize(ws["delayed"], offset, P, stream)

    def _log_new_eos(self, ws, eos_prev, off_last):
        """model.py:381's message for the rows that entered EOS mode during the last poll.
        A row detected at offset o has had its hold-off counter (6 at detection, model.py:384)
        decremented once per later step (model.py:360-362), so o = off_last - 6 + steps_after
        while the poll is at most 6 steps long."""
        eos1 = ws["eos_mode"].cpu()
        new = ((eos1 != 0) & (eos_prev == 0)).nonzero(as_tuple=True)[0].tolist()
        if new:
            sa = ws["steps_after"].cpu()
            by_off = {}
            for r in new:
                by_off.setdefault(off_last - 6 + int(sa[r]), []).append(r)
            for off in sorted(by_off):
                logging.debug(f"Detected EOS in codebook 0 for samples: {by_off[off]} at offset {off}. "
                              "Resampling with -torch.inf.")
        return eos1

    def _log_step(self, ws, spd, pre, force_full_length):
        """Debug logging of one executed decode step (per_poll = 1): the sampler statistics of
        utterance 0 / codebook 0 on the zonos.sampling loggers and model.py:381's EOS message."""
        scal0, act0, rp0, eos0 = pre
        off = int(scal0[0])                 # the reference's `offset` of this step
        if int(scal0[3]):
            return                          # generation had finished: the step was a no-op
        scal1 = ws["scal"].cpu()
        resampled = int(scal1[4]) > int(scal0[4])
        if resampled:
            eos1 = ws["eos_mode"].cpu()
            rows = ((eos1 != 0) & (eos0 == 0)).nonzero(as_tuple=True)[0].tolist()
            logging.debug(f"Detected EOS in codebook 0 for samples: {rows} at offset {off}. "
                          "Resampling with -torch.inf.")
        if not zsampling.debug_enabled():
            return
        x = zsampling.engine_logits_row(ws["dbg"][0, 0], False, bool(act0), EOS, force_full_length)
        gen = ws["delayed"][0, 0, :off]
        zsampling.log_sampling_stats(x, spd, gen, rp0, EOS)
        if resampled:                       # the second sample_from_logits call (model.py:388)
            if int(ws["eos_mode"][0].item()) and not int(eos0[0]):
                x[EOS] = -math.inf
            zsampling.log_sampling_stats(x, spd, gen, rp0, EOS)

    def last_logits(self) -> torch.Tensor:
        """fp32 CFG logits (before bias) of the last executed step [B][9][1026] (test hook)."""
        return self._ws["dbg"]

    def last_tokens(self) -> torch.Tensor:
        """Sampled tokens (first draw) of the last executed step, int32 [B][9] (test hook; the
        frame may hold the delay pattern's MASK or a prefix code instead, model.py:305-306)."""
        return self._ws["tok0"].view(-1, N_CB)

    def _capture(self, ws, B, st, sp, stream, steps: int = 1):
        if ws.get("graph"):
            call("zk_graph_destroy", ws["graph"])
            ws["graph"] = None
        # capture on a side stream (torch's default stream cannot be captured)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        sp_ = s.cuda_stream
        call("zk_graph_begin", sp_)
        try:
            for _ in range(steps):
                self._decode_step(ws, B, st, sp, sp_)
        finally:
            g = _lib.P()
            call("zk_graph_end", sp_, C.byref(g))
        torch.cuda.current_stream(self.device).wait_stream(s)
        ws["graph"] = g.value
        ws["_keep"] = (st, sp)
        return g.value


import ctypes as C  # noqa: E402


def C_ref(x):
    return C.byref(x)


def finalize(delayed: torch.Tensor, offset: int, P: int, stream) -> list:
    """Output trim (model.py:437-457), on the device."""
    B, K, Ld = delayed.shape
    out = torch.empty(B, K, Ld - K, dtype=torch.int64, device=delayed.device)
    call("zk_delay_revert", ptr(delayed), B, K, Ld, ptr(out), stream)
    eos_pos = (out[:, 0, :] == EOS).int().argmax(dim=-1)
    eos_pos[eos_pos == 0] = out.shape[2]
    out = out[..., : offset - 9]
    out.masked_fill_(out >= 1024, 0)
    eos_pos = eos_pos.tolist()
    return [out[i, :, P:eos_pos[i]].clone() for i in range(out.shape[0])]
