"""Hybrid (Mamba2 + attention) backbone on the MI355X engine: Zonos-v0.1-hybrid
(zonos/backbone/_mamba_ssm.py:9-57 -> mamba_ssm create_block / Block / Mamba2 / MHA / GatedMLP).

Same generate() machinery as the transformer engine (device-side step state, one hipGraph per
decode step, shared embed / heads / sampler / EOS kernels); only the per-layer launch sequence
differs:

  Mamba2 layer : gemm(in_proj, split-K) -> mamba_step (slab reduce, conv update, SSM state
                 update, y * silu(z)) -> gated_rmsnorm -> gemm(out_proj, split-K)
                 -> resid_ln(ln_on_sum: fused add + LayerNorm of the fp32 sum)
  attention    : gemm(Wqkv) -> attn_decode_qkv (GPT-NeoX RoPE, bf16 cos/sin cache)
                 -> gemm(out_proj) -> resid_ln(norm2) -> gemm(fc1, SwiGLU) -> gemm(fc2) -> resid_ln

State: per attention layer the KV cache (fragment order, zonos_amd.kvlayout); per Mamba layer the
conv state (bf16 [R][conv_dim][4], double-buffered by step parity) and the SSM state (bf16
[R][nheads][headdim][d_state], as Zonos allocates the inference cache in bf16, model.py:204-208).
Prefill runs the causal conv over the prefix and the exact recurrence (zk_mamba_prefill).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import call, ptr
from .engine import ATTN_CHUNK, N_CB, VOCAB, HipDecoder, _split_for, attn_splits_for, pack_weights

# split-K of the Mamba in_proj GEMM at decode (k_mamba_step reads the slabs: 1, 2 or 4); unsplit is fastest, again in
# round 6 after the step-word change: 4.263-4.280 / 4.316-4.317 / 4.585-4.586 ms (profiles/r6_c5_inp_split_ab.txt)
MAMBA_INP_SPLIT = 1


@dataclass
class HybridEngineConfig:
    d_model: int
    n_layer: int
    attn_layer_idx: tuple
    n_heads: int
    n_kv: int
    d_ff: int
    d_state: int = 128
    d_conv: int = 4
    expand: int = 2
    headdim: int = 64
    ngroups: int = 1
    rotary_base: float = 10000.0
    eps: float = 1e-5
    d_mlp: int = 0                   # GatedMLP width of the Mamba2 blocks (BackboneConfig.d_intermediate; 0: none)
    rms_norm: bool = False           # block norms RMSNorm (bias-free), norm_f an RMS norm (with its bias)
    residual_in_fp32: bool = False   # residual stream kept in fp32

    @property
    def norm_flags(self) -> int:
        """zk_hybrid_desc.norm_flags: bit 1 rms_norm, bit 2 residual_in_fp32."""
        return (2 if self.rms_norm else 0) | (4 if self.residual_in_fp32 else 0)

    @property
    def resid_flags(self) -> int:
        """zk_resid_ln flag word of every block-boundary add + norm (include/zonos_hip.h)."""
        return 1 | (2 if self.rms_norm else 0) | (12 if self.residual_in_fp32 else 0)

    @property
    def head_dim(self):
        return self.d_model // self.n_heads

    @property
    def d_inner(self):
        return self.expand * self.d_model

    @property
    def nheads_ssm(self):
        return self.d_inner // self.headdim

    @property
    def conv_dim(self):
        return self.d_inner + 2 * self.ngroups * self.d_state

    @property
    def d_in_proj(self):
        return 2 * self.d_inner + 2 * self.ngroups * self.d_state + self.nheads_ssm

    @classmethod
    def from_backbone_config(cls, bc) -> "HybridEngineConfig":
        """zonos.config.BackboneConfig of a hybrid checkpoint (mamba_ssm create_block arguments)."""
        a, s = dict(bc.attn_cfg or {}), dict(bc.ssm_cfg or {})
        has_ssm = len(set(bc.attn_layer_idx or [])) < bc.n_layer
        # mamba_ssm create_block: ssm_cfg.pop("layer", "Mamba1") selects the SSM layer class
        if has_ssm and s.pop("layer", "Mamba1") != "Mamba2":
            raise ValueError("only Mamba2 SSM layers are supported")
        if a.get("qkv_proj_bias", False) or a.get("out_proj_bias", False):
            raise ValueError("biased attention projections are not supported")
        if a.get("rotary_emb_interleaved", False):
            raise ValueError("interleaved rotary embeddings are not supported (GPT-NeoX rotate-half only)")
        if a.get("rotary_emb_dim", bc.d_model // a.get("num_heads", 16)) != bc.d_model // a.get("num_heads", 16):
            raise ValueError("partial rotary embeddings are not supported")

        def gated_width(n):          # mamba_ssm GatedMLP: hidden_features rounded up to multiple_of = 128
            return (n + 127) // 128 * 128 if n else 0

        # create_block (_mamba_ssm.py:18-31): Mamba2 blocks get GatedMLP(d_intermediate) when it is
        # nonzero, attention blocks GatedMLP(attn_mlp_d_intermediate); rms_norm / residual_in_fp32
        # go to every Block and to the final layer_norm_fn (:49-57)
        return cls(d_model=bc.d_model, n_layer=bc.n_layer, attn_layer_idx=tuple(bc.attn_layer_idx),
                   n_heads=a.get("num_heads", 16), n_kv=a.get("num_heads_kv", a.get("num_heads", 16)),
                   d_ff=gated_width(bc.attn_mlp_d_intermediate), d_state=s.get("d_state", 128),
                   d_conv=s.get("d_conv", 4), expand=s.get("expand", 2), headdim=s.get("headdim", 64),
                   ngroups=s.get("ngroups", 1), rotary_base=a.get("rotary_emb_base", 10000.0), eps=bc.norm_epsilon,
                   d_mlp=gated_width(bc.d_intermediate) if has_ssm else 0, rms_norm=bool(bc.rms_norm),
                   residual_in_fp32=bool(bc.residual_in_fp32))


def rotary_table(seq_len: int, dim: int, base: float = 10000.0) -> torch.Tensor:
    """flash_attn RotaryEmbedding cos/sin cache (fp32 math, cached in bf16 as the model dtype),
    returned as fp32 [seq_len][dim/2][2] holding the bf16-rounded values."""
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
    f = torch.outer(torch.arange(seq_len, dtype=torch.float32), inv)
    return torch.stack([torch.cos(f).to(torch.bfloat16).float(), torch.sin(f).to(torch.bfloat16).float()],
                       dim=-1).contiguous()


class HybridBackbone:
    """The hybrid layers + final LayerNorm on the device (_mamba_ssm.py:9-57): bf16 weights in the
    engine's layouts and the per-layer launch sequence. Shared by the generate() engine
    (HybridDecoder) and the backbone plugin (zonos_amd.backbone.HipHybridBackbone); ``prefix`` is
    "backbone." for a Zonos state dict and "" for the backbone's own."""

    def __init__(self, cfg: HybridEngineConfig, weights: dict, device="cuda", prefix: str = "backbone."):
        _lib.load()
        if cfg.d_conv != 4 or cfg.ngroups != 1:
            raise ValueError("Mamba2 d_conv=4, ngroups=1 only")
        self.cfg = cfg
        self.fuse_qkv = True
        self.rope_neox = 1
        self.device = torch.device(device)
        dev, bf = self.device, torch.bfloat16

        def w(name):
            return weights[prefix + name].to(device=dev, dtype=bf).contiguous()

        def f32(name):
            return weights[prefix + name].to(device=dev, dtype=bf).float().contiguous()

        def wb(name):                # a norm bias: absent from a bias-free RMSNorm (rms_norm)
            return None if cfg.rms_norm else w(name)

        def mlp(p, width):           # norm2 + GatedMLP (fc1 rows interleaved for the SwiGLU epilogue)
            fc1 = w(p + "mlp.fc1.weight")
            if fc1.shape[0] != 2 * width:
                raise ValueError(f"{p}mlp.fc1.weight has {fc1.shape[0]} rows, the config says 2 x {width}")
            fc1p = torch.empty_like(fc1)
            call("zk_permute_fc1", ptr(fc1), width, cfg.d_model, ptr(fc1p), stream)
            return dict(ln2_w=w(p + "norm2.weight"), ln2_b=wb(p + "norm2.bias"), d_mlp=width,
                        fc1=pack_weights(fc1p, stream), fc2=pack_weights(w(p + "mlp.fc2.weight"), stream))

        stream = _lib.stream_ptr(dev)
        self.layers = []
        for i in range(cfg.n_layer):
            p = f"layers.{i}."
            L = dict(ln1_w=w(p + "norm.weight"), ln1_b=wb(p + "norm.bias"), d_mlp=0)
            if i in cfg.attn_layer_idx:
                L.update(type="attn", wqkv=pack_weights(w(p + "mixer.in_proj.weight"), stream),
                         wo=pack_weights(w(p + "mixer.out_proj.weight"), stream), **mlp(p, cfg.d_ff))
            else:
                cw = weights[prefix + p + "mixer.conv1d.weight"].to(device=dev, dtype=bf).float()
                L.update(type="mamba", w_in=pack_weights(w(p + "mixer.in_proj.weight"), stream),
                         conv_w=cw.reshape(cfg.conv_dim, cfg.d_conv).contiguous(),
                         conv_b=f32(p + "mixer.conv1d.bias"),
                         A=(-torch.exp(weights[prefix + p + "mixer.A_log"].to(bf).float())).to(dev).contiguous(),
                         dt_bias=f32(p + "mixer.dt_bias"), D=f32(p + "mixer.D"),
                         norm_w=f32(p + "mixer.norm.weight"),
                         w_out=pack_weights(w(p + "mixer.out_proj.weight"), stream))
                if cfg.d_mlp:
                    L.update(mlp(p, cfg.d_mlp))
            self.layers.append(L)
        self.attn_ids = [i for i in range(cfg.n_layer) if i in cfg.attn_layer_idx]
        self.mamba_ids = [i for i in range(cfg.n_layer) if i not in cfg.attn_layer_idx]
        self.lnf_w = w("norm_f.weight")
        self.lnf_b = w("norm_f.bias")
        self.freqs = rotary_table(16384, cfg.head_dim, cfg.rotary_base).to(dev)

    def _kv(self, ws, layer):
        if "kv_layers" in ws:            # caches handed out per layer (backbone plugin)
            kv = ws["kv_layers"][layer]
            return kv[0], kv[1]
        j = self.attn_ids.index(layer)
        return ws["kv"][j, 0], ws["kv"][j, 1]

    def _states(self, ws, layer):
        """(conv, ssm) state pair of a Mamba layer, each [2 parity buffers][...]."""
        if "state_layers" in ws:         # backbone plugin
            return ws["state_layers"][layer]
        j = self.mamba_ids.index(layer)
        return ws["conv"][j], ws["ssm"][j]

    # ------------------------------------------------------------------ layer loop
    def _layers(self, ws, M: int, R: int, S: int, prefill: bool, stream, skip):
        c = self.cfg
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        di, nin, nh = c.d_inner, c.d_in_proj, c.nheads_ssm
        Nqkv = (H + 2 * Hk) * hd
        sp = ws["splits"] if not prefill else dict(qkv=1, o=1, fc2=1, inp=1, out=1)
        x, xn, q, y, h, part = ws["x"], ws["xn"], ws["q"], ws["y"], ws["h"], ws["part"]
        xr = ws["xf"] if c.residual_in_fp32 else x           # the residual stream
        rf = c.resid_flags
        scal = ws["scal"]
        pos_dev = None if prefill else ptr(scal[1:2])
        for i, L in enumerate(self.layers):
            if i + 1 < len(self.layers):
                nw, nb = self.layers[i + 1]["ln1_w"], self.layers[i + 1]["ln1_b"]
            else:
                nw, nb = self.lnf_w, self.lnf_b
            if c.norm_flags or c.d_mlp:
                # the same sequence as zk_hybrid_decode_step's (capi.cpp hybrid_layers) for the variants
                self._layer_var(ws, i, L, M, R, S, prefill, stream, skip, sp, xr, rf, nw, nb, pos_dev)
                continue
            if L["type"] == "attn":
                kc, vt = self._kv(ws, i)
                call("zk_gemm_bf16", ptr(xn), D, ptr(L["wqkv"]), M, Nqkv, D, sp["qkv"], 0, ptr(part), None, skip,
                     stream)
                if prefill:
                    call("zk_qkv_rope", ptr(part), 1, R, S, H, Hk, hd, ptr(self.freqs), 0, None, ptr(q), ptr(kc),
                         ptr(vt), ws["smax"], None, 1, skip, stream)
                    call("zk_attn_prefill", ptr(q), ptr(kc), ptr(vt), R, S, H, Hk, hd, ws["smax"], ptr(y), stream)
                else:
                    call("zk_attn_decode_qkv", ptr(part), sp["qkv"], ptr(self.freqs), ptr(kc), ptr(vt), R, H, Hk, hd,
                         ws["smax"], 1, ptr(scal[1:2]), ptr(ws["attn_work"]), ws["attn_splits"], ptr(y), 1, skip,
                         stream)
                call("zk_gemm_bf16", ptr(y), H * hd, ptr(L["wo"]), M, D, H * hd, sp["o"], 0, ptr(part), None, skip,
                     stream)
                call("zk_resid_ln", ptr(part), sp["o"], ptr(x), ptr(L["ln2_w"]), ptr(L["ln2_b"]), c.eps, M, D,
                     ptr(x), ptr(xn), 1, skip, stream)
                call("zk_gemm_bf16", ptr(xn), D, ptr(L["fc1"]), M, 2 * Fd, D, 1, 1, None, ptr(h), skip, stream)
                call("zk_gemm_bf16", ptr(h), Fd, ptr(L["fc2"]), M, D, Fd, sp["fc2"], 0, ptr(part), None, skip, stream)
                call("zk_resid_ln", ptr(part), sp["fc2"], ptr(x), ptr(nw), ptr(nb), c.eps, M, D, ptr(x), ptr(xn), 1,
                     skip, stream)
            else:
                conv, ssm = self._states(ws, i)
                # SSM state double-buffered by position parity
                sr = S & 1
                ssm_b = ptr(ssm[1])
                call("zk_gemm_bf16", ptr(xn), D, ptr(L["w_in"]), M, nin, D, sp["inp"], 0, ptr(part), None, skip,
                     stream)
                if prefill:
                    # the first decode step (position S) reads conv buffer (S & 1)
                    call("zk_mamba_prefill", ptr(part), R, S, di, nh, c.headdim, c.d_state, ptr(L["conv_w"]),
                         ptr(L["conv_b"]), ptr(ws["xc"]), ptr(conv[S & 1]), ptr(ssm[sr]), ptr(L["A"]),
                         ptr(L["dt_bias"]),
                         ptr(L["D"]), ptr(ws["yz"]), stream)
                else:
                    call("zk_mamba_step", ptr(part), sp["inp"], R, di, nh, c.headdim, c.d_state, ptr(L["conv_w"]),
                         ptr(L["conv_b"]), ptr(conv[0]), ptr(conv[1]), pos_dev, ptr(ssm[0]), ssm_b, ptr(L["A"]),
                         ptr(L["dt_bias"]), ptr(L["D"]), ptr(ws["yz"]), skip, stream)
                call("zk_gated_rmsnorm", ptr(ws["yz"]), M, di, ptr(L["norm_w"]), 1e-5, ptr(ws["ym"]), skip, stream)
                call("zk_gemm_bf16", ptr(ws["ym"]), di, ptr(L["w_out"]), M, D, di, sp["out"], 0, ptr(part), None,
                     skip, stream)
                call("zk_resid_ln", ptr(part), sp["out"], ptr(x), ptr(nw), ptr(nb), c.eps, M, D, ptr(x), ptr(xn), 1,
                     skip, stream)


    def _layer_var(self, ws, i, L, M, R, S, prefill, stream, skip, sp, xr, rf, nw, nb, pos_dev):
        """One block under rms_norm / residual_in_fp32 / a Mamba-block MLP (capi.cpp hybrid_layers)."""
        c = self.cfg
        D, H, Hk, hd = c.d_model, c.n_heads, c.n_kv, c.head_dim
        di, nin, nh = c.d_inner, c.d_in_proj, c.nheads_ssm
        Nqkv = (H + 2 * Hk) * hd
        xn, q, y, h, part = ws["xn"], ws["q"], ws["y"], ws["h"], ws["part"]
        if L["type"] == "attn":
            kc, vt = self._kv(ws, i)
            call("zk_gemm_bf16", ptr(xn), D, ptr(L["wqkv"]), M, Nqkv, D, sp["qkv"], 0, ptr(part), None, skip, stream)
            if prefill:
                call("zk_qkv_rope", ptr(part), 1, R, S, H, Hk, hd, ptr(self.freqs), 0, None, ptr(q), ptr(kc), ptr(vt),
                     ws["smax"], None, 1, skip, stream)
                call("zk_attn_prefill", ptr(q), ptr(kc), ptr(vt), R, S, H, Hk, hd, ws["smax"], ptr(y), stream)
            else:
                call("zk_attn_decode_qkv", ptr(part), sp["qkv"], ptr(self.freqs), ptr(kc), ptr(vt), R, H, Hk, hd,
                     ws["smax"], 1, pos_dev, ptr(ws["attn_work"]), ws["attn_splits"], ptr(y), 1, skip, stream)
            call("zk_gemm_bf16", ptr(y), H * hd, ptr(L["wo"]), M, D, H * hd, sp["o"], 0, ptr(part), None, skip, stream)
            smix = sp["o"]
        else:
            conv, ssm = self._states(ws, i)
            call("zk_gemm_bf16", ptr(xn), D, ptr(L["w_in"]), M, nin, D, sp["inp"], 0, ptr(part), None, skip, stream)
            if prefill:
                call("zk_mamba_prefill", ptr(part), R, S, di, nh, c.headdim, c.d_state, ptr(L["conv_w"]),
                     ptr(L["conv_b"]), ptr(ws["xc"]), ptr(conv[S & 1]), ptr(ssm[S & 1]), ptr(L["A"]),
                     ptr(L["dt_bias"]), ptr(L["D"]), ptr(ws["yz"]), stream)
            else:
                call("zk_mamba_step", ptr(part), sp["inp"], R, di, nh, c.headdim, c.d_state, ptr(L["conv_w"]),
                     ptr(L["conv_b"]), ptr(conv[0]), ptr(conv[1]), pos_dev, ptr(ssm[0]), ptr(ssm[1]), ptr(L["A"]),
                     ptr(L["dt_bias"]), ptr(L["D"]), ptr(ws["yz"]), skip, stream)
            call("zk_gated_rmsnorm", ptr(ws["yz"]), M, di, ptr(L["norm_w"]), 1e-5, ptr(ws["ym"]), skip, stream)
            call("zk_gemm_bf16", ptr(ws["ym"]), di, ptr(L["w_out"]), M, D, di, sp["out"], 0, ptr(part), None, skip,
                 stream)
            smix = sp["out"]
        Fl = L["d_mlp"]
        if Fl:
            sfl = fit_split(Fl, sp["fc2"])
            call("zk_resid_ln", ptr(part), smix, ptr(xr), ptr(L["ln2_w"]), ptr(L["ln2_b"]), c.eps, M, D, ptr(xr),
                 ptr(xn), rf, skip, stream)
            call("zk_gemm_bf16", ptr(xn), D, ptr(L["fc1"]), M, 2 * Fl, D, 1, 1, None, ptr(h), skip, stream)
            call("zk_gemm_bf16", ptr(h), Fl, ptr(L["fc2"]), M, D, Fl, sfl, 0, ptr(part), None, skip, stream)
            smix = sfl
        call("zk_resid_ln", ptr(part), smix, ptr(xr), ptr(nw), ptr(nb), c.eps, M, D, ptr(xr), ptr(xn), rf, skip,
             stream)

    def _prenorm(self, ws, M: int, stream, skip):
        """The first block's norm of the embedding rows in ws["x"] under the config variants
        (layer_norm_fn with residual = None; capi.cpp hybrid_prenorm)."""
        c = self.cfg
        L0 = self.layers[0]
        xr = ws["xf"] if c.residual_in_fp32 else ws["x"]
        call("zk_resid_ln", None, 0, ptr(ws["x"]), ptr(L0["ln1_w"]), ptr(L0["ln1_b"]), c.eps, M, c.d_model, ptr(xr),
             ptr(ws["xn"]), 1 | (2 if c.rms_norm else 0) | (8 if c.residual_in_fp32 else 0), skip, stream)


def fit_split(K: int, s: int) -> int:
    """capi.cpp fit_split: the requested split-K, lowered until it divides K into 64-deep chunks."""
    while s > 1 and K % (s * 64):
        s -= 1
    return s


class HybridDecoder(HybridBackbone, HipDecoder):
    """generate() for the hybrid backbone (the layer loop and state differ from HipDecoder)."""

    small_batch_path = False      # the hybrid block sequence has its own _layers (prenorm add + norm)
    # the step / prefill sequences are enqueued by the C ABI (zk_hybrid_decode_step / zk_hybrid_prefill);
    # False issues the same sequence from Python (bit-identical; the reference for the test)
    c_step = True

    def __init__(self, cfg: HybridEngineConfig, weights: dict, device="cuda"):
        HybridBackbone.__init__(self, cfg, weights, device)
        self.embed_norm = not cfg.norm_flags
        dev, bf = self.device, torch.bfloat16

        def w(name):
            return weights[name].to(device=dev, dtype=bf).contiguous()

        self.emb = torch.stack([w(f"embeddings.{k}.weight") for k in range(N_CB)]).contiguous()
        heads = []
        for k in range(N_CB):
            h = w(f"heads.{k}.weight")
            if h.shape[0] < VOCAB:
                h = torch.cat([h, h.new_zeros(VOCAB - h.shape[0], h.shape[1])])
            heads.append(h)
        self.heads = pack_weights(torch.cat(heads).contiguous(), _lib.stream_ptr(dev))
        self._ws = None
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------ workspace
    def _alloc(self, B: int, Lc: int, P: int, max_new: int) -> dict:
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
            ws["conv"].zero_()
            ws["ssm"].zero_()
            return ws
        self.release()
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        di, nin = c.d_inner, c.d_in_proj
        Nqkv = (H + 2 * Hk) * hd
        Nh = N_CB * VOCAB
        Mp = R * S_pre
        f32, bf, i32 = torch.float32, torch.bfloat16, torch.int32
        # Mamba in_proj (N = 8512, K = 2048) without split-K: 133 workgroups, no fp32 slab round trip
        # for k_mamba_step (c5 decode step 4.67 vs 4.87 ms with 2 splits, 4.96 with 4; tools/c5_split_ab.sh;
        # round 4 with 80-column split-2 workgroups: the GEMM 15.3 -> 12.8 us alone, the step 4.34 -> 4.39 ms,
        # profiles/r4s3_hyb_inp_split_ab.txt)
        # (attention out_proj 4-way and the heads unsplit, as the transformer engine: 4.645 vs 4.670 ms)
        splits = dict(qkv=_split_for(Nqkv, D, R), o=_split_for(D, H * hd, R, target_blocks=128),
                      fc2=_split_for(D, max(Fd, 64), R), heads=1, inp=MAMBA_INP_SPLIT, out=_split_for(D, di, R))
        part_n = max(Mp * Nqkv, Mp * D, Mp * nin, splits["qkv"] * R * Nqkv, splits["o"] * R * D,
                     splits["fc2"] * R * D, splits["heads"] * R * Nh, splits["inp"] * R * nin, splits["out"] * R * D)
        if c.d_mlp and not Fd:       # a Mamba-block MLP without attention MLPs: its own fc2 split
            splits["fc2"] = _split_for(D, c.d_mlp, R)
            part_n = max(part_n, splits["fc2"] * R * D)
        attn_splits = attn_splits_for(R, Hk, smax)
        na, nm = len(self.attn_ids), len(self.mamba_ids)
        ws = dict(
            key=key, R=R, T=T, Ld=Ld, smax=smax, S_pre=S_pre, splits=splits, attn_splits=attn_splits,
            kv=torch.zeros(max(na, 1), 2, R * Hk * smax * hd, dtype=bf, device=dev),
            conv=torch.zeros(max(nm, 1), 2, R * c.conv_dim * 4, dtype=bf, device=dev),
            # double-buffered by step parity like the conv state (zk_mamba_step reads one, writes the other)
            ssm=torch.zeros(max(nm, 1), 2, R * c.nheads_ssm * c.headdim * c.d_state, dtype=bf, device=dev),
            x=torch.empty(Mp, D, dtype=bf, device=dev), xn=torch.empty(Mp, D, dtype=bf, device=dev),
            q=torch.empty(Mp, H * hd, dtype=bf, device=dev), y=torch.empty(Mp, H * hd, dtype=bf, device=dev),
            h=torch.empty(Mp, max(Fd, c.d_mlp, 1), dtype=bf, device=dev), part=torch.empty(part_n, dtype=f32, device=dev),
            xf=torch.empty(Mp, D, dtype=f32, device=dev) if c.residual_in_fp32 else None,
            yz=torch.empty(Mp, di, dtype=f32, device=dev), ym=torch.empty(Mp, di, dtype=bf, device=dev),
            xc=torch.empty(Mp, c.conv_dim, dtype=bf, device=dev),
            attn_work=torch.empty(max(1, R * Hk * attn_splits * (8 + 4 * hd)), dtype=f32, device=dev),
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

    # ------------------------------------------------------------------ C ABI descriptor
    def _step_desc(self, ws, B, st, sp):
        """zk_hybrid_desc of this workspace: per-layer weights + states, buffers, state, params."""
        c = self.cfg
        if "hybrid_layers" not in ws:
            arr = (_lib.HybridLayer * c.n_layer)()
            for i, L in enumerate(self.layers):
                e = _lib.HybridLayer()
                e.ln1_w, e.ln1_b = ptr(L["ln1_w"]), ptr(L["ln1_b"])
                e.d_mlp = L["d_mlp"] if L["type"] != "attn" else 0
                if L["d_mlp"]:
                    e.ln2_w, e.ln2_b, e.fc1, e.fc2 = ptr(L["ln2_w"]), ptr(L["ln2_b"]), ptr(L["fc1"]), ptr(L["fc2"])
                if L["type"] == "attn":
                    kc, vt = self._kv(ws, i)
                    e.type = 0
                    e.wqkv, e.wo, e.ln2_w, e.ln2_b = ptr(L["wqkv"]), ptr(L["wo"]), ptr(L["ln2_w"]), ptr(L["ln2_b"])
                    e.fc1, e.fc2, e.k_cache, e.vt_cache = ptr(L["fc1"]), ptr(L["fc2"]), ptr(kc), ptr(vt)
                else:
                    j = self.mamba_ids.index(i)
                    e.type = 1
                    e.w_in, e.conv_w, e.conv_b = ptr(L["w_in"]), ptr(L["conv_w"]), ptr(L["conv_b"])
                    e.A, e.dt_bias, e.Dskip = ptr(L["A"]), ptr(L["dt_bias"]), ptr(L["D"])
                    e.norm_w, e.w_out = ptr(L["norm_w"]), ptr(L["w_out"])
                    e.conv_state[0], e.conv_state[1] = ptr(ws["conv"][j][0]), ptr(ws["conv"][j][1])
                    e.ssm_state[0], e.ssm_state[1] = ptr(ws["ssm"][j][0]), ptr(ws["ssm"][j][1])
                arr[i] = e
            ws["hybrid_layers"] = arr
        sps = ws["splits"]
        return _lib.HybridDesc(B, c.n_layer, c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff, ws["smax"],
                               c.d_inner, c.nheads_ssm, c.headdim, c.d_state, sps["qkv"], sps["o"], sps["fc2"],
                               sps["heads"], sps["inp"], sps["out"], ws["attn_splits"], c.norm_flags, c.eps, 1e-5,
                               C.cast(ws["hybrid_layers"], C.c_void_p), ptr(self.emb), ptr(self.heads),
                               ptr(self.lnf_w), ptr(self.lnf_b), ptr(self.freqs), ptr(ws["x"]), ptr(ws["xn"]),
                               ptr(ws["y"]), ptr(ws["h"]), ptr(ws["part"]), ptr(ws["attn_work"]), ptr(ws["yz"]),
                               ptr(ws["ym"]), ptr(ws["xc"]), ptr(ws["dbg"]), st, sp, ptr(ws["xf"]))

    def _c_decode(self, ws, B, st, sp, stream):
        call("zk_hybrid_decode_step", C.byref(self._step_desc(ws, B, st, sp)), stream)

    def _c_prefill(self, ws, B, st, sp, cond, Lc, P, stream):
        call("zk_hybrid_prefill", C.byref(self._step_desc(ws, B, st, sp)), ptr(cond), Lc, P, ptr(ws["q"]), stream)

