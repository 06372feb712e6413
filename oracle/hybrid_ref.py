"""CPU oracle (test infrastructure only) for the hybrid backbone, Zonos-v0.1-hybrid
(zonos/backbone/_mamba_ssm.py:9-57 -> mamba_ssm create_block / Block / Mamba2 / MHA /
GatedMLP, layer_norm_fn).

mamba-ssm (pinned 2.2.4, uv.lock:715-716), causal-conv1d (1.5.0.post8, uv.lock:118-119) and
flash-attn (2.7.4.post1, uv.lock:398-399) are NOT installed in this container and the hybrid
config.json is not here. This module restates their published semantics:

  Block (fused_add_norm, prenorm): residual = hidden + residual (fp32 add of the bf16 values,
    stored bf16 since residual_in_fp32 = False); hidden = LayerNorm(fp32 sum) -> bf16
    (layer_norm_fn, mamba_ssm/ops/triton/layer_norm.py). Blocks whose d_intermediate is 0 (the
    Mamba2 layers) have no MLP; attention layers have norm2 + GatedMLP(fc1 -> y * silu(gate) -> fc2).
  Mamba2 (d_state 128, d_conv 4, expand 2, headdim 64, ngroups 1, rmsnorm gated, no biases):
    in_proj -> [z, xBC, dt]; causal depthwise conv1d (+bias) over xBC, SiLU (causal_conv1d, fp32
    compute, bf16 out); x, B, C = split(xBC); dt = softplus(dt + dt_bias) (threshold 20);
    A = -exp(A_log); h = exp(dt A) h + (B dt) x; y = C.h + D x (selective_state_update /
    SSD scan, fp32 math; the cached SSM state is bf16 because Zonos allocates the inference
    cache in bf16, model.py:204-208); y -> bf16; RMSNormGated(norm_before_gate=False):
    out = rmsnorm(y * silu(z)) * w, eps 1e-5; out_proj.
  MHA: in_proj -> q, k, v; rotary (flash_attn RotaryEmbedding, GPT-NeoX "rotate half", base
    10000, cos/sin cached in bf16, math in fp32) on q and k; KV cache; causal SDPA (GQA);
    out_proj.
  Final: LayerNorm(hidden + residual).

  Config variants (BackboneConfig fields that create_block and the final layer_norm_fn honour,
  _mamba_ssm.py:18-31,49-57; restated from mamba_ssm 2.2.4 Block / GatedMLP / layer_norm_fn):
    rms_norm: block norms are RMSNorm (weight only); layer_norm_fn(is_rms_norm=True) computes
      rstd = 1 / sqrt(mean(x^2) + eps), y = x * rstd * w (+ b: norm_f keeps its LayerNorm bias).
    residual_in_fp32: the residual stream is fp32 (the first block's residual_out = fp32(hidden);
      later blocks keep the fp32 residual they are given); hidden + residual is added in fp32.
    d_intermediate != 0: Mamba2 blocks get norm2 + GatedMLP(d_intermediate rounded up to 128) too.

Parity with the real hybrid is UNPINNED (no mamba_ssm, no checkpoint, no config here); the
prefill scan is run as the exact recurrence (the reference's SSD chunked scan computes the same
recurrence with a different summation order).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

bf = torch.bfloat16


@dataclass
class HybridCfg:
    d_model: int = 2048
    n_layer: int = 46
    attn_layer_idx: tuple = (9, 18, 27, 36, 45)     # assumed (hybrid config.json is not available)
    n_heads: int = 16
    n_kv: int = 4
    d_ff: int = 8192                                # attn_mlp_d_intermediate (attention layers' MLP)
    d_state: int = 128
    d_conv: int = 4
    expand: int = 2
    headdim: int = 64
    ngroups: int = 1
    rotary_base: float = 10000.0
    eps: float = 1e-5
    n_cb: int = 9
    vocab: int = 1026
    d_mlp: int = 0                                  # d_intermediate: GatedMLP width of the Mamba2 blocks
    rms_norm: bool = False
    residual_in_fp32: bool = False

    def mlp_width(self, i: int) -> int:
        return self.d_ff if self.is_attn(i) else self.d_mlp

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

    def is_attn(self, i: int) -> bool:
        return i in self.attn_layer_idx

    @classmethod
    def from_zonos_config(cls, d: dict) -> "HybridCfg":
        b = d["backbone"]
        a, s = b.get("attn_cfg", {}), dict(b.get("ssm_cfg", {}))
        assert s.pop("layer", "Mamba2") == "Mamba2", "only Mamba2 SSM layers"
        assert not a.get("qkv_proj_bias", False) and not a.get("out_proj_bias", False), "biased MHA not supported"
        r128 = lambda n: (n + 127) // 128 * 128 if n else 0     # GatedMLP multiple_of = 128
        return cls(d_mlp=r128(b.get("d_intermediate", 0)), rms_norm=bool(b.get("rms_norm", False)),
                   residual_in_fp32=bool(b.get("residual_in_fp32", False)),d_model=b["d_model"], n_layer=b["n_layer"], attn_layer_idx=tuple(b.get("attn_layer_idx", [])),
                   n_heads=a.get("num_heads", 16), n_kv=a.get("num_heads_kv", a.get("num_heads", 16)),
                   d_ff=r128(b.get("attn_mlp_d_intermediate", 0)), d_state=s.get("d_state", 128),
                   d_conv=s.get("d_conv", 4), expand=s.get("expand", 2), headdim=s.get("headdim", 64),
                   ngroups=s.get("ngroups", 1), rotary_base=a.get("rotary_emb_base", 10000.0),
                   eps=b.get("norm_epsilon", 1e-5))

    def to_zonos_config(self) -> dict:
        return {
            "backbone": {"d_model": self.d_model, "d_intermediate": self.d_mlp, "attn_mlp_d_intermediate": self.d_ff,
                         "n_layer": self.n_layer, "ssm_cfg": {"layer": "Mamba2", "d_state": self.d_state, "d_conv": self.d_conv,
                                                                 "expand": self.expand, "headdim": self.headdim,
                                                                 "ngroups": self.ngroups},
                         "attn_layer_idx": list(self.attn_layer_idx),
                         "attn_cfg": {"causal": True, "num_heads": self.n_heads, "num_heads_kv": self.n_kv,
                                      "rotary_emb_dim": self.head_dim, "qkv_proj_bias": False,
                                      "out_proj_bias": False},
                         "rms_norm": self.rms_norm, "residual_in_fp32": self.residual_in_fp32,
                         "norm_epsilon": self.eps},
            "prefix_conditioner": {"conditioners": [], "projection": "none"},
            "eos_token_id": 1024, "masked_token_id": 1025, "pad_vocab_to_multiple_of": 8,
        }


ZONOS_V01_HYBRID = HybridCfg()


def weight_shapes(c: HybridCfg) -> dict:
    s = {}
    D = c.d_model
    for k in range(c.n_cb):
        s[f"embeddings.{k}.weight"] = (c.vocab, D)
        s[f"heads.{k}.weight"] = (c.vocab - 1, D)
    for i in range(c.n_layer):
        p = f"backbone.layers.{i}."
        s[p + "norm.weight"] = (D,)
        if not c.rms_norm:
            s[p + "norm.bias"] = (D,)
        if c.is_attn(i):
            hd = c.head_dim
            s[p + "mixer.in_proj.weight"] = ((c.n_heads + 2 * c.n_kv) * hd, D)
            s[p + "mixer.out_proj.weight"] = (D, c.n_heads * hd)
        else:
            s[p + "mixer.in_proj.weight"] = (c.d_in_proj, D)
            s[p + "mixer.conv1d.weight"] = (c.conv_dim, 1, c.d_conv)
            s[p + "mixer.conv1d.bias"] = (c.conv_dim,)
            s[p + "mixer.dt_bias"] = (c.nheads_ssm,)
            s[p + "mixer.A_log"] = (c.nheads_ssm,)
            s[p + "mixer.D"] = (c.nheads_ssm,)
            s[p + "mixer.norm.weight"] = (c.d_inner,)
            s[p + "mixer.out_proj.weight"] = (D, c.d_inner)
        # (after the mixer: make_weights draws in this order, so the default geometry's seeded weights
        # -- and the fixtures' checksums -- are those of the round-4 layout)
        if c.mlp_width(i):
            s[p + "norm2.weight"] = (D,)
            if not c.rms_norm:
                s[p + "norm2.bias"] = (D,)
            s[p + "mlp.fc1.weight"] = (2 * c.mlp_width(i), D)
            s[p + "mlp.fc2.weight"] = (D, c.mlp_width(i))
    s["backbone.norm_f.weight"] = (D,)
    s["backbone.norm_f.bias"] = (D,)
    return s


def make_weights(c: HybridCfg, seed: int = 0, head_scale: float = 1.0, eos_bias: float = 0.0) -> dict:
    """Seeded bf16 weights of the hybrid layout (mamba_ssm parameter names), scaled so the
    recurrence stays well conditioned: A_log ~ log U(1, 16), dt_bias = softplus^-1 of
    U(1e-3, 1e-1) (Mamba2's own init ranges), D = 1."""
    g = torch.Generator().manual_seed(seed)
    W = {}
    for k, shp in weight_shapes(c).items():
        if k.endswith("norm.weight") or k.endswith("norm2.weight") or k.endswith("norm_f.weight"):
            t = 1.0 + 0.1 * torch.randn(shp, generator=g)
        elif k.endswith(".bias") and "conv1d" not in k:
            t = 0.1 * torch.randn(shp, generator=g)
        elif k.endswith("A_log"):
            t = torch.log(1 + 15 * torch.rand(shp, generator=g))
        elif k.endswith("dt_bias"):
            dt = torch.exp(torch.rand(shp, generator=g) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
            t = dt + torch.log(-torch.expm1(-dt))
        elif k.endswith(".D"):
            t = torch.ones(shp)
        elif k.endswith("conv1d.weight"):
            t = torch.randn(shp, generator=g) / math.sqrt(c.d_conv)
        elif k.endswith("conv1d.bias"):
            t = 0.1 * torch.randn(shp, generator=g)
        elif k.startswith("embeddings"):
            t = torch.randn(shp, generator=g)
        else:
            t = torch.randn(shp, generator=g) / math.sqrt(shp[-1])
            if k.startswith("heads"):
                t = t * head_scale
        W[k] = t.to(bf)
    if eos_bias:
        W["heads.0.weight"][1024] += eos_bias / math.sqrt(c.d_model)
    for k in range(c.n_cb):      # pad_weight_ (utils.py:22-37)
        h = W[f"heads.{k}.weight"]
        W[f"heads.{k}.weight"] = torch.cat([h, h.new_zeros(c.vocab - h.shape[0], h.shape[1])])
    return W


def rotary_table(seq_len: int, dim: int, base: float = 10000.0) -> torch.Tensor:
    """flash_attn RotaryEmbedding cache: cos/sin(t * inv_freq) rounded to bf16 ([seq][dim/2][2],
    values returned in fp32)."""
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
    f = torch.outer(torch.arange(seq_len, dtype=torch.float32), inv)
    return torch.stack([torch.cos(f).to(bf).float(), torch.sin(f).to(bf).float()], dim=-1).contiguous()


def rope_neox(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    """apply_rotary (non-interleaved): x [R,S,H,hd] bf16, cs [R,S,hd/2,2] fp32 -> bf16."""
    h = x.shape[-1] // 2
    x0, x1 = x[..., :h].float(), x[..., h:].float()
    c, s = cs[..., 0].unsqueeze(2), cs[..., 1].unsqueeze(2)
    return torch.cat([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1).to(bf)


class HybridCache:
    """Per attention layer a KV cache [R][S_max][2][Hkv][hd] bf16; per Mamba layer a conv state
    [R][conv_dim][d_conv] and an SSM state [R][nheads][headdim][d_state], both bf16."""

    def __init__(self, c: HybridCfg, rows: int, max_seqlen: int):
        S = max_seqlen + (-max_seqlen) % 8
        self.kv, self.conv, self.ssm = {}, {}, {}
        for i in range(c.n_layer):
            if c.is_attn(i):
                self.kv[i] = torch.zeros(rows, S, 2, c.n_kv, c.head_dim, dtype=bf)
            else:
                self.conv[i] = torch.zeros(rows, c.conv_dim, c.d_conv, dtype=bf)
                self.ssm[i] = torch.zeros(rows, c.nheads_ssm, c.headdim, c.d_state, dtype=bf)
        self.seqlen_offset = 0
        self.lengths = torch.zeros(rows, dtype=torch.int32)


def norm(s, w, b, eps, rms: bool = False):
    """layer_norm_fn's normalisation of the fp32 sum s -> bf16: LayerNorm, or is_rms_norm
    (y = s * rsqrt(mean(s^2) + eps) * w, + b when there is a bias)."""
    if not rms:
        return F.layer_norm(s, (s.shape[-1],), w.float(), b.float(), eps).to(bf)
    y = s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return (y if b is None else y + b.float()).to(bf)


def add_norm(x, residual, w, b, eps, rms: bool = False, resid_f32: bool = False):
    """layer_norm_fn(..., prenorm=True, residual_in_fp32, is_rms_norm): hidden + residual in fp32,
    the residual returned in fp32 (residual_in_fp32, or a fp32 residual given) or bf16."""
    s = x.float() if residual is None else x.float() + residual.float()
    keep32 = resid_f32 or (residual is not None and residual.dtype == torch.float32)
    return norm(s, w, b, eps, rms), (s if keep32 else s.to(bf))


def mha(W, c: HybridCfg, i, x, cache: HybridCache, rot):
    R, S, _ = x.shape
    hd, H, Hk = c.head_dim, c.n_heads, c.n_kv
    p = f"backbone.layers.{i}.mixer."
    qkv = F.linear(x, W[p + "in_proj.weight"])
    q, k, v = qkv.split([H * hd, Hk * hd, Hk * hd], dim=-1)
    pos = torch.arange(S)[None, :] + cache.lengths[:, None].long()
    cs = rot[pos]
    q = rope_neox(q.reshape(R, S, H, hd), cs)
    k = rope_neox(k.reshape(R, S, Hk, hd), cs)
    v = v.reshape(R, S, Hk, hd)
    kv = cache.kv[i]
    o = cache.seqlen_offset
    kv[:, o:o + S, 0] = k
    kv[:, o:o + S, 1] = v
    kk, vv = kv[:, :o + S].unbind(dim=-3)
    y = F.scaled_dot_product_attention(q.transpose(1, 2), kk.transpose(1, 2), vv.transpose(1, 2),
                                       is_causal=S > 1, enable_gqa=True)
    return F.linear(y.transpose(1, 2).reshape(R, S, H * hd), W[p + "out_proj.weight"])


def mamba2(W, c: HybridCfg, i, u, cache: HybridCache):
    """Mamba2.forward (prefill, seqlen_offset == 0) / Mamba2.step (decode), recurrence form."""
    R, S, _ = u.shape
    p = f"backbone.layers.{i}.mixer."
    di, ds, nh, hp, K = c.d_inner, c.d_state, c.nheads_ssm, c.headdim, c.d_conv
    zx = F.linear(u, W[p + "in_proj.weight"])                     # bf16
    z, xBC, dt = zx.split([di, c.conv_dim, nh], dim=-1)
    wconv = W[p + "conv1d.weight"][:, 0, :].float()                 # [conv_dim][K]
    bconv = W[p + "conv1d.bias"].float()
    st = cache.conv[i]                                               # [R][conv_dim][K] bf16
    hist = torch.cat([st[:, :, 1:].transpose(1, 2), xBC], dim=1)   # [R][K-1+S][conv_dim]
    conv = bconv.expand(R, S, -1).clone()                            # bias + w0 x0 + w1 x1 + ... (fp32)
    for k in range(K):
        conv = conv + hist[:, k:k + S, :].float() * wconv[:, k]
    xc = (conv / (1 + torch.exp(-conv))).to(bf)                      # SiLU in fp32, bf16 out
    cache.conv[i] = hist[:, -K:, :].transpose(1, 2).contiguous()    # last K inputs
    x, Bm, Cm = xc.split([di, ds, ds], dim=-1)
    A = -torch.exp(W[p + "A_log"].float())
    dtb = W[p + "dt_bias"].float()
    Dv = W[p + "D"].float()
    h = cache.ssm[i].float()                                         # [R][nh][hp][ds]
    ys = []
    for t in range(S):
        d = dt[:, t].float() + dtb
        d = torch.where(d <= 20.0, F.softplus(d), d)                 # [R][nh]
        dA = torch.exp(d * A)
        xt = x[:, t].float().view(R, nh, hp)
        dB = Bm[:, t].float()[:, None, :] * d[:, :, None]            # [R][nh][ds]
        h = h * dA[:, :, None, None] + dB[:, :, None, :] * xt[:, :, :, None]
        y = (h * Cm[:, t].float()[:, None, None, :]).sum(-1) + xt * Dv[None, :, None]
        ys.append(y.reshape(R, di).to(bf))
        if S == 1:
            pass
    cache.ssm[i] = h.to(bf)
    y = torch.stack(ys, dim=1)                                       # [R][S][di] bf16
    zf = z.float()
    g = y.float() * (zf * torch.sigmoid(zf))
    rstd = torch.rsqrt(g.pow(2).mean(-1, keepdim=True) + 1e-5)
    yn = (g * rstd * W[p + "norm.weight"].float()).to(bf)
    return F.linear(yn, W[p + "out_proj.weight"])


def backbone(W, c: HybridCfg, h: torch.Tensor, cache: HybridCache, rot: torch.Tensor) -> torch.Tensor:
    """MambaSSMZonosBackbone.forward (_mamba_ssm.py:47-57)."""
    hidden, residual = h, None
    kw = dict(rms=c.rms_norm, resid_f32=c.residual_in_fp32)
    for i in range(c.n_layer):
        p = f"backbone.layers.{i}."
        xn, residual = add_norm(hidden, residual, W[p + "norm.weight"], W.get(p + "norm.bias"), c.eps, **kw)
        if c.is_attn(i):
            hidden = mha(W, c, i, xn, cache, rot)
        else:
            hidden = mamba2(W, c, i, xn, cache)
        if c.mlp_width(i):                      # Block.mlp: norm2 + GatedMLP
            xn, residual = add_norm(hidden, residual, W[p + "norm2.weight"], W.get(p + "norm2.bias"), c.eps, **kw)
            y, gate = F.linear(xn, W[p + "mlp.fc1.weight"]).chunk(2, dim=-1)
            hidden = F.linear(y * F.silu(gate), W[p + "mlp.fc2.weight"])
    s = hidden.float() + residual.float()
    return norm(s, W["backbone.norm_f.weight"], W["backbone.norm_f.bias"], c.eps, c.rms_norm)
