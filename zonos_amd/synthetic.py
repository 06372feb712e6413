"""Synthetic inputs and seeded random weights in the reference's layouts, for benchmarks
and smoke runs (no trained checkpoint is available offline). Shapes follow the reference
state dicts: zonos/model.py:36-37, zonos/backbone/_torch.py:61-62,88-91,114-115,147-148 and
transformers' DacModel (modeling_dac.py:175-264, 347-371, 407-441)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

ZONOS_V01 = dict(d_model=2048, n_layer=26, n_heads=16, n_kv=4, d_ff=8192)


def backbone_shapes(d_model, n_layer, n_heads, n_kv, d_ff, n_cb=9, vocab=1026) -> dict:
    hd = d_model // n_heads
    s = {}
    for i in range(n_layer):
        p = f"backbone.layers.{i}."
        s[p + "norm.weight"] = (d_model,)
        s[p + "norm.bias"] = (d_model,)
        s[p + "mixer.in_proj.weight"] = ((n_heads + 2 * n_kv) * hd, d_model)
        s[p + "mixer.out_proj.weight"] = (d_model, n_heads * hd)
        s[p + "norm2.weight"] = (d_model,)
        s[p + "norm2.bias"] = (d_model,)
        s[p + "mlp.fc1.weight"] = (2 * d_ff, d_model)
        s[p + "mlp.fc2.weight"] = (d_model, d_ff)
    s["backbone.norm_f.weight"] = (d_model,)
    s["backbone.norm_f.bias"] = (d_model,)
    for k in range(n_cb):
        s[f"embeddings.{k}.weight"] = (vocab, d_model)
    for k in range(n_cb):
        s[f"heads.{k}.weight"] = (vocab - 1, d_model)
    return s


def backbone_weights(device, seed=0, **cfg) -> dict:
    c = dict(ZONOS_V01)
    c.update(cfg)
    g = torch.Generator(device=device).manual_seed(seed)
    W = {}
    for k, shape in backbone_shapes(**c).items():
        if k.endswith(("norm.weight", "norm2.weight", "norm_f.weight")):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g, device=device)
        elif k.endswith(".bias"):
            t = 0.1 * torch.randn(shape, generator=g, device=device)
        elif k.startswith("embeddings"):
            t = torch.randn(shape, generator=g, device=device)
        else:
            t = torch.randn(shape, generator=g, device=device) / math.sqrt(shape[1])
        W[k] = t.to(torch.bfloat16)
    return W


# Zonos-v0.1-hybrid geometry as assumed here (the hybrid config.json is not available offline;
# mamba_ssm Mamba2 defaults for the SSM layers). Every size is a parameter.
ZONOS_V01_HYBRID = dict(d_model=2048, n_layer=46, attn_layer_idx=(9, 18, 27, 36, 45), n_heads=16, n_kv=4,
                        d_ff=8192, d_state=128, d_conv=4, expand=2, headdim=64)


def hybrid_shapes(d_model, n_layer, attn_layer_idx, n_heads, n_kv, d_ff, d_state=128, d_conv=4, expand=2,
                  headdim=64, n_cb=9, vocab=1026) -> dict:
    """mamba_ssm parameter names (create_block: Mamba2 / MHA / GatedMLP, Block norms)."""
    hd = d_model // n_heads
    di = expand * d_model
    nh = di // headdim
    conv_dim = di + 2 * d_state
    s = {}
    for i in range(n_layer):
        p = f"backbone.layers.{i}."
        s[p + "norm.weight"] = (d_model,)
        s[p + "norm.bias"] = (d_model,)
        if i in attn_layer_idx:
            s[p + "mixer.in_proj.weight"] = ((n_heads + 2 * n_kv) * hd, d_model)
            s[p + "mixer.out_proj.weight"] = (d_model, n_heads * hd)
            s[p + "norm2.weight"] = (d_model,)
            s[p + "norm2.bias"] = (d_model,)
            s[p + "mlp.fc1.weight"] = (2 * d_ff, d_model)
            s[p + "mlp.fc2.weight"] = (d_model, d_ff)
        else:
            s[p + "mixer.in_proj.weight"] = (2 * di + 2 * d_state + nh, d_model)
            s[p + "mixer.conv1d.weight"] = (conv_dim, 1, d_conv)
            s[p + "mixer.conv1d.bias"] = (conv_dim,)
            s[p + "mixer.dt_bias"] = (nh,)
            s[p + "mixer.A_log"] = (nh,)
            s[p + "mixer.D"] = (nh,)
            s[p + "mixer.norm.weight"] = (di,)
            s[p + "mixer.out_proj.weight"] = (d_model, di)
    s["backbone.norm_f.weight"] = (d_model,)
    s["backbone.norm_f.bias"] = (d_model,)
    for k in range(n_cb):
        s[f"embeddings.{k}.weight"] = (vocab, d_model)
        s[f"heads.{k}.weight"] = (vocab - 1, d_model)
    return s


def hybrid_weights(device, seed=0, **cfg) -> dict:
    """Seeded bf16 hybrid weights generated on the device (Mamba2's init ranges for A_log and dt)."""
    c = dict(ZONOS_V01_HYBRID)
    c.update(cfg)
    g = torch.Generator(device=device).manual_seed(seed)
    W = {}
    for k, shape in hybrid_shapes(**c).items():
        if k.endswith(("norm.weight", "norm2.weight", "norm_f.weight")):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g, device=device)
        elif k.endswith("A_log"):
            t = torch.log(1 + 15 * torch.rand(shape, generator=g, device=device))
        elif k.endswith("dt_bias"):
            dt = torch.exp(torch.rand(shape, generator=g, device=device) * (math.log(0.1) - math.log(1e-3))
                           + math.log(1e-3))
            t = dt + torch.log(-torch.expm1(-dt))
        elif k.endswith(".D"):
            t = torch.ones(shape, device=device)
        elif k.endswith("conv1d.weight"):
            t = torch.randn(shape, generator=g, device=device) / 2.0
        elif k.endswith(".bias"):
            t = 0.1 * torch.randn(shape, generator=g, device=device)
        elif k.startswith("embeddings"):
            t = torch.randn(shape, generator=g, device=device)
        else:
            t = torch.randn(shape, generator=g, device=device) / math.sqrt(shape[1])
        W[k] = t.to(torch.bfloat16)
    return W


def dac_shapes(hidden=1024, dec=1536, ratios=(8, 8, 4, 2), ncb=9, ncode=1024, cdim=8) -> dict:
    s = {}
    for k in range(ncb):
        q = f"quantizer.quantizers.{k}."
        s[q + "codebook.weight"] = (ncode, cdim)
        s[q + "out_proj.weight"] = (hidden, cdim, 1)
        s[q + "out_proj.bias"] = (hidden,)
    s["decoder.conv1.weight"] = (dec, hidden, 7)
    s["decoder.conv1.bias"] = (dec,)
    for i, st in enumerate(ratios):
        cin, cout = dec // 2 ** i, dec // 2 ** (i + 1)
        b = f"decoder.block.{i}."
        s[b + "snake1.alpha"] = (1, cin, 1)
        s[b + "conv_t1.weight"] = (cin, cout, 2 * st)
        s[b + "conv_t1.bias"] = (cout,)
        for r in (1, 2, 3):
            u = b + f"res_unit{r}."
            s[u + "snake1.alpha"] = (1, cout, 1)
            s[u + "conv1.weight"] = (cout, cout, 7)
            s[u + "conv1.bias"] = (cout,)
            s[u + "snake2.alpha"] = (1, cout, 1)
            s[u + "conv2.weight"] = (cout, cout, 1)
            s[u + "conv2.bias"] = (cout,)
    cl = dec // 2 ** len(ratios)
    s["decoder.snake1.alpha"] = (1, cl, 1)
    s["decoder.conv2.weight"] = (1, cl, 7)
    s["decoder.conv2.bias"] = (1,)
    return s


def dac_weights(device, seed=0, gain=0.5, **cfg) -> dict:
    g = torch.Generator(device=device).manual_seed(seed)
    W = {}
    for k, shape in dac_shapes(**cfg).items():
        if k.endswith("alpha"):
            t = 0.5 + torch.rand(shape, generator=g, device=device)
        elif k.endswith("bias"):
            t = 0.05 * torch.randn(shape, generator=g, device=device)
        elif k.endswith("codebook.weight"):
            t = torch.randn(shape, generator=g, device=device)
        else:
            fan = shape[0] * 2 if "conv_t1" in k else shape[1] * shape[2]
            t = torch.randn(shape, generator=g, device=device) * (gain / math.sqrt(fan))
        W[k] = t.float()
    return W


def conditioning(batch: int, Lc: int, D: int, seed: int = 1, device="cpu") -> torch.Tensor:
    """[2B, Lc, D] bf16 stand-in for PrefixConditioner output (ends in LayerNorm, conditioning.py:389)."""
    g = torch.Generator().manual_seed(seed)
    return F.layer_norm(torch.randn(2 * batch, Lc, D, generator=g), (D,)).to(torch.bfloat16).to(device)


def prefix_codes(batch: int, P: int, seed: int = 3, device="cpu") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 1024, (batch, 9, P), generator=g).to(device)
