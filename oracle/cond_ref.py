"""CPU oracle (test infrastructure only) for PrefixConditioner.forward
(zonos/conditioning.py:373-389) and its conditioners (Conditioner.forward 45-53,
EspeakPhonemeConditioner.apply_cond 300-315, FourierConditioner 318-337,
IntegerConditioner 340-349, PassthroughConditioner 352-358), at the bf16 rounding points of the
bf16 model (Zonos.from_pretrained casts the whole module to bf16, model.py:57-88; buffers too).

Pinned bit-exactly against the reference module itself on this container
(tests/golden/cond.npz, made by tests/golden/make_golden.py). The eSpeak front end (text
cleaning, phonemize) is not restated: the oracle takes phoneme strings and tokenises them with
the reference's symbol table (conditioning.py:143-191; table in zonos_amd/conditioning.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# Zonos-v0.1 conditioner lists (CONDITIONING_README.md; the hybrid adds the last four).
TRANSFORMER_CONDITIONERS = [
    {"type": "EspeakPhonemeConditioner", "name": "espeak"},
    {"type": "PassthroughConditioner", "name": "speaker", "cond_dim": 128, "uncond_type": "learned",
     "projection": "linear"},
    {"type": "FourierConditioner", "name": "emotion", "input_dim": 8, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "fmax", "min_val": 0, "max_val": 24000, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "pitch_std", "min_val": 0, "max_val": 400, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "speaking_rate", "min_val": 0, "max_val": 40, "uncond_type": "learned"},
    {"type": "IntegerConditioner", "name": "language_id", "min_val": -1, "max_val": 126, "uncond_type": "learned"},
]
HYBRID_CONDITIONERS = TRANSFORMER_CONDITIONERS + [
    {"type": "FourierConditioner", "name": "vqscore_8", "input_dim": 8, "min_val": 0.5, "max_val": 0.8,
     "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "ctc_loss", "min_val": -1.0, "max_val": 1000, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "dnsmos_ovrl", "min_val": 1, "max_val": 5, "uncond_type": "learned"},
    {"type": "IntegerConditioner", "name": "speaker_noised", "min_val": 0, "max_val": 1, "uncond_type": "learned"},
]
N_PHONEME_IDS = 4 + 24 + 52 + 109   # SPECIAL_TOKEN_IDS + symbols (conditioning.py:143-156)


def _proj_shapes(pre, proj, cin, d):
    if proj == "linear":
        return {pre + "project.weight": (d, cin), pre + "project.bias": (d,)}
    if proj == "mlp":
        return {pre + "project.0.weight": (d, cin), pre + "project.0.bias": (d,),
                pre + "project.2.weight": (d, d), pre + "project.2.bias": (d,)}
    return {}


def weight_shapes(conditioners: list, d: int, projection: str = "none") -> dict:
    """Parameter/buffer names of PrefixConditioner (relative to ``prefix_conditioner.``)."""
    s = {}
    for i, c in enumerate(conditioners):
        pre = f"conditioners.{i}."
        t = c["type"]
        cin = c.get("cond_dim") or d
        if t == "EspeakPhonemeConditioner":
            s[pre + "phoneme_embedder.weight"] = (N_PHONEME_IDS, d)
        elif t == "FourierConditioner":
            s[pre + "weight"] = (d // 2, c.get("input_dim", 1))
        elif t == "IntegerConditioner":
            s[pre + "int_embedder.weight"] = (c.get("max_val", 512) - c.get("min_val", 0) + 1, d)
        if c.get("uncond_type", "none") == "learned":
            s[pre + "uncond_vector"] = (d,)
        s.update(_proj_shapes(pre, c.get("projection", "none"), cin, d))
    s.update(_proj_shapes("", projection, d, d))
    s["norm.weight"] = (d,)
    s["norm.bias"] = (d,)
    return s


def make_weights(conditioners: list, d: int, projection: str = "none", seed: int = 0) -> dict:
    """Seeded bf16 weights in the module's layout (Fourier buffers ~ randn * std as at init)."""
    out = {}
    for idx, (k, shape) in enumerate(weight_shapes(conditioners, d, projection).items()):
        g = torch.Generator().manual_seed(seed * 7_000_003 + 131 * idx + 17)
        if k == "norm.weight":
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif k.endswith("bias"):
            t = 0.05 * torch.randn(shape, generator=g)
        elif k.endswith(".weight") and "project" in k:
            t = torch.randn(shape, generator=g) / math.sqrt(shape[1])
        elif k.endswith("uncond_vector"):
            t = 0.5 * torch.randn(shape, generator=g)
        else:                                 # embeddings, Fourier frequencies (std 1)
            i = int(k.split(".")[1])
            std = conditioners[i].get("std", 1.0) if k.endswith(f"{i}.weight") else 1.0
            t = torch.randn(shape, generator=g) * std
        out[k] = t.to(torch.bfloat16)
    return out


def _project(W, pre, proj, x):
    if proj == "linear":
        return F.linear(x, W[pre + "project.weight"], W[pre + "project.bias"])
    if proj == "mlp":
        h = F.silu(F.linear(x, W[pre + "project.0.weight"], W[pre + "project.0.bias"]))
        return F.linear(h, W[pre + "project.2.weight"], W[pre + "project.2.bias"])
    return x


def conditioner(W, i: int, c: dict, value, phoneme_ids=None) -> torch.Tensor:
    """Conditioner.forward for conditioner i (conditioning.py:45-53)."""
    pre = f"conditioners.{i}."
    if value is None:
        return W[pre + "uncond_vector"].view(1, 1, -1)
    t = c["type"]
    if t == "EspeakPhonemeConditioner":
        x = F.embedding(phoneme_ids, W[pre + "phoneme_embedder.weight"])
    else:
        (x,) = tuple(value)          # apply_cond(*inputs): the batch-1 tensor unpacks to [seq, n]
        if t == "FourierConditioner":
            lo, hi = c.get("min_val", 0.0), c.get("max_val", 1.0)
            x = (x - lo) / (hi - lo)
            f = 2 * torch.pi * x.to(torch.bfloat16) @ W[pre + "weight"].T
            x = torch.cat([f.cos(), f.sin()], dim=-1)
        elif t == "IntegerConditioner":
            x = F.embedding(x.squeeze(-1) - c.get("min_val", 0), W[pre + "int_embedder.weight"])
        elif t == "PassthroughConditioner":
            assert x.shape[-1] == (c.get("cond_dim") or x.shape[-1])
        else:
            raise ValueError(t)
    return _project(W, pre, c.get("projection", "none"), x)


def prefix_conditioner(W, conditioners: list, cond_dict: dict, phoneme_ids=None,
                       projection: str = "none") -> torch.Tensor:
    """PrefixConditioner.forward (conditioning.py:380-389): [B, sum L_i, D] bf16."""
    conds = [conditioner(W, i, c, cond_dict.get(c["name"]), phoneme_ids) for i, c in enumerate(conditioners)]
    B = max(map(len, conds))
    conds = [c.expand(B, -1, -1) for c in conds]
    x = _project(W, "", projection, torch.cat(conds, dim=-2))
    return F.layer_norm(x, (x.shape[-1],), W["norm.weight"], W["norm.bias"], 1e-5)
