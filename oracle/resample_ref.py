"""CPU oracle (test infrastructure only) for DACAutoencoder.preprocess (zonos/autoencoder.py:21-25):
torchaudio.functional.resample(wav, sr, 44100) with its defaults (sinc_interp_hann,
lowpass_filter_width=6, rolloff=0.99) then left padding to a multiple of 512.

torchaudio (uv.lock pins torchaudio 2.5.1) is NOT installed here; this restates its published
_get_sinc_resample_kernel / _apply_sinc_resample_kernel (kernel in the waveform dtype; input padded
(width, width + orig); conv1d with stride orig; output truncated to ceil(new * length / orig)).
Parity with torchaudio itself is UNPINNED (no fixture from it exists in the reference).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _kernel(orig, new, gcd, width_lp=6, rolloff=0.99, dtype=torch.float32):
    orig, new = orig // gcd, new // gcd
    base = min(orig, new) * rolloff
    width = math.ceil(width_lp * orig / base)
    idx = torch.arange(-width, width + orig, dtype=dtype)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=dtype)[:, None, None] / new + idx
    t *= base
    t = t.clamp_(-width_lp, width_lp)
    window = torch.cos(t * math.pi / width_lp / 2) ** 2
    t *= math.pi
    k = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    k *= window * (base / orig)
    return k, width


def resample(wav: torch.Tensor, orig: int, new: int) -> torch.Tensor:
    if orig == new:
        return wav
    g = math.gcd(int(orig), int(new))
    k, width = _kernel(int(orig), int(new), g, dtype=wav.dtype)
    shape = wav.shape
    x = wav.reshape(-1, shape[-1])
    n, length = x.shape
    o, nw = int(orig) // g, int(new) // g
    x = F.pad(x, (width, width + o))
    y = F.conv1d(x[:, None], k, stride=o).transpose(1, 2).reshape(n, -1)
    y = y[..., :int(math.ceil(nw * length / o))]
    return y.reshape(*shape[:-1], y.shape[-1])


def preprocess(wav: torch.Tensor, sr: int) -> torch.Tensor:
    wav = resample(wav, sr, 44_100)
    left = math.ceil(wav.shape[-1] / 512) * 512 - wav.shape[-1]
    return F.pad(wav, (left, 0), value=0)
