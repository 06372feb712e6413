"""Prefix-audio input side of DACAutoencoder (zonos/autoencoder.py:21-42): WAV reading
(torchaudio.load for RIFF/WAVE files), the resampler of ``preprocess`` on the GPU (zk_resample),
and the 512-sample left padding.

torchaudio is not a dependency here. ``sinc_kernel`` restates torchaudio.functional.resample's
default "sinc_interp_hann" filter (lowpass_filter_width 6, rolloff 0.99, table computed in the
waveform's dtype, fp32); the polyphase sum runs in the HIP kernel.
"""
from __future__ import annotations

import math
import struct

import torch

from . import _lib
from ._lib import call, ptr


def sinc_kernel(orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """Windowed-sinc polyphase table [up][2*width + down] (fp32), its width, up and down."""
    g = math.gcd(int(orig), int(new))
    down, up = int(orig) // g, int(new) // g
    base = min(down, up) * rolloff
    width = math.ceil(lowpass_filter_width * down / base)
    idx = torch.arange(-width, width + down, dtype=torch.float32)[None, None] / down
    t = torch.arange(0, -up, -1, dtype=torch.float32)[:, None, None] / up + idx
    t *= base
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base / down
    k = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    k *= window * scale
    return k.reshape(up, -1).contiguous(), width, up, down


def resample(wav: torch.Tensor, orig: int, new: int) -> torch.Tensor:
    """[..., T] -> [..., ceil(T * up / down)] on the GPU (the tensor must live on a GPU)."""
    _lib.require_gpu(wav, "wav")
    if int(orig) == int(new):
        return wav
    kern, width, up, down = sinc_kernel(orig, new)
    shape = wav.shape
    x = wav.reshape(-1, shape[-1]).to(torch.float32).contiguous()
    B, T = x.shape
    Tout = math.ceil(up * T / down)
    out = torch.empty(B, Tout, device=wav.device)
    kern = kern.to(wav.device)
    call("zk_resample", ptr(x), B, T, ptr(kern), up, down, width, kern.shape[1], ptr(out), Tout,
         _lib.stream_ptr(wav.device))
    return out.reshape(*shape[:-1], Tout)


def left_pad(wav: torch.Tensor, multiple: int = 512) -> torch.Tensor:
    pad = math.ceil(wav.shape[-1] / multiple) * multiple - wav.shape[-1]
    return torch.nn.functional.pad(wav, (pad, 0), value=0.0)


def read_wav(path: str):
    """RIFF/WAVE -> (float32 [channels, n], rate), normalised like torchaudio.load: integer PCM
    divided by its full scale (u8 offset 128), IEEE float passed through."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
            if fmt[0] == 0xFFFE and len(body) >= 26:          # WAVE_FORMAT_EXTENSIBLE: sub-format GUID
                fmt = (struct.unpack("<H", body[24:26])[0],) + fmt[1:]
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, _, align, bits = fmt
    n = len(payload) // align
    raw = torch.frombuffer(bytearray(payload[:n * align]), dtype=torch.uint8)
    if tag == 3 and bits == 32:
        x = raw.view(torch.float32)
    elif tag == 3 and bits == 64:
        x = raw.view(torch.float64).float()
    elif tag == 1 and bits == 16:
        x = raw.view(torch.int16).float() / 32768.0
    elif tag == 1 and bits == 32:
        x = raw.view(torch.int32).double().div(2.0 ** 31).float()
    elif tag == 1 and bits == 24:
        b3 = raw.view(-1, 3).to(torch.int32)
        v = (b3[:, 0] | (b3[:, 1] << 8) | (b3[:, 2] << 16))
        v = torch.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.double().div(2.0 ** 23).float()
    elif tag == 1 and bits == 8:
        x = (raw.float() - 128.0) / 128.0
    else:
        raise ValueError(f"{path}: unsupported WAV format tag {tag}, {bits} bits")
    return x.reshape(n, ch).t().contiguous(), rate
