"""CPU oracle (test infrastructure only) for the post-processing half of
DACAutoencoder.codes_to_wavs (zonos/autoencoder.py:172-245): loudness normalisation to
-23 LUFS, energy-based silence trim, fade-in / log fade-out.

Loudness: the reference calls pyloudnorm (pinned pyloudnorm 0.1.1, uv.lock:1350-1360;
autoencoder.py:172-186), which is NOT installed in this container. This module restates
pyloudnorm 0.1.1's published algorithm (ITU-R BS.1770-4): `Meter(rate, block_size)`
with the "K-weighting" filter = high shelf (G 4 dB, Q 1/sqrt(2), fc 1500 Hz) then high pass
(G 0, Q 0.5, fc 38 Hz), RBJ-cookbook biquads applied with scipy.signal.lfilter in float64;
400 ms (or 100 ms for short audio) gating blocks with 75 % overlap; absolute gate
-70 LUFS, relative gate -10 LU; channel weight 1.0 (mono). pyloudnorm itself is absent and no
fixture from it exists, so parity is pinned to the standard it implements instead: EBU Tech
3341's known-answer cases 1-5 (tests/loudness_kat.py, +-0.1 LU, tests/test_loudness_kat_cpu.py),
and anchored on the reference's call site (autoencoder.py:175-181: block size rule, target,
gain = 10**((target - loudness)/20), exception -> unchanged audio).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.signal
import torch


def _biquad(G: float, Q: float, fc: float, rate: float, kind: str):
    """pyloudnorm IIRfilter.generate_coefficients (RBJ audio-EQ cookbook)."""
    A = 10 ** (G / 40.0)
    w0 = 2.0 * np.pi * (fc / rate)
    alpha = np.sin(w0) / (2.0 * Q)
    if kind == "high_shelf":
        b0 = A * ((A + 1) + (A - 1) * np.cos(w0) + 2 * np.sqrt(A) * alpha)
        b1 = -2 * A * ((A - 1) + (A + 1) * np.cos(w0))
        b2 = A * ((A + 1) + (A - 1) * np.cos(w0) - 2 * np.sqrt(A) * alpha)
        a0 = (A + 1) - (A - 1) * np.cos(w0) + 2 * np.sqrt(A) * alpha
        a1 = 2 * ((A - 1) - (A + 1) * np.cos(w0))
        a2 = (A + 1) - (A - 1) * np.cos(w0) - 2 * np.sqrt(A) * alpha
    elif kind == "high_pass":
        b0 = (1 + np.cos(w0)) / 2
        b1 = -(1 + np.cos(w0))
        b2 = (1 + np.cos(w0)) / 2
        a0 = 1 + alpha
        a1 = -2 * np.cos(w0)
        a2 = 1 - alpha
    else:
        raise ValueError(kind)
    return np.array([b0, b1, b2]) / a0, np.array([a0, a1, a2]) / a0


def k_weighting(rate: float):
    return [_biquad(4.0, 1 / np.sqrt(2), 1500.0, rate, "high_shelf"), _biquad(0.0, 0.5, 38.0, rate, "high_pass")]


def integrated_loudness(data: np.ndarray, rate: float, block_size: float = 0.400) -> float:
    """pyloudnorm 0.1.1 Meter.integrated_loudness for mono data [n] or [n, 1]."""
    x = np.asarray(data, dtype=np.float64).reshape(-1)
    if x.shape[0] < block_size * rate:
        raise ValueError("Audio must have length greater than the block size.")
    for b, a in k_weighting(rate):
        x = scipy.signal.lfilter(b, a, x)
    T_g, gamma_a, step = block_size, -70.0, 1.0 - 0.75
    T = x.shape[0] / rate
    nblocks = int(np.round(((T - T_g) / (T_g * step)))) + 1
    z = np.zeros(nblocks)
    for j in range(nblocks):
        lo = int(T_g * (j * step) * rate)
        hi = int(T_g * (j * step + 1) * rate)
        z[j] = (1.0 / (T_g * rate)) * np.sum(np.square(x[lo:hi]))
    with np.errstate(divide="ignore"):
        lj = -0.691 + 10.0 * np.log10(z)
        J = lj >= gamma_a
        z_avg = np.mean(z[J]) if J.any() else np.nan
        gamma_r = -0.691 + 10.0 * np.log10(z_avg) - 10.0
        J = (lj > gamma_r) & (lj > gamma_a)
        z_avg = np.nan_to_num(np.mean(z[J]) if J.any() else np.nan)
        return float(-0.691 + 10.0 * np.log10(z_avg))


def loudness_gain(wav: torch.Tensor, sr: int, target_lufs: float = -23.0) -> float:
    """The gain normalize_loudness (autoencoder.py:172-186) multiplies by; 1.0 where the
    reference's try/except returns the audio unchanged (too short)."""
    block = 0.400 if wav.shape[1] > 2.0 * sr else 0.100
    try:
        loud = integrated_loudness(wav.cpu().numpy().T, sr, block)
    except ValueError:
        return 1.0
    return 10 ** ((target_lufs - loud) / 20.0)


def trim_silence(wav: torch.Tensor, threshold: float = 1e-5, frame_size: int = 512) -> torch.Tensor:
    """autoencoder.py:49-90, literally: the tail loop's first frame is wav[:, -512:-0] (empty,
    mean = nan, never above the threshold), so the last frame is never tested; a found tail
    frame i cuts at the negative index -(i+1)*512."""
    n = min((wav.shape[1] // frame_size) // 4, 16)
    start, end = 0, wav.shape[1]
    for i in range(n):
        if wav[:, i * frame_size:(i + 1) * frame_size].pow(2).mean() > threshold:
            start = i * frame_size
            break
    for i in range(n):
        if wav[:, -((i + 1) * frame_size): -i * frame_size].pow(2).mean() > threshold:
            end = -((i + 1) * frame_size)
            break
    return wav[:, start:end] if (start > 0 or end < wav.shape[1]) else wav


def postprocess(wav: torch.Tensor, sr: int) -> torch.Tensor:
    """codes_to_wavs per-utterance tail (autoencoder.py:226-243) on a decoded [1, n] fp32 CPU wav."""
    wav = wav * loudness_gain(wav, sr, -23.0)
    wav = trim_silence(wav)
    bs = 512
    wav[:, :bs] *= torch.linspace(0, 1, bs).unsqueeze(0)
    nb = min((wav.shape[1] // bs) // 4, 20)
    if nb > 0:
        wav[:, -(nb * bs):] *= torch.logspace(0, -10, nb * bs).unsqueeze(0)
    return wav


def _self_check():
    rate = 44100
    t = np.arange(int(3 * rate)) / rate
    x = 0.1 * np.sin(2 * np.pi * 997 * t)
    # a 997 Hz sine at -20 dBFS peak reads about -23 LUFS-ish after K-weighting; sanity only
    return integrated_loudness(x, rate), math.isfinite(integrated_loudness(x, rate))
