"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the DAC decoder (codes -> waveform).

Functional fp32 restatement of the third-party decoder the reference calls
(zonos/autoencoder.py:44-47 -> transformers DacModel.decode, modeling_dac.py:610-640;
transformers 4.48.3 pinned by uv.lock:2063-2064, 5.15.0 in this image -- the decode
arithmetic is the same in both). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it.

Parity with transformers' DacModel is pinned by tests/test_oracle_golden.py against
tests/golden/dac_*.npz, produced by tests/golden/make_golden.py from an actual
``DacModel(DacConfig(sampling_rate=44100))`` loaded with the same synthetic weights.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F


@dataclass
class DacCfg:
    """configuration_dac.py defaults for descript/dac_44khz."""
    hidden_size: int = 1024          # latent channels
    decoder_hidden_size: int = 1536
    upsampling_ratios: tuple = (8, 8, 4, 2)
    n_codebooks: int = 9
    codebook_size: int = 1024
    codebook_dim: int = 8
    sampling_rate: int = 44100
    encoder_hidden_size: int = 64
    downsampling_ratios: tuple = (2, 4, 8, 8)

    @property
    def hop_length(self):
        return int(math.prod(self.upsampling_ratios))


DAC_44KHZ = DacCfg()


def dac_weight_shapes(c: DacCfg) -> dict:
    """Decoder + quantizer-decode keys in transformers' DacModel state dict."""
    s = {}
    for k in range(c.n_codebooks):
        q = f"quantizer.quantizers.{k}."
        s[q + "codebook.weight"] = (c.codebook_size, c.codebook_dim)
        s[q + "out_proj.weight"] = (c.hidden_size, c.codebook_dim, 1)
        s[q + "out_proj.bias"] = (c.hidden_size,)
    s["decoder.conv1.weight"] = (c.decoder_hidden_size, c.hidden_size, 7)
    s["decoder.conv1.bias"] = (c.decoder_hidden_size,)
    for i, st in enumerate(c.upsampling_ratios):
        cin = c.decoder_hidden_size // 2 ** i
        cout = c.decoder_hidden_size // 2 ** (i + 1)
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
    cl = c.decoder_hidden_size // 2 ** len(c.upsampling_ratios)
    s["decoder.snake1.alpha"] = (1, cl, 1)
    s["decoder.conv2.weight"] = (1, cl, 7)
    s["decoder.conv2.bias"] = (1,)
    return s


def make_dac_weights(c: DacCfg = DAC_44KHZ, seed: int = 0, gain: float = 0.5) -> dict:
    """Seeded synthetic DAC weights. Variance-preserving init (std = gain/sqrt(fan_in)) so the
    waveform is not near-silent (random HF init gives RMS ~5e-3), which would make
    an RMS-error criterion vacuous."""
    out = {}
    for idx, (k, shape) in enumerate(dac_weight_shapes(c).items()):
        g = torch.Generator().manual_seed(seed * 1_000_003 + 7919 * idx + 17)
        if k.endswith("alpha"):
            t = 0.5 + torch.rand(shape, generator=g)
        elif k.endswith("bias"):
            t = 0.05 * torch.randn(shape, generator=g)
        elif k.endswith("codebook.weight"):
            t = torch.randn(shape, generator=g)
        elif "conv_t1" in k:
            cin, cout, ks = shape
            t = torch.randn(shape, generator=g) * (gain / math.sqrt(cin * 2))
        else:
            fan_in = shape[1] * shape[2]
            t = torch.randn(shape, generator=g) * (gain / math.sqrt(fan_in))
        out[k] = t.float()
    return out


def snake(x, alpha):
    """Snake1d.forward (modeling_dac.py:95-100): x + 1/(a+1e-9) * sin(a x)^2."""
    shape = x.shape
    x = x.reshape(shape[0], shape[1], -1)
    x = x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)
    return x.reshape(shape)


def from_codes(W, c: DacCfg, codes: torch.Tensor) -> torch.Tensor:
    """DacResidualVectorQuantizer.from_codes (modeling_dac.py:347-371): sum_k out_proj_k(codebook_k[c_k])."""
    z = 0.0
    for k in range(codes.shape[1]):
        q = f"quantizer.quantizers.{k}."
        lat = F.embedding(codes[:, k, :], W[q + "codebook.weight"]).transpose(1, 2)
        z = z + F.conv1d(lat, W[q + "out_proj.weight"], W[q + "out_proj.bias"])
    return z


def res_unit(W, p, x, dil):
    """DacResidualUnit.forward (modeling_dac.py:175-209)."""
    y = F.conv1d(snake(x, W[p + "snake1.alpha"]), W[p + "conv1.weight"], W[p + "conv1.bias"],
                 dilation=dil, padding=3 * dil)
    y = F.conv1d(snake(y, W[p + "snake2.alpha"]), W[p + "conv2.weight"], W[p + "conv2.bias"])
    pad = (x.shape[-1] - y.shape[-1]) // 2
    if pad > 0:
        x = x[..., pad:-pad]
    return x + y


def decoder(W, c: DacCfg, z: torch.Tensor) -> torch.Tensor:
    """DacDecoder.forward (modeling_dac.py:431-441) with DacDecoderBlock (236-264)."""
    x = F.conv1d(z, W["decoder.conv1.weight"], W["decoder.conv1.bias"], padding=3)
    for i, st in enumerate(c.upsampling_ratios):
        b = f"decoder.block.{i}."
        x = snake(x, W[b + "snake1.alpha"])
        x = F.conv_transpose1d(x, W[b + "conv_t1.weight"], W[b + "conv_t1.bias"], stride=st,
                               padding=math.ceil(st / 2))
        for r, dil in ((1, 1), (2, 3), (3, 9)):
            x = res_unit(W, b + f"res_unit{r}.", x, dil)
    x = snake(x, W["decoder.snake1.alpha"])
    x = F.conv1d(x, W["decoder.conv2.weight"], W["decoder.conv2.bias"], padding=3)
    return torch.tanh(x)


def decode(W, c: DacCfg, codes: torch.Tensor) -> torch.Tensor:
    """DACAutoencoder.decode on CPU (autoencoder.py:44-47, fp32): codes [B,9,T] -> [B,1,hop*T]."""
    assert codes.shape[1] == c.n_codebooks
    with torch.no_grad():
        return decoder(W, c, from_codes(W, c, codes)).squeeze(1).unsqueeze(1).float()


def decode_list(W, c: DacCfg, codes_list) -> list:
    """The decode half of codes_to_wavs (autoencoder.py:219-226): one utterance at a time."""
    out = []
    for x in codes_list:
        x = x.unsqueeze(0) if x.dim() == 2 else x
        if x.shape[2] == 0:
            continue
        out.append(decode(W, c, x).squeeze(0))
    return out


# ----------------------------------------------------------------------------------------
# Encoder (prefix audio -> codes): DACAutoencoder.encode (autoencoder.py:27-28) ->
# DacModel.encode -> DacEncoder (modeling_dac.py DacEncoder / DacEncoderBlock / DacResidualUnit)
# -> DacResidualVectorQuantizer / DacVectorQuantize.decode_latents (cosine nearest code).
# ----------------------------------------------------------------------------------------

def enc_weight_shapes(c: DacCfg) -> dict:
    s = {}
    e = c.encoder_hidden_size
    s["encoder.conv1.weight"] = (e, 1, 7)
    s["encoder.conv1.bias"] = (e,)
    for i, st in enumerate(c.downsampling_ratios):
        dim = e * 2 ** (i + 1)
        b = f"encoder.block.{i}."
        for r in (1, 2, 3):
            u = b + f"res_unit{r}."
            s[u + "snake1.alpha"] = (1, dim // 2, 1)
            s[u + "conv1.weight"] = (dim // 2, dim // 2, 7)
            s[u + "conv1.bias"] = (dim // 2,)
            s[u + "snake2.alpha"] = (1, dim // 2, 1)
            s[u + "conv2.weight"] = (dim // 2, dim // 2, 1)
            s[u + "conv2.bias"] = (dim // 2,)
        s[b + "snake1.alpha"] = (1, dim // 2, 1)
        s[b + "conv1.weight"] = (dim, dim // 2, 2 * st)
        s[b + "conv1.bias"] = (dim,)
    d = e * 2 ** len(c.downsampling_ratios)
    s["encoder.snake1.alpha"] = (1, d, 1)
    s["encoder.conv2.weight"] = (c.hidden_size, d, 3)
    s["encoder.conv2.bias"] = (c.hidden_size,)
    for k in range(c.n_codebooks):
        q = f"quantizer.quantizers.{k}."
        s[q + "in_proj.weight"] = (c.codebook_dim, c.hidden_size, 1)
        s[q + "in_proj.bias"] = (c.codebook_dim,)
    return s


def make_enc_weights(c: DacCfg = DAC_44KHZ, seed: int = 0, gain: float = 0.5) -> dict:
    """Seeded encoder + quantizer-encode weights (the decode-side quantizer weights come from
    make_dac_weights with the same seed)."""
    out = {}
    for idx, (k, shape) in enumerate(enc_weight_shapes(c).items()):
        g = torch.Generator().manual_seed(seed * 1_000_003 + 7919 * idx + 99991)
        if k.endswith("alpha"):
            t = 0.5 + torch.rand(shape, generator=g)
        elif k.endswith("bias"):
            t = 0.05 * torch.randn(shape, generator=g)
        else:
            fan_in = shape[1] * shape[2]
            t = torch.randn(shape, generator=g) * (gain / math.sqrt(fan_in))
        out[k] = t.float()
    return out


def encoder(W, c: DacCfg, wav: torch.Tensor) -> torch.Tensor:
    """DacEncoder.forward: wav [B,1,T] -> latent [B, hidden, T/hop]."""
    x = F.conv1d(wav, W["encoder.conv1.weight"], W["encoder.conv1.bias"], padding=3)
    for i, st in enumerate(c.downsampling_ratios):
        b = f"encoder.block.{i}."
        for r, dil in ((1, 1), (2, 3), (3, 9)):
            x = res_unit(W, b + f"res_unit{r}.", x, dil)
        x = F.conv1d(snake(x, W[b + "snake1.alpha"]), W[b + "conv1.weight"], W[b + "conv1.bias"], stride=st,
                     padding=math.ceil(st / 2))
    return F.conv1d(snake(x, W["encoder.snake1.alpha"]), W["encoder.conv2.weight"], W["encoder.conv2.bias"],
                    padding=1)


def quantize(W, c: DacCfg, z: torch.Tensor, margins: list | None = None) -> torch.Tensor:
    """DacResidualVectorQuantizer.forward (eval): per codebook in_proj -> L2-normalised nearest
    code (max of -(|e|^2 - 2 e.c) + |c|^2) -> codebook row -> out_proj -> residual update.
    ``margins`` (optional) receives per codebook the top-1/top-2 distance gap [B, T]."""
    B, _, T = z.shape
    residual = z
    codes = []
    for k in range(c.n_codebooks):
        q = f"quantizer.quantizers.{k}."
        proj = F.conv1d(residual, W[q + "in_proj.weight"], W[q + "in_proj.bias"])
        enc = F.normalize(proj.permute(0, 2, 1).reshape(B * T, -1))
        cb = F.normalize(W[q + "codebook.weight"])
        dist = -(enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cb.t()) + cb.pow(2).sum(1, keepdim=True).t()
        idx = dist.max(1)[1]
        if margins is not None:
            top = dist.topk(2, dim=1).values
            margins.append((top[:, 0] - top[:, 1]).reshape(B, T))
        idx = idx.reshape(B, T)
        quant = F.embedding(idx, W[q + "codebook.weight"]).transpose(1, 2)
        residual = residual - F.conv1d(quant, W[q + "out_proj.weight"], W[q + "out_proj.bias"])
        codes.append(idx)
    return torch.stack(codes, dim=1)


def encode(W, c: DacCfg, wav: torch.Tensor, margins: list | None = None):
    z = encoder(W, c, wav)
    return z, quantize(W, c, z, margins)
