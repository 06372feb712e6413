"""GPU parity of the DAC decoder (HIP) vs the reference's DacModel outputs (golden)."""
import os

import numpy as np
import pytest
import torch

from oracle import dac_ref

from .golden_util import TINY_DAC

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _dec(name, precision="fp16x3"):
    from zonos_amd.autoencoder import DacSpec, HipDacDecoder
    d = np.load(os.path.join(G, f"{name}.npz"))
    c = TINY_DAC if name == "dac_tiny" else dac_ref.DAC_44KHZ
    W = dac_ref.make_dac_weights(c, seed=int(d["seed"]))
    spec = DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios)
    return HipDacDecoder(spec, W, "cuda", precision=precision), d, c, W


@pytest.mark.parametrize("name,precision", [("dac_tiny", "fp16x3"), ("dac_44k", "fp16x3"), ("dac_44k", "fp32"),
                                            ("dac_44k", "fp16")])
def test_dac_decode_golden(name, precision):
    """fp16x3 (default) and fp32 are ~fp32-exact; fp16 = the reference's GPU autocast numerics
    (measured on CPU emulation: RMS 6.3e-5 on this fixture) -- all within the 1e-4 bar."""
    dec, d, c, W = _dec(name, precision)
    codes = torch.from_numpy(d["codes"].astype(np.int64)).cuda()
    wav = dec.decode_padded(codes).cpu()
    ref = torch.from_numpy(d["wav"])
    assert wav.shape == ref.shape
    rms = (wav - ref).pow(2).mean().sqrt().item()
    assert rms <= 1e-4, rms                       # north_star: waveform RMS error <= 1e-4 (fp32)
    assert (wav - ref).abs().max().item() < (2e-3 if precision == "fp16" else 1e-4)
    if precision != "fp16":
        assert rms <= 1e-5, rms


@pytest.mark.parametrize("name", ["dac_tiny", "dac_44k"])
def test_dac_ragged_batch_equals_per_utterance(name):
    """codes_to_wavs decodes one utterance at a time (autoencoder.py:219-226); the batched,
    length-masked decode must give the same waveform for the short utterance."""
    dec, d, c, W = _dec(name)
    codes = torch.from_numpy(d["codes"].astype(np.int64)).cuda()
    L = int(d["short_len"])
    wavs = dec.decode_list([codes[0], codes[1, :, :L], codes[1, :, :0]])
    assert len(wavs) == 2                         # empty utterance skipped (autoencoder.py:221-223)
    ref_s = torch.from_numpy(d["wav_short"][0])
    assert wavs[1].shape == ref_s.shape
    rms = (wavs[1].cpu() - ref_s).pow(2).mean().sqrt().item()
    assert rms <= 1e-4, rms
    ref_full = torch.from_numpy(d["wav"][0])
    assert (wavs[0].cpu() - ref_full).pow(2).mean().sqrt().item() <= 1e-4
