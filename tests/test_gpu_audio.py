"""GPU: DACAutoencoder.preprocess resampler (zk_resample) and the prefix-audio path vs the oracle
restatement of torchaudio.functional.resample (oracle/resample_ref.py; parity with torchaudio
itself unpinned -- torchaudio is absent and the reference holds no resampled fixture)."""
import math
import os

import pytest
import torch

from oracle import resample_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("orig,T", [(24000, 24000), (16000, 7777), (48000, 4800), (22050, 1000), (44100, 512 * 3),
                                    (8000, 1)])
def test_resample_matches_oracle(orig, T):
    from zonos_amd import audio
    g = torch.Generator().manual_seed(orig + T)
    x = torch.randn(2, T, generator=g) * 0.3
    got = audio.resample(x.cuda(), orig, 44100).cpu()
    ref = resample_ref.resample(x, orig, 44100)
    assert got.shape == ref.shape == (2, math.ceil(T * 44100 / orig)) or orig == 44100
    assert (got - ref).abs().max().item() < 2e-6


def test_preprocess_and_encode_from_wav(tmp_path):
    """load_prefix_audio: 16-bit stereo WAV at 24 kHz -> mono -> 44.1 kHz -> left pad -> codes."""
    import numpy as np

    from oracle import dac_ref
    from zonos_amd.audio import read_wav
    from zonos_amd.autoencoder import DacSpec, DACAutoencoder

    from .golden_util import ENC_DAC
    c = ENC_DAC
    W = dict(dac_ref.make_dac_weights(c, seed=2))
    W.update(dac_ref.make_enc_weights(c, seed=2))
    spec = DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios)
    ae = DACAutoencoder(W, spec, "cuda")
    n, sr = 9000, 24000
    t = np.arange(n) / sr
    pcm = np.stack([0.4 * np.sin(2 * np.pi * 220 * t), 0.2 * np.sin(2 * np.pi * 330 * t)], 1)
    pcm = np.round(pcm * 32767).astype("<i2")
    p = os.path.join(tmp_path, "prefix.wav")
    import wave
    with wave.open(p, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm.tobytes())
    x, rate = read_wav(p)
    assert rate == sr and x.shape == (2, n)
    assert torch.equal(x, torch.from_numpy(pcm.T.astype(np.float32) / 32768.0))
    wav_ref = resample_ref.preprocess(x.mean(0, keepdim=True), sr)
    wav = ae.preprocess(x.mean(0, keepdim=True).cuda(), sr)
    assert wav.shape == wav_ref.shape and wav.shape[-1] % 512 == 0
    assert (wav.cpu() - wav_ref).abs().max().item() < 2e-6
    codes = ae.load_prefix_audio(p)
    assert codes.shape == (1, c.n_codebooks, wav.shape[-1] // 512) and codes.dtype == torch.int64
    z = ae.encoder.latents(wav_ref.unsqueeze(0).cuda())
    assert torch.equal(codes.cpu(), ae.encoder.quantize(z).cpu())
