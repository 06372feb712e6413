"""codes_to_wavs post-processing on the GPU vs the CPU oracle (oracle/loudness_ref.py, a
restatement of pyloudnorm 0.1.1 -- pyloudnorm itself is absent here: parity with it is
unpinned; the reference's call sites autoencoder.py:172-245 are followed exactly)."""
import math
import os
import struct

import numpy as np
import pytest
import torch

from oracle import dac_ref, loudness_ref

from .golden_util import TINY_DAC

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _ae():
    from zonos_amd.autoencoder import DACAutoencoder, DacSpec
    d = np.load(os.path.join(G, "dac_44k.npz"))
    c = dac_ref.DAC_44KHZ
    W = dac_ref.make_dac_weights(c, seed=int(d["seed"]))
    return DACAutoencoder(W, DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios)), d


def _signal(n, seed, sr=44100):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n) / sr
    x = 0.05 * torch.sin(2 * math.pi * (220 + 40 * seed) * t) * (1 + 0.5 * torch.sin(2 * math.pi * 3 * t))
    x += 0.01 * torch.randn(n, generator=g)
    x[: n // 7] *= 1e-3           # quiet lead-in (exercises the relative gate)
    return x.unsqueeze(0)


def test_loudness_gains_match_oracle():
    ae, _ = _ae()
    sr = ae.sampling_rate
    # lengths: shorter than a 100 ms block (gain 1), 100 ms blocks (<= 2 s), 400 ms blocks, odd lengths
    wavs = [_signal(n, i) for i, n in enumerate([3000, 4410, 30000, 88200, 88201, 200003, 441000])]
    wavs.append(torch.zeros(1, 50000))                     # silence: loudness -inf -> gain inf (as pyloudnorm)
    got = ae.loudness_gains(wavs, -23.0)
    for w, gg in zip(wavs, got):
        ref = loudness_ref.loudness_gain(w, sr, -23.0)
        if math.isinf(ref):
            assert math.isinf(gg)
        else:
            assert abs(gg - ref) <= 1e-9 * abs(ref), (w.shape, gg, ref)
    assert got[0] == 1.0


def test_codes_to_wavs_matches_oracle_postprocess():
    ae, d = _ae()
    codes = torch.from_numpy(d["codes"].astype(np.int64))
    L = int(d["short_len"])
    wavs = ae.codes_to_wavs([codes[0], codes[1, :, :L], codes[1, :, :0]])
    assert len(wavs) == 2
    dec = ae.decode_list([codes[0], codes[1, :, :L]])
    for w, raw in zip(wavs, dec):
        ref = loudness_ref.postprocess(raw.cpu().clone(), ae.sampling_rate)
        assert w.shape == ref.shape
        assert torch.allclose(w, ref, rtol=1e-6, atol=1e-7)


def test_save_codes_writes_float_wav(tmp_path):
    ae, d = _ae()
    codes = torch.from_numpy(d["codes"].astype(np.int64))
    p = str(tmp_path / "a.wav")
    ae.save_codes(p, codes[0])
    raw = open(p, "rb").read()
    assert raw[:4] == b"RIFF" and raw[8:12] == b"WAVE"
    fmt_tag, ch, sr = struct.unpack("<HHI", raw[20:28])
    assert (fmt_tag, ch, sr) == (3, 1, 44100)
    w = ae.codes_to_wavs(codes[0])[0]
    data = np.frombuffer(raw[raw.index(b"data") + 8:], dtype="<f4")
    assert np.array_equal(data, w.numpy().reshape(-1))


def test_loudness_gpu_ebu3341_known_answers():
    """The batched GPU meter (post.hip) on EBU Tech 3341 cases 1-5 (tests/loudness_kat.py): the
    integrated loudness it implies (target - 20 log10 gain) is the standard's answer within
    +-0.1 LU -- pins the meter to BS.1770-4 / EBU R 128 (pyloudnorm itself is absent)."""
    from .loudness_kat import EBU3341, ebu_expected_mono, ebu_signal
    ae, _ = _ae()
    sr = ae.sampling_rate
    cases = sorted(EBU3341)
    wavs = [torch.from_numpy(ebu_signal(c, sr)).float().unsqueeze(0) for c in cases]
    gains = ae.loudness_gains(wavs, -23.0)
    for c, g in zip(cases, gains):
        loud = -23.0 - 20.0 * math.log10(g)
        assert abs(loud - ebu_expected_mono(c)) <= 0.1, (c, loud, ebu_expected_mono(c))
