"""GPU parity of the DAC encoder (prefix audio -> codes; DACAutoencoder.encode, autoencoder.py:27-28)
against transformers' DacModel.encode outputs (tests/golden/dac_enc.npz) and the oracle."""
import pytest
import torch

from oracle import dac_ref

from .golden_util import ENC_DAC, load_enc_case

pytestmark = pytest.mark.gpu

# Latent bar: fp16 conv operands with fp32 accumulation (the reference runs the encoder in fp32
# under cuDNN's default TF32 convolutions -- the same 10-bit operand mantissa).
Z_REL_RMS = 3e-3
# Codes: an RVQ index is a discontinuous function of the latent; a code may differ only where
# the oracle's top-1/top-2 distance gap (cosine units) is below this.
MARGIN = 2e-3


def _spec(c):
    from zonos_amd.autoencoder import DacSpec
    return DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios, c.n_codebooks, c.codebook_size,
                   c.codebook_dim)


def _check_codes(codes, codes_ref, margins):
    """Per frame: codebooks are sequential (later residuals depend on earlier picks), so a frame
    must match exactly up to its first codebook whose oracle margin is < MARGIN."""
    B, K, T = codes_ref.shape
    m = torch.stack(margins, 1)                      # [B, K, T]
    bad = 0
    for b in range(B):
        for t in range(T):
            for k in range(K):
                if codes[b, k, t] != codes_ref[b, k, t]:
                    if m[b, k, t] >= MARGIN:
                        bad += 1
                    break
                if m[b, k, t] < MARGIN:
                    break
    return bad


def test_dac_encode_golden():
    from zonos_amd.autoencoder import HipDacEncoder
    W, wav, z_ref, codes_ref = load_enc_case()
    enc = HipDacEncoder(_spec(ENC_DAC), W, "cuda")
    z = enc.latents(wav.cuda())
    z_cf = z.permute(0, 2, 1).float().cpu()
    rel = ((z_cf - z_ref).pow(2).mean().sqrt() / z_ref.pow(2).mean().sqrt()).item()
    assert rel < Z_REL_RMS, rel
    # teacher-forced quantizer: the reference latent through the GPU RVQ kernel
    codes_tf = enc.quantize(z_ref.permute(0, 2, 1).contiguous().cuda()).cpu()
    margins = []
    dac_ref.quantize(W, ENC_DAC, z_ref, margins)
    assert _check_codes(codes_tf, codes_ref, margins) == 0
    # end to end: codes from the GPU latent, margin-aware against the oracle on that latent's path
    codes = enc.encode(wav.cuda()).cpu()
    assert codes.shape == codes_ref.shape and codes.dtype == torch.int64
    agree = (codes[:, 0] == codes_ref[:, 0]).float().mean().item()
    assert agree > 0.9, agree
    margins = []
    codes_o = dac_ref.quantize(W, ENC_DAC, z_cf, margins)
    assert _check_codes(codes, codes_o, margins) == 0


@pytest.mark.parametrize("T", [512 * 6])
def test_dac_encode_44k_geometry(T):
    """Full descript/dac_44khz widths (64 -> 1024 channels, hidden 1024) on a short clip vs the oracle."""
    from zonos_amd.autoencoder import HipDacEncoder
    c = dac_ref.DAC_44KHZ
    W = dict(dac_ref.make_dac_weights(c, seed=11))
    W.update(dac_ref.make_enc_weights(c, seed=11))
    g = torch.Generator().manual_seed(3)
    wav = 0.2 * torch.randn(2, 1, T, generator=g)
    enc = HipDacEncoder(_spec(c), W, "cuda")
    z = enc.latents(wav.cuda()).permute(0, 2, 1).float().cpu()
    with torch.no_grad():
        z_ref = dac_ref.encoder(W, c, wav)
    rel = ((z - z_ref).pow(2).mean().sqrt() / z_ref.pow(2).mean().sqrt()).item()
    assert rel < Z_REL_RMS, rel
    margins = []
    codes_o = dac_ref.quantize(W, c, z, margins)
    codes = enc.quantize(z.permute(0, 2, 1).contiguous().cuda()).cpu()
    assert _check_codes(codes, codes_o, margins) == 0


def test_rvq_encode_ties_first_index():
    """Duplicate codebook rows: the first index wins (torch max semantics)."""
    from zonos_amd.autoencoder import HipDacEncoder
    W, wav, _, _ = load_enc_case()
    W = dict(W)
    for k in range(ENC_DAC.n_codebooks):
        cb = W[f"quantizer.quantizers.{k}.codebook.weight"].clone()
        cb[512:] = cb[:512]
        W[f"quantizer.quantizers.{k}.codebook.weight"] = cb
    enc = HipDacEncoder(_spec(ENC_DAC), W, "cuda")
    z = torch.randn(1, 40, ENC_DAC.hidden_size)
    codes = enc.quantize(z.cuda()).cpu()
    assert int(codes.max()) < 512
    agree = (codes[:, 0] == dac_ref.quantize(W, ENC_DAC, z.permute(0, 2, 1))[:, 0]).float().mean().item()
    assert agree > 0.95, agree
