"""DAC encoder: latent error vs the golden / oracle and timing at the 44.1 kHz geometry."""
import sys
import time

import torch

sys.path.insert(0, ".")
from oracle import dac_ref  # noqa: E402
from tests.golden_util import ENC_DAC, load_enc_case  # noqa: E402
from zonos_amd.autoencoder import DacSpec, HipDacEncoder  # noqa: E402


def spec(c):
    return DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios)


W, wav, z_ref, codes_ref = load_enc_case()
enc = HipDacEncoder(spec(ENC_DAC), W)
z = enc.latents(wav.cuda()).permute(0, 2, 1).cpu()
rel = ((z - z_ref).pow(2).mean().sqrt() / z_ref.pow(2).mean().sqrt()).item()
codes = enc.encode(wav.cuda()).cpu()
print(f"golden: z rel rms {rel:.2e}, codes agree {(codes == codes_ref).float().mean().item():.4f}, "
      f"cb0 agree {(codes[:, 0] == codes_ref[:, 0]).float().mean().item():.4f}")
c = dac_ref.DAC_44KHZ
W = dict(dac_ref.make_dac_weights(c, seed=11))
W.update(dac_ref.make_enc_weights(c, seed=11))
enc = HipDacEncoder(spec(c), W)
for B, secs in ((1, 10), (8, 10)):
    T = int(secs * 44100) // 512 * 512
    x = 0.2 * torch.randn(B, 1, T, device="cuda")
    for _ in range(2):
        enc.encode(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        enc.encode(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"44k encode B={B} {secs}s: {dt * 1e3:.2f} ms ({B * secs / dt:.0f}x real time)")
