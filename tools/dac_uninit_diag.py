"""Diagnostic: detect reads of uninitialised memory in the fp16 DAC path by poisoning the
caching allocator's free blocks with NaN before decoding."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import dac_ref  # noqa: E402
from zonos_amd.autoencoder import DacSpec, HipDacDecoder  # noqa: E402

d = np.load("tests/golden/dac_44k.npz")
c = dac_ref.DAC_44KHZ
W = dac_ref.make_dac_weights(c, seed=int(d["seed"]))
codes = torch.from_numpy(d["codes"].astype(np.int64)).cuda()
ref = torch.from_numpy(d["wav"])
spec = DacSpec(c.hidden_size, c.decoder_hidden_size, c.upsampling_ratios)
dec = HipDacDecoder(spec, W, "cuda", precision="fp16")
w0 = dec.decode_padded(codes).cpu()
print("fresh   rms", (w0 - ref).pow(2).mean().sqrt().item())
for fill in (float("nan"), 1e4):
    junk = [torch.full((1 << 24,), fill, device="cuda") for _ in range(64)]
    del junk
    w1 = dec.decode_padded(codes).cpu()
    print(f"poison {fill}: rms", (w1 - ref).pow(2).mean().sqrt().item(), "nan", torch.isnan(w1).sum().item(),
          "equal fresh", torch.equal(w0, w1))
d32 = HipDacDecoder(spec, W, "cuda", precision="fp32")
_ = d32.decode_padded(codes)
w2 = dec.decode_padded(codes).cpu()
print("after fp32 decode rms", (w2 - ref).pow(2).mean().sqrt().item(), "equal fresh", torch.equal(w0, w2))
dec2 = HipDacDecoder(spec, W, "cuda", precision="fp16")
w3 = dec2.decode_padded(codes).cpu()
print("new decoder rms", (w3 - ref).pow(2).mean().sqrt().item(), "equal fresh", torch.equal(w0, w3))
