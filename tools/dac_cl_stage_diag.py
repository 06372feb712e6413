"""Diagnostic: run the channels-last fp16 DAC decode on the dac_44k golden fixture and report
(1) the waveform error vs the golden, (2) a torch emulation of the same numerics on the GPU
(fp32 convs of fp16-rounded operands), (3) per-stage errors of the HIP path vs that emulation."""
import math
import sys

import numpy as np
import torch
import torch.nn.functional as F

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
wav = dec.decode_padded(codes).cpu()
print("HIP fp16 vs golden rms", (wav - ref).pow(2).mean().sqrt().item())

Wg = {k: v.cuda().double() for k, v in W.items()}


def r16(t):
    return t.half().double()


def snake(x, a):
    a = a.view(1, -1, 1)
    return x + (a + 1e-9).reciprocal() * torch.sin(a * x).pow(2)


def emul(round_act=True, round_w=True, snake_f32=False):
    ra = r16 if round_act else (lambda t: t)
    rw = r16 if round_w else (lambda t: t)
    with torch.no_grad():
        z = dac_ref.from_codes({k: v.cpu() for k, v in W.items()}, c, codes.cpu()).cuda().double()
        x = F.conv1d(ra(z), rw(Wg["decoder.conv1.weight"]), Wg["decoder.conv1.bias"], padding=3)
        for i, st in enumerate(c.upsampling_ratios):
            b = f"decoder.block.{i}."
            x = F.conv_transpose1d(ra(snake(x, Wg[b + "snake1.alpha"])), rw(Wg[b + "conv_t1.weight"]),
                                   Wg[b + "conv_t1.bias"], stride=st, padding=math.ceil(st / 2), output_padding=st % 2)
            for r, dil in ((1, 1), (2, 3), (3, 9)):
                u = b + f"res_unit{r}."
                y = F.conv1d(ra(snake(x, Wg[u + "snake1.alpha"])), rw(Wg[u + "conv1.weight"]), Wg[u + "conv1.bias"],
                             padding=3 * dil, dilation=dil)
                y = F.conv1d(ra(snake(y, Wg[u + "snake2.alpha"])), rw(Wg[u + "conv2.weight"]), Wg[u + "conv2.bias"])
                x = x + y
        x = snake(x, Wg["decoder.snake1.alpha"])
        x = F.conv1d(x, Wg["decoder.conv2.weight"], Wg["decoder.conv2.bias"], padding=3)
        return torch.tanh(x).float().cpu()


for ra_, rw_ in ((False, False), (True, True), (True, False), (False, True)):
    e = emul(ra_, rw_)
    print(f"GPU fp64 emulation round_act={ra_} round_w={rw_}: vs golden rms {(e - ref).pow(2).mean().sqrt().item():.3e}"
          f"  vs HIP rms {(e - wav).pow(2).mean().sqrt().item():.3e}")
