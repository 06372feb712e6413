"""CPU emulation of the channels-last fp16 DAC pipeline against the fp32 reference goldens (VERDICT r4
item 4: keep the residual stream in fp16, the dtype of the reference's GPU autocast?).

  x32: the shipped form -- fp16 conv operands (weights and Snake outputs), fp32 accumulation, the
       residual stream x in fp32;
  x16: the same with x rounded to fp16 at every write (ConvTranspose output, every residual add:
       x = fp16(x + fp16(conv2 + b)), as torch.autocast(fp16) around DacModel.decode stores it).

    python tools/dac_x16_emul.py dac_44k_long      (tests/golden/*.npz; output: profiles/r5_dac_x16_emulation.txt)
"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import dac_ref as DR  # noqa: E402
torch.set_num_threads(8)
h = lambda t: t.half().float()
def snake(x, a): return DR.snake(x, a)
def conv(x, w, b, **kw): return F.conv1d(h(x), h(w), b, **kw)
def convt(x, w, b, **kw): return F.conv_transpose1d(h(x), h(w), b, **kw)
def emul(W, c, codes, x16):
    X = h if x16 else (lambda t: t)
    z = h(DR.from_codes(W, c, codes))
    x = conv(z, W["decoder.conv1.weight"], W["decoder.conv1.bias"], padding=3)
    for i, st in enumerate(c.upsampling_ratios):
        b = f"decoder.block.{i}."
        s = snake(x, W[b + "snake1.alpha"])
        x = X(convt(s, W[b + "conv_t1.weight"], W[b + "conv_t1.bias"], stride=st, padding=math.ceil(st / 2)))
        for r, dil in ((1, 1), (2, 3), (3, 9)):
            p = b + f"res_unit{r}."
            y = conv(snake(x, W[p + "snake1.alpha"]), W[p + "conv1.weight"], W[p + "conv1.bias"], dilation=dil, padding=3 * dil)
            y = conv(snake(y, W[p + "snake2.alpha"]), W[p + "conv2.weight"], W[p + "conv2.bias"])
            x = X(x + (X(y) if x16 else y))
    x = snake(x, W["decoder.snake1.alpha"])
    x = F.conv1d(x, W["decoder.conv2.weight"], W["decoder.conv2.bias"], padding=3)
    return torch.tanh(x)
name = sys.argv[1]
d = np.load(os.path.join(REPO, 'tests', 'golden', f'{name}.npz'))
c = DR.DAC_44KHZ
W = DR.make_dac_weights(c, seed=int(d['seed']))
codes = torch.from_numpy(d['codes'].astype(np.int64))
if 'wav' in d: ref = torch.from_numpy(d['wav'])
else: ref = torch.from_numpy(d['wav_q'].astype(np.float32)) * float(d['wav_scale'])
n = int(sys.argv[2]) if len(sys.argv) > 2 else codes.shape[0]
with torch.no_grad():
    for x16 in (False, True):
        for bi in range(n):
            out = emul(W, c, codes[bi:bi+1], x16)
            L = min(out.shape[-1], ref.shape[-1])
            e = (out[0, 0, :L] - ref[bi, 0, :L])
            print(name, 'x16' if x16 else 'x32', bi, 'rms', float(e.pow(2).mean().sqrt()), 'max', float(e.abs().max()), flush=True)
