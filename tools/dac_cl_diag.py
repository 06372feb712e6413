"""Diagnostic: relative error of zk_dac_conv_cl vs torch fp32 conv on identical fp16 operands."""
import math
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from tests.test_gpu_dac_cl import _prep  # noqa: E402
from zonos_amd import _lib as L  # noqa: E402

L.load()
dev = "cuda"
for Cin, Cout, ks, dil, T, wscale in [(64, 128, 7, 1, 300, 1.0), (96, 96, 7, 9, 517, 1.0), (1024, 1536, 7, 1, 40, 1.0),
                                      (384, 384, 1, 1, 129, 1.0), (384, 384, 7, 1, 129, 1e-3)]:
    torch.manual_seed(0)
    B = 2
    x = torch.randn(B, T, Cin, device=dev).half()
    w = (torch.randn(Cout, Cin, ks, device=dev) / math.sqrt(Cin * ks) * wscale).float()
    bias = torch.zeros(Cout, device=dev)
    alpha = torch.ones(Cout, device=dev)
    w16 = _prep(w, 0)
    xo = torch.empty(B, T, Cout, device=dev)
    so = torch.empty(B, T, Cout, dtype=torch.int16, device=dev)
    pad = (ks - 1) // 2 * dil
    L.call("zk_dac_conv_cl", L.ptr(x), B, Cin, T, L.ptr(w16), 0, L.ptr(bias), Cout, ks, dil, pad, T, 1, 1, 0, T,
           None, L.ptr(xo), L.ptr(alpha), L.ptr(so), 0, None, 1, 1, L.stream_ptr(torch.device(dev)))
    torch.cuda.synchronize()
    wh = w.half().float()
    y = F.conv1d(x.float().transpose(1, 2), wh, bias, padding=pad, dilation=dil).transpose(1, 2)
    y64 = F.conv1d(x.double().transpose(1, 2), wh.double(), bias.double(), padding=pad, dilation=dil).transpose(1, 2)
    e = (xo.double() - y64)
    e32 = (y.double() - y64)
    print(f"Cin={Cin} Cout={Cout} ks={ks} dil={dil} wscale={wscale}: kernel rel-rms {e.pow(2).mean().sqrt() / y64.pow(2).mean().sqrt():.3e} "
          f"max {e.abs().max() / y64.abs().max():.3e} | torch-fp32 rel-rms {e32.pow(2).mean().sqrt() / y64.pow(2).mean().sqrt():.3e}; "
          f"w16 subnormal frac {(wh.abs() < 6.1e-5).float().mean():.3f}")
