"""Per-launch timing of the channels-last DAC decode (GPU box): which conv shapes take the time.
    python tools/dac_layers.py [B] [T]
Each zk_dac_* launch is bracketed by HIP events (the wrapped call synchronises, so the numbers
are isolated kernel times); flops per conv = 2 * Cout * Cin * taps * output positions."""
import ctypes as C
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_amd import _lib, autoencoder, synthetic  # noqa: E402
from zonos_amd.autoencoder import DacSpec, HipDacDecoder  # noqa: E402

_lib.load()
HipDacDecoder.c_dac = False      # per-launch timing needs the Python-issued sequence
dev = torch.device("cuda")
S = _lib.stream_ptr()
e0, e1 = _lib.P(), _lib.P()
_lib.call("zk_event_create", C.byref(e0))
_lib.call("zk_event_create", C.byref(e1))
rows = defaultdict(lambda: [0, 0.0, 0.0])
orig = autoencoder.call


def timed(name, *args):
    if name == "zk_dac_resunit_cl":          # fused residual unit: k7 + 1x1 flops
        B, Cc, T = args[1], args[2], args[3]
        orig("zk_event_record", e0.value, S)
        r = orig(name, *args)
        orig("zk_event_record", e1.value, S)
        ms = C.c_float()
        orig("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
        key = (Cc, Cc, 8, T, 1)              # "taps 8" = the fused unit (7 + 1)
        rows[key][0] += 1
        rows[key][1] += ms.value
        rows[key][2] += 2.0 * Cc * Cc * 8 * T * B
        return r
    if name != "zk_dac_conv_cl":
        return orig(name, *args)
    Cin, Tin, Cout, ks, Qn, nphase_stride = args[2], args[3], args[7], args[8], args[11], args[5]
    B = args[1]
    orig("zk_event_record", e0.value, S)
    r = orig(name, *args)
    orig("zk_event_record", e1.value, S)
    ms = C.c_float()
    orig("zk_event_elapsed_ms", e0.value, e1.value, C.byref(ms))
    nph = 1 if nphase_stride == 0 else args[12]          # ConvTranspose: out_stride phases
    fl = 2.0 * Cout * Cin * ks * Qn * B * nph
    key = (Cin, Cout, ks, Tin, nph)
    rows[key][0] += 1
    rows[key][1] += ms.value
    rows[key][2] += fl
    return r


autoencoder.call = timed
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2589
d = HipDacDecoder(DacSpec(), synthetic.dac_weights(dev), dev, precision="fp16")
codes = torch.randint(0, 1024, (B, 9, T), device=dev)
d.decode_padded(codes)          # warm-up
rows.clear()
d.decode_padded(codes)
tot_ms = sum(v[1] for v in rows.values())
tot_fl = sum(v[2] for v in rows.values())
print(f"DAC decode B={B} T={T}: conv total {tot_ms:.1f} ms, {tot_fl / tot_ms / 1e9:.0f} TFLOP/s")
for (cin, cout, ks, tin, nph), (n, ms, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
    print(f"  Cin {cin:5d} Cout {cout:5d} taps {ks} Tin {tin:7d} phases {nph}: {n} x {ms / n:7.2f} ms "
          f"{fl / ms / 1e9:6.0f} TFLOP/s  ({100 * ms / tot_ms:4.1f} %)")
