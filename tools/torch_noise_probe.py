"""Which float32 log makes a restatement of torch's CUDA `Tensor.exponential_(1)` bit-identical?
Runs on the GPU box: compares tools/torch_noise_probe.so (log variants 0-3, see the .hip) with
torch's own output for several sizes and generator offsets, and prints the policy constants.

    python tools/torch_noise_probe.py
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def policy(n: int, mp: int, maxthr: int):
    """calc_execution_policy (ATen/native/hip/DistributionTemplates.h): grid-stride of the
    distribution kernel and the Philox offset one call consumes."""
    grid = min(mp * (maxthr // 256), (n + 255) // 256)
    stride = 256 * grid
    incr = ((n - 1) // (stride * 4) + 1) * 4
    return stride, incr


def main():
    libs = []
    for name, f in (("p", "torch_noise_probe.so"), ("f", "torch_noise_probe_fast.so")):
        lib = ctypes.CDLL(os.path.join(HERE, f))
        lib.probe_noise.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.c_int]
        libs.append((name, lib))
    p = torch.cuda.get_device_properties(0)
    mp, maxthr = p.multi_processor_count, p.max_threads_per_multi_processor
    print(f"multi_processor_count {mp} max_threads_per_multi_processor {maxthr}")
    g = torch.Generator(device="cuda")
    for seed in (0, 421):
        g.manual_seed(seed)
        for n in (9 * 1026, 64 * 9 * 1026):
            off = g.get_offset()
            ref = torch.empty(n, device="cuda").exponential_(1, generator=g)
            stride, incr = policy(n, mp, maxthr)
            line = f"seed {seed} n {n} off {off} -> {g.get_offset()} (policy incr {incr}, stride {stride}):"
            for name, lb in libs:
                for v in range(10):
                    out = torch.empty(n, device="cuda")
                    assert lb.probe_noise(out.data_ptr(), n, seed, off, stride, v) == 0
                    bad = (out.view(torch.int32) != ref.view(torch.int32))
                    ulp = (out.view(torch.int32) - ref.view(torch.int32)).abs().max().item()
                    line += f" {name}{v} {int(bad.sum())}/{ulp}"
                    if name == "p" and v == 1 and n > 100000 and seed == 0:
                        u = torch.exp(-out[bad].double())
                        h = torch.histc(u, bins=10, min=0, max=1).long().tolist()
                        hu = torch.histc(torch.exp(-out.double()), bins=10, min=0, max=1).long().tolist()
                        print("  v1 mismatch u-deciles", h, "of", hu)
                        print("  sample mismatches (ours, torch):", list(zip(out[bad][:6].tolist(), ref[bad][:6].tolist())))
            print(line, flush=True)


if __name__ == "__main__":
    main()
