"""Fixture of torch's own GPU `Tensor.exponential_(1)` stream -> tests/golden/torch_exp_noise.npz.

Runs on the GPU box (torch only; no reference code involved), then copy the file here:
    python tests/golden/make_torch_noise.py gpurun_out/torch_exp_noise.npz
It pins oracle/torch_philox.py (the CPU restatement of that stream, tests/test_torch_noise_cpu.py):
for each case the generator's (seed, offset) before the call, its offset after, and the values --
every value for the small tensors, 4096 evenly spaced ones for the [64][9][1026] and [300][9][1026]
tensors (the grid-capped and the two-iteration cases of torch's grid-stride kernel).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SIZES = (17, 9 * 1026, 3 * 9 * 1026, 64 * 9 * 1026, 300 * 9 * 1026)
SEEDS = (0, 421, 2 ** 40 + 7)


def main():
    p = torch.cuda.get_device_properties(0)
    out = dict(mp_count=np.int64(p.multi_processor_count), max_threads_per_mp=np.int64(p.max_threads_per_multi_processor),
               torch_version=np.array(torch.__version__), device=np.array(p.name))
    g = torch.Generator(device="cuda")
    i = 0
    for seed in SEEDS:
        g.manual_seed(seed)
        for n in SIZES:
            off = g.get_offset()
            q = torch.empty(n, device="cuda").exponential_(1, generator=g).cpu().numpy()
            idx = np.arange(n) if n < 50000 else np.linspace(0, n - 1, 4096).astype(np.int64)
            out[f"c{i}_seed"] = np.uint64(seed)
            out[f"c{i}_n"] = np.int64(n)
            out[f"c{i}_off"] = np.int64(off)
            out[f"c{i}_off_after"] = np.int64(g.get_offset())
            out[f"c{i}_idx"] = idx.astype(np.int64)
            out[f"c{i}_q"] = q[idx].astype(np.float32)
            i += 1
    out["n_cases"] = np.int64(i)
    np.savez_compressed(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "torch_exp_noise.npz"), **out)
    print(f"{i} cases; mp {p.multi_processor_count} max_threads {p.max_threads_per_multi_processor}")


if __name__ == "__main__":
    main()
