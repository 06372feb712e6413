"""One channels-last fp16 DAC decode (B=8, 1024 frames, synthetic weights) for PMC collection:

    rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/dpmc -o run \
        --output-format csv -- python3 tools/dac_pmc.py
    python tools/mfma_summary.py gpurun_out/dpmc --match k_conv_cl
"""
import sys

import torch

sys.path.insert(0, ".")
from zonos_amd import _lib, synthetic  # noqa: E402
from zonos_amd.autoencoder import DacSpec, HipDacDecoder  # noqa: E402

_lib.load()
dev = torch.device("cuda")
d = HipDacDecoder(DacSpec(), synthetic.dac_weights(dev), dev, precision="fp16")
codes = torch.randint(0, 1024, (8, 9, 1024), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
for _ in range(2):
    d.decode_padded(codes)
torch.cuda.synchronize()
