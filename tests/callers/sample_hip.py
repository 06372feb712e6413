"""The reference's sample.py (import lines and call sequence verbatim) against the `zonos` import
surface of this repo. Differences forced by the offline image, and nothing else:
  * `import torchaudio` / `torchaudio.load` are absent: the speaker embedding (speaker_cloning.py,
    out of scope) is a precomputed tensor loaded from $ZONOS_SPEAKER;
  * Zonos.from_pretrained("Zyphra/Zonos-v0.1-transformer") needs the network: the same loader is
    called on a local checkpoint directory ($ZONOS_CKPT: config.json + model.safetensors), which
    from_pretrained resolves a local directory to (zonos_amd/utils.py hub_download);
  * the output path is $ZONOS_OUT.
"""
import os

import torch
import logging
#logging.basicConfig(level=logging.DEBUG)

# To set another device, use set_device before importing any other zonos module
# from zonos.utils import set_device
# set_device("cuda:1")
from zonos.model import Zonos
from zonos.conditioning import make_cond_dict
from zonos.utils import DEFAULT_DEVICE as device

# model = Zonos.from_pretrained("Zyphra/Zonos-v0.1-hybrid", device=device)
model = Zonos.from_pretrained(os.environ["ZONOS_CKPT"], device=device)

speaker = torch.load(os.environ["ZONOS_SPEAKER"], weights_only=True)

torch.manual_seed(421)

cond_dict = make_cond_dict(text="Hello, world!", speaker=speaker, language="en-us")
conditioning = model.prepare_conditioning(cond_dict)

codes = model.generate(conditioning, disable_torch_compile=True)

model.autoencoder.save_codes(os.environ["ZONOS_OUT"], codes)
