"""zonos_amd -- MI355X-native (gfx950) engine for the Zonos decode hot path.

Drop-in for the reference's generate() loop and DAC decode:
    from zonos_amd.model import Zonos
    model = Zonos.from_local(config_path, model_path)        # or Zonos.from_pretrained(repo_id)
    codes = model.generate(prefix_conditioning, ...)         # zonos/model.py:224-457
    wavs = model.autoencoder.decode(codes)                    # zonos/autoencoder.py:44-47

All compute runs in hand-written HIP kernels (zonos_amd/csrc, C ABI in
include/zonos_hip.h); there is no CPU fallback.
"""
__version__ = "0.1.0"
