"""CPU: the `zonos` import surface (the reference's module names) resolves to this repo's engine,
and the backbone plugin has the reference's parameter layout (no GPU compute here)."""
import torch

from oracle import zonos_ref

from .golden_util import TINY


def test_zonos_import_surface():
    from zonos.autoencoder import DACAutoencoder
    from zonos.backbone import BACKBONES
    from zonos.codebook_pattern import apply_delay_pattern, revert_delay_pattern  # noqa: F401
    from zonos.conditioning import make_cond_dict, supported_language_codes
    from zonos.config import BackboneConfig, InferenceParams, ZonosConfig  # noqa: F401
    from zonos.model import DEFAULT_BACKBONE_CLS, Zonos
    from zonos.sampling import sample_from_logits  # noqa: F401
    from zonos.utils import DEFAULT_DEVICE, find_multiple
    import zonos_amd.autoencoder
    import zonos_amd.model
    assert Zonos is zonos_amd.model.Zonos and DACAutoencoder is zonos_amd.autoencoder.DACAutoencoder
    assert DEFAULT_BACKBONE_CLS is BACKBONES["hip"]
    assert "transformer" in BACKBONES["hip"].supported_architectures
    assert isinstance(DEFAULT_DEVICE, torch.device) and find_multiple(1025, 8) == 1032
    assert "en-us" in supported_language_codes
    d = make_cond_dict(text="Hello", language="en-us", device="cpu")
    assert {"espeak", "speaker", "fmax", "pitch_std", "speaking_rate", "language_id"} <= set(d)


def test_backbone_plugin_parameter_layout():
    """HipZonosBackbone's state dict = TorchZonosBackbone's (reference key names and shapes), so
    the reference's Zonos.load_state_dict fills it unchanged."""
    from zonos.backbone import BACKBONES
    from zonos.config import BackboneConfig
    bb = BACKBONES["hip"](BackboneConfig(**TINY.to_zonos_config()["backbone"]))
    got = {k: tuple(v.shape) for k, v in bb.state_dict().items()}
    exp = {k[len("backbone."):]: v for k, v in zonos_ref.weight_shapes(TINY).items() if k.startswith("backbone.")}
    assert got == exp
