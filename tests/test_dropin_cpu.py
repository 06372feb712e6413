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


def test_pad_weight_matches_reference_branches():
    """zonos.utils.pad_weight_ follows utils.py:22-37 branch for branch: Embedding tested on
    embedding_dim (so Embedding(1026, 2048) stays), Linear padded on out_features
    (1025 -> 1026, in_features kept), both dims reset, other modules raise ValueError."""
    import pytest
    from zonos.utils import pad_weight_
    e = torch.nn.Embedding(1026, 2048)
    pad_weight_(e, 8)
    assert tuple(e.weight.shape) == (1026, 2048) and (e.num_embeddings, e.embedding_dim) == (1026, 2048)
    e2 = torch.nn.Embedding(1024, 2045)      # 2045 % 8 = 5 -> +5 rows (the reference's quirk)
    pad_weight_(e2, 8)
    assert tuple(e2.weight.shape) == (1029, 2045) and (e2.num_embeddings, e2.embedding_dim) == (1029, 2045)
    lin = torch.nn.Linear(2048, 1025)
    w0 = lin.weight.detach().clone()
    pad_weight_(lin, 8)
    assert tuple(lin.weight.shape) == (1026, 2048) and (lin.out_features, lin.in_features) == (1026, 2048)
    assert torch.equal(lin.weight[:1025], w0) and not lin.weight[1025].any()
    with pytest.raises(ValueError):
        pad_weight_(torch.nn.Conv1d(2, 2, 1), 8)
