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
    assert DEFAULT_BACKBONE_CLS is BACKBONES["hip_hybrid"]
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


def test_hybrid_backbone_plugin_parameter_layout_and_registry():
    """HipHybridBackbone's state dict = mamba_ssm's Block / Mamba2 / MHA names and shapes (the
    restatement's weight_shapes), the registry mirrors the reference's (hybrid-capable class first,
    its keys as aliases), and a transformer config builds the transformer blocks."""
    from oracle import hybrid_ref
    from zonos.backbone import BACKBONES
    from zonos.config import BackboneConfig
    from zonos.model import DEFAULT_BACKBONE_CLS
    c = hybrid_ref.HybridCfg(d_model=256, n_layer=4, attn_layer_idx=(2,), n_heads=2, n_kv=1, d_ff=512, d_state=64,
                             headdim=32)
    bb = BACKBONES["mamba_ssm"](BackboneConfig(**c.to_zonos_config()["backbone"]))
    got = {k: tuple(v.shape) for k, v in bb.state_dict().items()}
    exp = {k[len("backbone."):]: v for k, v in hybrid_ref.weight_shapes(c).items() if k.startswith("backbone.")}
    assert got == exp
    assert DEFAULT_BACKBONE_CLS.supported_architectures == ["transformer", "hybrid"]
    assert BACKBONES["torch"].supported_architectures == ["transformer"]
    tb = BACKBONES["mamba_ssm"](BackboneConfig(**TINY.to_zonos_config()["backbone"]))
    assert {k: tuple(v.shape) for k, v in tb.state_dict().items()} == \
        {k[len("backbone."):]: v for k, v in zonos_ref.weight_shapes(TINY).items() if k.startswith("backbone.")}


def test_from_local_backbone_selector_errors(tmp_path):
    """from_local(backbone=...) as the reference (model.py:69-70): an unknown key raises KeyError, a
    class without the checkpoint's architecture raises -- before any weight is read."""
    import json

    import pytest
    from oracle import hybrid_ref
    from zonos.model import Zonos
    cfg = tmp_path / "config.json"
    cfg.write_text(json.dumps(hybrid_ref.HybridCfg(n_layer=4, attn_layer_idx=(2,)).to_zonos_config()))
    with pytest.raises(KeyError):
        Zonos.from_local(str(cfg), str(tmp_path / "missing.safetensors"), backbone="nope")
    with pytest.raises(ValueError, match="hybrid"):
        Zonos.from_local(str(cfg), str(tmp_path / "missing.safetensors"), backbone="torch")
