"""Backbone registry (reference zonos/backbone/__init__.py:1-12) on the MI355X kernels, with the
reference's plugin interface (zonos_amd/backbone.py):

* "hip_hybrid" -- HipHybridBackbone, supported_architectures ["transformer", "hybrid"] (the role of
  the reference's MambaSSMZonosBackbone: Mamba2 + MHA blocks per attn_layer_idx);
* "hip" -- HipZonosBackbone, ["transformer"] (the role of TorchZonosBackbone).

The reference's own keys are aliases of the same classes, so ``Zonos.from_local(..., backbone="torch")``
or ``backbone="mamba_ssm"`` selects the corresponding HIP backbone. The hybrid-capable class comes
first, as mamba_ssm's does when it is installed (so DEFAULT_BACKBONE_CLS supports both architectures,
gradio_interface.py:213-217)."""
from zonos_amd.backbone import BACKBONES, HipHybridBackbone, HipZonosBackbone  # noqa: F401
