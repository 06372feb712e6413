"""Backbone registry (reference zonos/backbone/__init__.py:1-12): "hip" = the transformer blocks
on the MI355X kernels, with the reference's plugin interface (zonos_amd/backbone.py)."""
from zonos_amd.backbone import HipZonosBackbone

BACKBONES = {"hip": HipZonosBackbone}
