"""`zonos.config` import surface (reference zonos/config.py): same dataclasses and field names."""
from zonos_amd.config import BackboneConfig, InferenceParams, PrefixConditionerConfig, ZonosConfig  # noqa: F401
