"""Configuration dataclasses (mirror of zonos/config.py:8-62; same field names, so the
reference's config.json loads unchanged)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Literal

import torch


@dataclass
class InferenceParams:
    """zonos/config.py:8-25. The HIP backbone keeps seqlen_offset/lengths on the device
    during generate(); this host object is kept for the plugin API (prefill/forward)."""
    max_seqlen: int
    max_batch_size: int
    seqlen_offset: int = 0
    batch_size_offset: int = 0
    key_value_memory_dict: dict = field(default_factory=dict)
    lengths_per_sample: torch.Tensor | None = None

    def reset(self, max_seqlen, max_batch_size):
        self.max_seqlen = max_seqlen
        self.max_batch_size = max_batch_size
        self.seqlen_offset = 0
        if self.lengths_per_sample is not None:
            self.lengths_per_sample.zero_()


@dataclass
class BackboneConfig:
    d_model: int = 1024
    d_intermediate: int = 0
    attn_mlp_d_intermediate: int = 0
    n_layer: int = 16
    ssm_cfg: dict = field(default_factory=dict)
    attn_layer_idx: list = field(default_factory=list)
    attn_cfg: dict = field(default_factory=dict)
    rms_norm: bool = False
    residual_in_fp32: bool = False
    norm_epsilon: float = 1e-5


@dataclass
class PrefixConditionerConfig:
    conditioners: list
    projection: Literal["none", "linear", "mlp"]


@dataclass
class ZonosConfig:
    backbone: BackboneConfig
    prefix_conditioner: PrefixConditionerConfig
    eos_token_id: int = 1024
    masked_token_id: int = 1025
    pad_vocab_to_multiple_of: int = 8

    @classmethod
    def from_dict(cls, d: dict) -> "ZonosConfig":
        d = dict(d)
        bb = BackboneConfig(**d.pop("backbone"))
        pc = PrefixConditionerConfig(**d.pop("prefix_conditioner"))
        return cls(bb, pc, **d)
