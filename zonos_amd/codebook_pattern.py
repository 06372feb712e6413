"""Delay pattern on the GPU (zonos/codebook_pattern.py:5-12) via zk_delay_apply/revert."""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, ptr


def apply_delay_pattern(codes: torch.Tensor, mask_token: int) -> torch.Tensor:
    _lib.require_gpu(codes, "codes")
    codes = codes.to(torch.int64).contiguous()
    B, K, T = codes.shape
    out = torch.empty(B, K, T + K, dtype=torch.int64, device=codes.device)
    call("zk_delay_apply", ptr(codes), B, K, T, int(mask_token), ptr(out), _lib.stream_ptr(codes.device))
    return out


def revert_delay_pattern(codes: torch.Tensor) -> torch.Tensor:
    _lib.require_gpu(codes, "codes")
    codes = codes.to(torch.int64).contiguous()
    B, K, L = codes.shape
    out = torch.empty(B, K, L - K, dtype=torch.int64, device=codes.device)
    call("zk_delay_revert", ptr(codes), B, K, L, ptr(out), _lib.stream_ptr(codes.device))
    return out
