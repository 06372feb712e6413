"""Helpers mirrored from zonos/utils.py (find_multiple 7-10, pad_weight_ 22-37,
device selection 39-150, hub lookup 12-19 -- local cache only, there is no network)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F


def find_multiple(n: int, k: int) -> int:
    if k == 0 or n % k == 0:
        return n
    return n + k - (n % k)


def pad_rows_like_reference(w: torch.Tensor, multiple: int) -> torch.Tensor:
    """pad_weight_ on an nn.Linear weight: adds `rows % multiple` zero rows (1025 -> 1026)."""
    if w.shape[0] % multiple == 0:
        return w
    return F.pad(w, (0, 0, 0, w.shape[0] % multiple))


def hub_download(repo_id: str, filename: str, revision: str | None = None) -> str:
    """Resolve a file from the local Hugging Face cache (utils.py:12-19 without the network leg)."""
    if os.path.isdir(repo_id):
        p = os.path.join(repo_id, filename)
        if os.path.exists(p):
            return p
    from huggingface_hub import hf_hub_download
    return hf_hub_download(repo_id=repo_id, filename=filename, revision=revision, local_files_only=True)


def get_device() -> torch.device:
    return torch.device("cuda:0") if torch.cuda.device_count() > 0 else torch.device("cpu")


DEFAULT_DEVICE = get_device()
