"""`zonos.utils` import surface (reference zonos/utils.py): DEFAULT_DEVICE, find_multiple,
hub_download (local files / cache only), pad_weight_."""
import torch
import torch.nn.functional as F

from zonos_amd.utils import DEFAULT_DEVICE, find_multiple, get_device, hub_download  # noqa: F401


def pad_weight_(w, multiple: int):
    """utils.py:22-37, branch for branch.

    nn.Embedding: tested on dim 1 (embedding_dim) but padded by `embedding_dim % multiple`
    ROWS (the reference's own quirk -- Embedding(1026, 2048) is left alone); nn.Linear: tested
    and padded on dim 0 (out_features) by `out_features % multiple` rows (Linear(2048, 1025)
    with multiple 8 -> 1026 rows). Both branches reset both dims; other types raise
    ValueError."""
    if isinstance(w, torch.nn.Embedding):
        if w.weight.shape[1] % multiple == 0:
            return
        w.weight.data = F.pad(w.weight.data, (0, 0, 0, w.weight.shape[1] % multiple))
        w.num_embeddings, w.embedding_dim = w.weight.shape
    elif isinstance(w, torch.nn.Linear):
        if w.weight.shape[0] % multiple == 0:
            return
        w.weight.data = F.pad(w.weight.data, (0, 0, 0, w.weight.shape[0] % multiple))
        w.out_features, w.in_features = w.weight.shape
    else:
        raise ValueError(f"Unsupported weight type: {type(w)}")
