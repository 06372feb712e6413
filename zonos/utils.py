"""`zonos.utils` import surface (reference zonos/utils.py): DEFAULT_DEVICE, find_multiple,
hub_download (local files / cache only), pad_weight_."""
import torch
import torch.nn.functional as F

from zonos_amd.utils import DEFAULT_DEVICE, find_multiple, get_device, hub_download  # noqa: F401


def pad_weight_(w, multiple: int):
    """utils.py:22-37: pad an nn.Embedding / nn.Linear weight in place by `rows % multiple` rows."""
    if w.weight.shape[0] % multiple == 0:
        return
    w.weight.data = F.pad(w.weight.data, (0, 0, 0, w.weight.shape[0] % multiple))
    if isinstance(w, torch.nn.Embedding):
        w.num_embeddings = w.weight.shape[0]
    elif isinstance(w, torch.nn.Linear):
        w.out_features = w.weight.shape[0]
