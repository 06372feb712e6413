"""`zonos.sampling` import surface (reference zonos/sampling.py): the HIP sampler."""
from zonos_amd.sampling import sample_from_logits  # noqa: F401
