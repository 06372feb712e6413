"""`zonos.codebook_pattern` import surface (reference zonos/codebook_pattern.py)."""
from zonos_amd.codebook_pattern import apply_delay_pattern, revert_delay_pattern  # noqa: F401
