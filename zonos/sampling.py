"""`zonos.sampling` import surface (reference zonos/sampling.py): the HIP sampler and the
reference's loggers (`logger` = "zonos.sampling", `trace_logger` = "zonos.sampling.trace")."""
from zonos_amd.sampling import logger, sample_from_logits, trace_logger  # noqa: F401
