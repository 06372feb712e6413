"""sample_from_logits on the GPU (zonos/sampling.py:232-328), same signature plus the
noise-stream key (seed, step, draw, row_base); see oracle/philox.py for the stream."""
from __future__ import annotations

import torch

from . import _lib
from ._lib import SamplingParams, call, ptr


def sample_from_logits(logits: torch.Tensor, temperature: float = 1.0, top_p: float = 0.0, top_k: int = 0,
                       min_p: float = 0.0, linear: float = 0.0, conf: float = 0.0, quad: float = 0.0,
                       generated_tokens: torch.Tensor | None = None,
                       repetition_penalty: float | torch.Tensor = 3.0, repetition_penalty_window: int = 2,
                       eos_token_id: int = -1, *, seed: int = 0, step: int = 0, draw: int = 0,
                       row_base: int = 0) -> torch.Tensor:
    _lib.require_gpu(logits, "logits")
    lg = logits.float().contiguous()
    B, K, V = lg.shape
    if not isinstance(repetition_penalty, torch.Tensor):
        repetition_penalty = torch.full((B,), float(repetition_penalty))
    rp = repetition_penalty.to(device=lg.device, dtype=torch.float32).expand(B).contiguous()
    gen = None
    gen_len = 0
    if generated_tokens is not None:
        gen = generated_tokens.to(device=lg.device, dtype=torch.int64).contiguous()
        gen_len = gen.shape[2]
    sp = SamplingParams(float(temperature), float(top_p), float(min_p), float(linear), float(conf), float(quad),
                        int(top_k), int(repetition_penalty_window), 1.0, 0)
    out = torch.empty(B, K, 1, dtype=torch.int64, device=lg.device)
    call("zk_sample_logits", ptr(lg), B, K, V, ptr(gen), gen_len, gen_len, ptr(rp), _lib.C.byref(sp),
         int(seed) & 0xFFFFFFFFFFFFFFFF, int(step), int(draw), int(row_base), ptr(out),
         _lib.stream_ptr(lg.device))
    return out
