"""sample_from_logits on the GPU (zonos/sampling.py:232-328), same signature. The race noise is
the reference's own by default: the values `torch.empty_like(probs).exponential_(1)` draws from
torch's CUDA generator (or ``generator=``), which is then advanced exactly as that call advances
it (oracle/torch_philox.py). Passing ``seed=`` selects the engine's keyed stream instead, keyed by
(seed, step, draw, row_base); see oracle/philox.py.

Also the reference's sampling loggers (sampling.py:5-9): ``zonos.sampling`` (DEBUG: the
sampling parameters once, then probability statistics of utterance 0 / codebook 0 every 64th
sampled step) and ``zonos.sampling.trace`` (DEBUG: the same statistics every step). The
sampler runs inside the captured decode step, so the statistics are computed here, on the
host, from a copy of the logits the engine hands over -- only while one of the loggers is
enabled for DEBUG (`debug_enabled()`); the graph path is untouched otherwise. Like the
reference, the loggers gate the output and the lines themselves are printed to stdout."""
from __future__ import annotations

import logging
import math

import torch

from . import _lib
from ._lib import SamplingParams, call, ptr

# the reference's logger names (its module is zonos/sampling.py: __name__ == "zonos.sampling")
logger = logging.getLogger("zonos.sampling")
logger.setLevel(logging.INFO)
trace_logger = logging.getLogger("zonos.sampling.trace")
trace_logger.setLevel(logging.INFO)

LOG_EVERY_NTH = 64          # sampling.py:289
# module-global counters, as the reference keeps them (sampling.py:228-230)
offset = 0
distribution: list = []
num_non_zero_tokens: list = []


def sample_from_logits(logits: torch.Tensor, temperature: float = 1.0, top_p: float = 0.0, top_k: int = 0,
                       min_p: float = 0.0, linear: float = 0.0, conf: float = 0.0, quad: float = 0.0,
                       generated_tokens: torch.Tensor | None = None,
                       repetition_penalty: float | torch.Tensor = 3.0, repetition_penalty_window: int = 2,
                       eos_token_id: int = -1, *, seed: int | None = None, step: int = 0, draw: int = 0,
                       row_base: int = 0, generator: torch.Generator | None = None) -> torch.Tensor:
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
    if debug_enabled():
        log_sampling_stats(lg[0, 0], dict(temperature=temperature, top_p=top_p, top_k=top_k, min_p=min_p,
                                          linear=linear, conf=conf, quad=quad,
                                          repetition_penalty=repetition_penalty,
                                          repetition_penalty_window=repetition_penalty_window),
                           None if gen is None else gen[0, 0], float(rp[0]), eos_token_id)
    out = torch.empty(B, K, 1, dtype=torch.int64, device=lg.device)
    if seed is not None:
        call("zk_sample_logits", ptr(lg), B, K, V, ptr(gen), gen_len, gen_len, ptr(rp), _lib.C.byref(sp),
             int(seed) & 0xFFFFFFFFFFFFFFFF, int(step), int(draw), int(row_base), ptr(out),
             _lib.stream_ptr(lg.device))
        return out
    if step or draw or row_base:
        # the keyed stream's coordinates mean nothing to torch's generator stream: refuse them instead
        # of silently ignoring them (the default changed from the keyed stream to torch's in round 5)
        raise ValueError("step / draw / row_base select a keyed noise stream: pass seed= with them")
    g = generator if generator is not None else torch.cuda.default_generators[_lib.device_index(lg.device)]
    stride, incr = torch_noise_policy(B * K * V, lg.device)
    off = int(g.get_offset())
    call("zk_sample_logits_torch", ptr(lg), B, K, V, ptr(gen), gen_len, gen_len, ptr(rp), _lib.C.byref(sp),
         int(g.initial_seed()) & 0xFFFFFFFFFFFFFFFF, off, stride, ptr(out), _lib.stream_ptr(lg.device))
    if temperature > 0:                  # greedy decoding draws no noise (sampling.py:325-326)
        g.set_offset(off + incr)
    return out


def torch_noise_policy(n: int, device) -> tuple[int, int]:
    """(grid-stride, Philox offset increment) of torch's `exponential_` over n elements on
    ``device`` (zk_torch_noise_policy: DistributionTemplates.h calc_execution_policy)."""
    p = torch.cuda.get_device_properties(device)
    stride, incr = _lib.C.c_int(), _lib.C.c_long()
    rc = _lib.load().zk_torch_noise_policy(int(n), int(p.multi_processor_count),
                                           int(p.max_threads_per_multi_processor), _lib.C.byref(stride),
                                           _lib.C.byref(incr))
    if rc != 0:
        raise _lib.ZonosHipError(f"zk_torch_noise_policy failed: {_lib.load().zk_last_error().decode()}")
    return stride.value, incr.value


# ---------------------------------------------------------------- debug statistics (host side)
def debug_enabled() -> bool:
    return logger.isEnabledFor(logging.DEBUG) or trace_logger.isEnabledFor(logging.DEBUG)


def _shape_probs(probs: torch.Tensor, sp: dict) -> torch.Tensor:
    """The probability shaping of sampling.py:310-318 on one [V] row (statistics only)."""
    if sp.get("linear", 0) > 0:                                     # apply_unified 54-75
        lp = torch.log(probs.clamp_min(1e-20))
        ent = -torch.sum(probs * lp)
        probs = (lp * (sp["linear"] + ent * sp.get("conf", 0.0)) - lp ** 2 * sp.get("quad", 0.0)).softmax(-1)
    if sp.get("top_p", 0) > 0:                                      # apply_top_p 96-111
        ps, pi = torch.sort(probs, descending=True)
        keep = ~((torch.cumsum(ps, 0) - ps) > sp["top_p"])
        probs = probs.scatter(0, pi, ps * keep.float())
        probs = probs / probs.sum()
    if sp.get("top_k", 0) > 0:                                      # apply_top_k 77-93
        v, _ = torch.topk(probs, min(int(sp["top_k"]), probs.numel()))
        probs = torch.where(probs < v[-1], 0.0, probs)
        probs = probs / probs.sum()
    if sp.get("min_p", 0) > 0:                                      # apply_min_p 114-128
        probs = probs.masked_fill(probs < sp["min_p"] * probs.max(), 0.0)
        probs = probs / probs.sum()
    return probs


def _prob_stats_line(p: torch.Tensor, top_k: int, mass: float, before: bool, eos_token_id: int) -> tuple[str, int, int]:
    """print_prob_stats (sampling.py:206-226) for utterance 0 / codebook 0."""
    tp, ti = torch.topk(p, k=top_k)
    nnz = int((p > 0).sum())
    sp_, _ = torch.sort(p, descending=True)
    to_mass = int((torch.cumsum(sp_, 0) < mass).sum()) + 1
    tag = "Before" if before else "After "
    eos = f"p(EOS): {float(p[eos_token_id]):.3f} | " if eos_token_id != -1 else ""
    line = (f"{tag} Batch 0, Codebook 0 | Top {top_k}: [{', '.join(f'{t:>4}' for t in ti.tolist())}] | "
            f"Probs: [{', '.join(f'{v:.3f}' for v in tp.tolist())}] | Non-zero: {nnz:>4} | "
            f"{int(mass * 100)}% mass in: {to_mass:>4} tokens | {eos}{tag}")
    return line, to_mass, nnz


def log_sampling_stats(logits_row: torch.Tensor, sp: dict, generated_row: torch.Tensor | None, rp: float,
                       eos_token_id: int = -1) -> None:
    """Statistics of one sampler call for utterance 0 / codebook 0 (sampling.py:284-322), logged
    through the reference's loggers. ``logits_row`` [V] are the logits the sampler receives
    (after bias and EOS masks); the repetition penalty is applied here as sampling.py:131-169 does."""
    global offset
    debug = logger.isEnabledFor(logging.DEBUG)
    trace = trace_logger.isEnabledFor(logging.DEBUG)
    if not (debug or trace):
        return
    x = logits_row.detach().float().cpu().clone()
    V = x.numel()
    if offset == 0 and debug:
        print(f"Temperature: {sp['temperature']}, Top P: {sp['top_p']}, Top K: {sp['top_k']}, "
              f"Min P: {sp['min_p']}, Linear: {sp['linear']}, Conf: {sp['conf']}, Quad: {sp['quad']} | "
              f"RepPen: {sp['repetition_penalty']}, RepPenWindow: {sp['repetition_penalty_window']}")
    W = int(sp.get("repetition_penalty_window", 0))
    if rp != 1.0 and generated_row is not None and W > 0:
        g = generated_row.detach().cpu()[-W:].clamp_max(V - 1).long()
        f = torch.ones(V).scatter_reduce(0, g, torch.full((g.numel(),), float(rp)), reduce="prod")
        x = torch.where(x <= 0, x * f, x / f)
    temperature = float(sp["temperature"])
    if temperature <= 0:
        return
    probs = torch.softmax(x / temperature, dim=-1)
    offset += 1
    debug = debug and offset % LOG_EVERY_NTH == 0
    if not (debug or trace):
        return
    mass = sp["top_p"] if sp.get("top_p", 0) > 0 else 0.95
    line, _, _ = _prob_stats_line(probs, 5, mass, True, eos_token_id)
    print(line)
    probs = _shape_probs(probs, sp)
    line, to_mass, nnz = _prob_stats_line(probs, 5, mass, False, eos_token_id)
    print(line)
    distribution.append(to_mass)
    num_non_zero_tokens.append(nnz)
    print(f"  Average number of tokens to choose top 95%: {sum(distribution) / len(distribution):.2f}")
    print(f"  Average number of non-zero tokens: {sum(num_non_zero_tokens) / len(num_non_zero_tokens):.2f}")


def engine_logits_row(cfg_logits_row: torch.Tensor, prefill: bool, eos_active: bool, eos_token_id: int = 1024,
                      force_full_length: bool = False) -> torch.Tensor:
    """The logits utterance 0 / codebook 0 hands to the sampler in generate(): the engine's fp32
    CFG logits plus the EOS bias of model.py:322-324,353 and the hold-off mask of model.py:360-361."""
    x = cfg_logits_row.detach().float().cpu().clone()
    if not prefill:
        x[eos_token_id] = x[eos_token_id] - math.log(1024.0)
        if eos_active:
            x[eos_token_id] = -math.inf
    if force_full_length:
        x[eos_token_id] = -math.inf
    return x
