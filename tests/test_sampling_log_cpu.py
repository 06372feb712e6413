"""CPU: the reference's sampling loggers (zonos/sampling.py:5-9, 287-322) -- names, gating and
the statistics lines, computed host-side from a logits copy (no GPU compute)."""
import logging

import torch

from zonos_amd import sampling as zs


def _run(capsys, level_main, level_trace, n):
    zs.offset = 0
    zs.distribution.clear()
    zs.num_non_zero_tokens.clear()
    zs.logger.setLevel(level_main)
    zs.trace_logger.setLevel(level_trace)
    g = torch.Generator().manual_seed(0)
    sp = dict(temperature=1.0, top_p=0.0, top_k=0, min_p=0.0, linear=0.65, conf=0.4, quad=0.0,
              repetition_penalty=2.5, repetition_penalty_window=8)
    try:
        for _ in range(n):
            x = torch.randn(1026, generator=g) * 3
            x[1025] = -float("inf")
            zs.log_sampling_stats(x, sp, torch.randint(0, 1024, (20,), generator=g), 2.5, 1024)
    finally:
        zs.logger.setLevel(logging.INFO)
        zs.trace_logger.setLevel(logging.INFO)
    return capsys.readouterr().out.splitlines()


def test_logger_names_match_reference():
    from zonos.sampling import logger, trace_logger
    assert logger.name == "zonos.sampling" and trace_logger.name == "zonos.sampling.trace"
    assert logger is logging.getLogger("zonos.sampling")


def test_silent_unless_debug(capsys):
    assert _run(capsys, logging.INFO, logging.INFO, 130) == []
    assert zs.offset == 0


def test_debug_every_64th(capsys):
    out = _run(capsys, logging.DEBUG, logging.INFO, 130)
    assert out[0].startswith("Temperature: 1.0, Top P: 0.0")
    before = [l for l in out if l.startswith("Before Batch 0, Codebook 0 | Top 5:")]
    after = [l for l in out if l.startswith("After  Batch 0, Codebook 0 | Top 5:")]
    assert len(before) == len(after) == 2 and zs.offset == 130      # calls 64 and 128
    assert "95% mass in:" in after[0] and "p(EOS):" in after[0]
    assert sum("Average number of non-zero tokens" in l for l in out) == 2


def test_trace_every_step(capsys):
    out = _run(capsys, logging.INFO, logging.DEBUG, 5)
    assert sum(l.startswith("Before Batch 0") for l in out) == 5
    # the unified sampler zeroes no finite-logit token (sampling.py:65 clamps before the log)
    nz = [int(l.split("Non-zero:")[1].split("|")[0]) for l in out if l.startswith("After ")]
    assert len(nz) == 5 and all(n >= 1025 for n in nz)
