"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py

The reference package is imported from /root/reference with import-only stubs for
the front-end libraries that are absent here (torchaudio, inflect, kanjize,
phonemizer, sudachipy) -- they are not on the decode path. The reference's DAC
wrapper normally fetches "descript/dac_44khz" by name (autoencoder.py:15); offline we
build transformers' DacModel locally and load the same synthetic weights the oracle
uses (oracle.dac_ref.make_dac_weights).

Sampling noise: the reference draws Exp(1) noise from torch's generator in
zonos.sampling.multinomial (sampling.py:26-28). We replace that one function with
one that takes the engine's counter-based stream (oracle.philox.exp_noise), keyed by
(step, draw) exactly as the engine keys it, so seeded sampling is comparable.
Everything else runs unmodified reference code.

Outputs are small .npz files (inputs + expected outputs only); weights are
regenerated deterministically from their seeds by oracle.zonos_ref.make_weights /
oracle.dac_ref.make_dac_weights, and a checksum of them is stored for verification.
"""
from __future__ import annotations

import hashlib
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import transformers.models.dac.modeling_dac  # noqa: E402,F401  (before the torchaudio stub)
from transformers import DacConfig, DacModel  # noqa: E402


class _Any:
    def __init__(self, *a, **k): pass
    def __call__(self, *a, **k): return _Any()
    def __getattr__(self, n): return _Any()


class _Stub(types.ModuleType):
    def __getattr__(self, n):
        if n.startswith("__"):
            raise AttributeError(n)
        return _Any


for _m in ["torchaudio", "torchaudio.functional", "inflect", "kanjize", "phonemizer",
           "phonemizer.backend", "sudachipy"]:
    sys.modules[_m] = _Stub(_m)
sys.path.insert(0, "/root/reference")

import zonos.autoencoder as zae  # noqa: E402
import zonos.model as zm  # noqa: E402
import zonos.sampling as zs  # noqa: E402
from zonos.backbone import BACKBONES  # noqa: E402
from zonos.codebook_pattern import apply_delay_pattern, revert_delay_pattern  # noqa: E402
from zonos.config import ZonosConfig  # noqa: E402

from oracle import dac_ref, zonos_ref  # noqa: E402
from oracle.philox import exp_noise  # noqa: E402

TINY = zonos_ref.BackboneCfg(d_model=256, n_layer=2, n_heads=2, n_kv=1, d_ff=512)
TINY_DAC = dac_ref.DacCfg(hidden_size=64, decoder_hidden_size=64, upsampling_ratios=(4, 2))


def wsum(W: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(W):
        h.update(k.encode())
        h.update(W[k].float().contiguous().numpy().tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------- noise injection
class NoiseCtl:
    seed = 0
    step = 0
    draw = 0
    row_base = 0


def _patched_multinomial(input, num_samples, replacement=False, *, generator=None):
    assert num_samples == 1
    B, K, V = input.shape
    q = torch.from_numpy(exp_noise(NoiseCtl.seed, NoiseCtl.step, NoiseCtl.draw, B, K, V, NoiseCtl.row_base))
    return torch.argmax(input / q, dim=-1, keepdim=True).to(torch.int64)


zs.multinomial = _patched_multinomial
_orig_sample = zm.sample_from_logits
_last_off = {"v": None}


def _tracking_sample(logits, generated_tokens=None, **kw):
    """Map each reference sampler call to the engine's (step, draw) key."""
    if generated_tokens is None:
        NoiseCtl.step, NoiseCtl.draw = 0, 0
        _last_off["v"] = None
    else:
        off = generated_tokens.shape[2]
        if _last_off["v"] == off:
            NoiseCtl.draw = 1
        else:
            NoiseCtl.step += 1
            NoiseCtl.draw = 0
        _last_off["v"] = off
    return _orig_sample(logits, generated_tokens=generated_tokens, **kw)


zm.sample_from_logits = _tracking_sample


# ---------------------------------------------------------------- reference model build
def _dac_init(self):
    self.dac = DacModel(DacConfig(sampling_rate=44100))
    self.dac.eval().requires_grad_(False)
    self.codebook_size = self.dac.config.codebook_size
    self.num_codebooks = self.dac.quantizer.n_codebooks
    self.sampling_rate = self.dac.config.sampling_rate


zae.DACAutoencoder.__init__ = _dac_init


def build_ref_model(cfg, W):
    zc = ZonosConfig.from_dict(cfg.to_zonos_config())
    model = zm.Zonos(zc, BACKBONES["torch"]).to(torch.bfloat16)
    sd = model.state_dict()
    for k, v in W.items():
        sd[k] = v
    model.load_state_dict(sd)   # post-hook pads heads 1025 -> 1026 (model.py:46-51)
    model.eval()
    return model


def run_generate(model, cond, prefix, B, max_new, sp, seed, logits_steps=0):
    """Reference generate with the engine's noise; records the CFG logits of the first
    ``logits_steps`` steps (an int) or of the given step indices (a tuple)."""
    NoiseCtl.seed = seed
    rec = []
    orig = model._compute_logits
    n_call = [0]

    def rec_logits(*a, **k):
        out = orig(*a, **k)
        i = n_call[0]
        n_call[0] += 1
        if (i < logits_steps) if isinstance(logits_steps, int) else (i in logits_steps):
            rec.append(out.clone())
        return out

    model._compute_logits = rec_logits
    out = model.generate(cond, audio_prefix_codes=prefix, max_new_tokens=max_new, cfg_scale=2.0,
                         batch_size=B, sampling_params=sp, progress_bar=False, disable_torch_compile=True)
    model._compute_logits = orig
    return out, rec


def pack_codes(lst):
    T = max(int(x.shape[1]) for x in lst) if lst else 0
    arr = np.full((len(lst), 9, T), -1, dtype=np.int16)
    lens = np.zeros(len(lst), dtype=np.int32)
    for i, x in enumerate(lst):
        arr[i, :, :x.shape[1]] = x.numpy()
        lens[i] = x.shape[1]
    return arr, lens


GEN_CASES = {
    "greedy": dict(sp=dict(temperature=0.0, top_p=0, top_k=0, min_p=0, linear=0.0, conf=0.0, quad=0.0,
                           repetition_penalty=1.0, repetition_penalty_window=2), eos_bias=0.0, logits=6),
    "greedy_rep": dict(sp=dict(temperature=0.0, top_p=0, top_k=0, min_p=0, linear=0.0, conf=0.0, quad=0.0,
                               repetition_penalty=2.5, repetition_penalty_window=8), eos_bias=0.0, logits=0),
    "sampled_cli": dict(sp=dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0,
                                repetition_penalty=2.5, repetition_penalty_window=8, temperature=1.0),
                        eos_bias=0.0, logits=0),
    "sampled_knobs": dict(sp=dict(top_p=0.9, top_k=50, min_p=0.05, linear=0.0, conf=0.0, quad=0.0,
                                  repetition_penalty=1.5, repetition_penalty_window=4, temperature=0.8),
                          eos_bias=0.0, logits=0),
    "eos_greedy": dict(sp=dict(temperature=0.0, top_p=0, top_k=0, min_p=0, linear=0.0, conf=0.0, quad=0.0,
                               repetition_penalty=1.0, repetition_penalty_window=2), eos_bias=10.0, logits=0),
    "eos_sampled": dict(sp=dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0,
                                repetition_penalty=2.5, repetition_penalty_window=8, temperature=1.0),
                        eos_bias=10.0, logits=0),
}
GEN_B, GEN_LC, GEN_P, GEN_NEW, HEAD_SCALE = 3, 12, 4, 40, 4.0


def make_generate_fixtures():
    cond = zonos_ref.synthetic_conditioning(GEN_B, GEN_LC, TINY.d_model, seed=1)
    prefix = zonos_ref.synthetic_prefix_codes(GEN_B, GEN_P, seed=3)
    for name, case in GEN_CASES.items():
        W = zonos_ref.make_weights(TINY, seed=0, head_scale=HEAD_SCALE, eos_bias=case["eos_bias"])
        model = build_ref_model(TINY, W)
        seed = 1234
        out, rec = run_generate(model, cond, prefix, GEN_B, GEN_NEW, case["sp"], seed, case["logits"])
        # oracle cross-check right here (same container, same torch): must be bit-identical.
        trace = {}
        Wp = zonos_ref.pad_heads(W, TINY)
        out_o = zonos_ref.generate(Wp, TINY, cond, prefix, GEN_NEW, 2.0, GEN_B, case["sp"], seed=seed,
                                   trace=trace)
        same = all(torch.equal(a, b) for a, b in zip(out, out_o)) and len(out) == len(out_o)
        codes, lens = pack_codes(out)
        print(f"[gen:{name}] lens={lens.tolist()} oracle_match={same}")
        assert same, f"oracle diverges from reference on {name}"
        d = dict(codes=codes, lens=lens, cond=cond.view(torch.int16).numpy(), prefix=prefix.numpy().astype(np.int16),
                 seed=np.int64(seed), wsum=np.array(wsum(W)), eos_bias=np.float32(case["eos_bias"]),
                 head_scale=np.float32(HEAD_SCALE), max_new=np.int32(GEN_NEW),
                 delayed=trace["delayed"].numpy().astype(np.int16), offset=np.int32(trace["offset"]))
        for k, v in case["sp"].items():
            d["sp_" + k] = np.float64(v)
        if rec:
            d["logits"] = torch.stack(rec).numpy().astype(np.float32)
        np.savez_compressed(os.path.join(HERE, f"gen_{name}.npz"), **d)


def decision_margins(trace) -> np.ndarray:
    """[steps, B, 9] min over the draws of a step of the oracle's top-1/top-2 decision margin
    (logit units for greedy, log-ratio of probs/noise for sampling)."""
    out = []
    for dec in trace["decision"]:
        ms = []
        for kind, arr in dec:
            top = arr.topk(2, dim=-1).values
            ms.append((top[..., 0] - top[..., 1]) if kind == "logit"
                      else torch.log(top[..., 0] / top[..., 1].clamp_min(1e-38)))
        out.append(torch.stack(ms).min(dim=0).values.float())
    return torch.stack(out).numpy()


COPY_GAIN = 1.0
COPY_FIX = {   # name: (sampling, weight seed, eos trigger steps of utterance 0's cb0 chain)
    "copy_greedy": (GEN_CASES["greedy"]["sp"], 0, ()),
    "copy_rep": (GEN_CASES["greedy_rep"]["sp"], 2, ()),      # seed 2: the penalty bites with margin
    "copy_eos": (GEN_CASES["greedy"]["sp"], 0, (12, 24)),    # 1st EOS resampled (hold-off), 2nd accepted
}


def make_copy_fixtures():
    """Free-running greedy fixtures on copy heads (zonos_ref.make_copy_weights) at D=1024, run by
    the reference; the margins of every decision are stored for the tests to check."""
    from tests.golden_util import COPY
    cond = zonos_ref.synthetic_conditioning(GEN_B, GEN_LC, COPY.d_model, seed=1)
    prefix = zonos_ref.synthetic_prefix_codes(GEN_B, GEN_P, seed=3)
    for name, (sp, wseed, eos_steps) in COPY_FIX.items():
        eos_tokens = ()
        if eos_steps:
            chain = zonos_ref.copy_chain(zonos_ref.make_copy_weights(COPY, seed=wseed, copy_gain=COPY_GAIN), COPY, 0,
                                         int(prefix[0, 0, -1]), max(eos_steps) + 1)
            eos_tokens = tuple(chain[i] for i in eos_steps)
        W = zonos_ref.make_copy_weights(COPY, seed=wseed, copy_gain=COPY_GAIN, eos_tokens=eos_tokens)
        model = build_ref_model(COPY, W)
        seed = 1234
        out, rec = run_generate(model, cond, prefix, GEN_B, GEN_NEW, sp, seed, 2)
        trace = {}
        out_o = zonos_ref.generate(zonos_ref.pad_heads(W, COPY), COPY, cond, prefix, GEN_NEW, 2.0, GEN_B, sp,
                                   seed=seed, trace=trace)
        same = len(out) == len(out_o) and all(torch.equal(a, b) for a, b in zip(out, out_o))
        m = decision_margins(trace)
        codes, lens = pack_codes(out)
        print(f"[gen:{name}] lens={lens.tolist()} oracle_match={same} min margin {m.min():.3f}")
        assert same, f"oracle diverges from reference on {name}"
        d = dict(codes=codes, lens=lens, cond=cond.view(torch.int16).numpy(), prefix=prefix.numpy().astype(np.int16),
                 seed=np.int64(seed), wsum=np.array(wsum(W)), wseed=np.int64(wseed), copy_gain=np.float32(COPY_GAIN),
                 eos_tokens=np.array(eos_tokens, dtype=np.int64), max_new=np.int32(GEN_NEW),
                 delayed=trace["delayed"].numpy().astype(np.int16), offset=np.int32(trace["offset"]),
                 margins=m.astype(np.float32), logits=torch.stack(rec).numpy().astype(np.float32))
        for k, v in sp.items():
            d["sp_" + k] = np.float64(v)
        np.savez_compressed(os.path.join(HERE, f"gen_{name}.npz"), **d)


# Edge shapes of generate() (model.py:264-301 sizes every buffer from P and max_new_tokens): no audio
# prefix, one new token, fewer new tokens than codebooks (the delay pattern's diagonal never
# completes), exactly 9 / 10, odd batch sizes. Copy heads, greedy: every decision has a wide margin.
EDGE_CASES = [  # (B, P, max_new, Lc)
    (1, 0, 1, 5), (1, 0, 9, 8), (2, 4, 2, 12), (3, 1, 10, 7), (2, 0, 17, 3), (1, 6, 5, 12),
]


def make_edge_fixtures():
    from tests.golden_util import COPY
    sp = GEN_CASES["greedy"]["sp"]
    W = zonos_ref.make_copy_weights(COPY, seed=0, copy_gain=COPY_GAIN)
    model = build_ref_model(COPY, W)
    d = dict(wsum=np.array(wsum(W)), copy_gain=np.float32(COPY_GAIN), n=np.int32(len(EDGE_CASES)))
    for i, (B, P, max_new, Lc) in enumerate(EDGE_CASES):
        cond = zonos_ref.synthetic_conditioning(B, Lc, COPY.d_model, seed=10 + i)
        prefix = zonos_ref.synthetic_prefix_codes(B, P, seed=20 + i) if P else None
        seed = 77 + i
        out, _ = run_generate(model, cond, prefix, B, max_new, sp, seed, 0)
        trace = {}
        out_o = zonos_ref.generate(zonos_ref.pad_heads(W, COPY), COPY, cond, prefix, max_new, 2.0, B, sp,
                                   seed=seed, trace=trace)
        same = len(out) == len(out_o) and all(torch.equal(a, b) for a, b in zip(out, out_o))
        m = decision_margins(trace)
        codes, lens = pack_codes(out)
        print(f"[gen:edge{i}] B={B} P={P} new={max_new} lens={lens.tolist()} oracle_match={same} "
              f"min margin {m.min():.3f}")
        assert same, f"oracle diverges from reference on edge case {i}"
        d.update({f"e{i}_shape": np.array([B, P, max_new, Lc, seed], dtype=np.int64),
                  f"e{i}_cond": cond.view(torch.int16).numpy(), f"e{i}_codes": codes, f"e{i}_lens": lens,
                  f"e{i}_margins": m.astype(np.float32), f"e{i}_delayed": trace["delayed"].numpy().astype(np.int16)})
        if P:
            d[f"e{i}_prefix"] = prefix.numpy().astype(np.int16)
    for k, v in sp.items():
        d["sp_" + k] = np.float64(v)
    np.savez_compressed(os.path.join(HERE, "gen_edge.npz"), **d)


def ref_forced_steps(model, cond, delayed, P, windows, sp, seed, row_base):
    """The reference's own prefill (model.py:181-202) over a forced history, then its single-token
    decode (model.py:118-142), its logit bias (332-334, EOS never accepted: benchmark mode) and
    sample_from_logits with the engine's noise key. Mirrors zonos_ref.forced_steps."""
    import zonos.sampling as zs_
    R, Lc, _ = cond.shape
    B = R // 2
    rp = float(sp["repetition_penalty"])
    spk = {k: v for k, v in sp.items() if k != "repetition_penalty"}
    out = {}
    for s0, n in windows:
        ip = model.setup_cache(batch_size=R, max_seqlen=Lc + delayed.shape[2] + 9)
        logits = model._prefill(cond, delayed[..., :P + 1 + s0], ip, 2.0)
        ip.seqlen_offset += Lc + P + 1 + s0
        ip.lengths_per_sample[:] += Lc + P + 1 + s0
        for j in range(n):
            s = s0 + j
            off = P + 1 + s
            if j > 0:
                logits = model._decode_one_token(delayed[..., off - 1:off], ip, torch.tensor(2.0), allow_cudagraphs=False)
                ip.seqlen_offset += 1
                ip.lengths_per_sample[:] += 1
            raw = logits.clone()
            lg = logits.clone()
            if s > 0:
                lg[:, 1:, 1024] = -torch.inf
                lg[:, 0, 1024] -= torch.log(torch.tensor(1024.0))
            lg[:, 0, 1024] = -torch.inf
            NoiseCtl.seed, NoiseCtl.step, NoiseCtl.draw, NoiseCtl.row_base = seed, s, 0, row_base
            tok = zs_.sample_from_logits(lg, generated_tokens=delayed[..., :off] if s > 0 else None,
                                         repetition_penalty=torch.full((B,), rp), eos_token_id=1024, **spk)
            out[s] = (raw.detach(), tok[..., 0].detach())
    NoiseCtl.row_base = 0
    return out


def make_full_fixtures(which=("c1", "c2", "c3")):
    """Full-width (D=2048, 26 layers) fixtures of SURVEY §8(d) c1/c2/c3, run by the reference
    (about 5 min on 8 cores). c1: free-running greedy on copy heads. c2/c3: teacher-forced windows
    on a seeded synthetic history, CLI sampling, random weights; only the utterances in `utts`."""
    from tests.golden_util import CLI_SP, FULL, FULL_CASES, FULL_SEED, GREEDY_SP, forced_history, full_weights
    for name in which:
        c = FULL_CASES[name]
        B, Lc, P, T = c["B"], c["Lc"], c["P"], c["T"]
        cond = zonos_ref.synthetic_conditioning(B, Lc, FULL.d_model, seed=c.get("cond_seed", 1))
        prefix = zonos_ref.synthetic_prefix_codes(B, P, seed=c.get("prefix_seed", 3)) if P else None
        rb = c.get("row_base", 0)
        W = full_weights("copy" if name == "c1" else "random")
        model = build_ref_model(FULL, {k: (v[:1025] if k.startswith("heads") else v) for k, v in W.items()})
        d = dict(seed=np.int64(FULL_SEED))
        if name == "c1":
            out, rec = run_generate(model, cond, prefix, B, T, GREEDY_SP, FULL_SEED, tuple(c["logit_steps"]))
            trace = {}
            out_o = zonos_ref.generate(W, FULL, cond, prefix, T, 2.0, B, GREEDY_SP, seed=FULL_SEED, trace=trace)
            same = all(torch.equal(a, b) for a, b in zip(out, out_o))
            m = decision_margins(trace)
            codes, lens = pack_codes(out)
            print(f"[full c1] lens={lens.tolist()} oracle_match={same} min margin {m.min():.3f}")
            assert same
            d.update(codes=codes, lens=lens, margins=m.astype(np.float32), logits=torch.stack(rec).numpy(),
                     delayed=trace["delayed"].numpy().astype(np.int16), offset=np.int32(trace["offset"]))
        else:
            hist = forced_history(B, P, c.get("hist_T", T), prefix, seed=c.get("hist_seed", 7))
            logits, toks, margins, steps = [], [], [], []
            for u in c["utts"]:
                cu = torch.cat([cond[u:u + 1], cond[B + u:B + u + 1]])
                r = ref_forced_steps(model, cu, hist[u:u + 1], P, c["windows"], CLI_SP, FULL_SEED, rb + u)
                o = zonos_ref.forced_steps(W, FULL, cu, hist[u:u + 1], P, c["windows"], CLI_SP, FULL_SEED, rb + u)
                steps = sorted(r)
                for s in steps:
                    assert torch.equal(r[s][0], o[s][0]) and torch.equal(r[s][1], o[s][1]), (name, u, s)
                logits.append(torch.stack([r[s][0][0] for s in c["logit_steps"]]))
                toks.append(torch.stack([r[s][1][0] for s in steps]))
                margins.append(torch.stack([o[s][2][0] for s in steps]))
                print(f"[full {name}] utt {u}: {len(steps)} steps, oracle bit-exact, "
                      f"min margin {float(torch.stack(margins[-1:]).min()):.3f}")
            d.update(steps=np.array(steps, dtype=np.int32), logits=torch.stack(logits).numpy(),
                     tokens=torch.stack(toks).numpy().astype(np.int16), margins=torch.stack(margins).numpy())
        np.savez_compressed(os.path.join(HERE, f"gen_full_{name}.npz"), **d)


SAMPLER_CASES = [
    dict(temperature=0.0, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=0.0, repetition_penalty=2.5, repetition_penalty_window=8),
    dict(temperature=1.0, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=0.7, repetition_penalty=3.0, repetition_penalty_window=2),
    dict(temperature=1.0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5, repetition_penalty_window=8),
    dict(temperature=1.0, linear=0.5, conf=0.2, quad=0.3, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=1.0, top_p=0.8, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=1.0, top_k=20, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=1.0, top_k=1, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=1.0, min_p=0.1, repetition_penalty=1.0, repetition_penalty_window=2),
    dict(temperature=0.9, top_p=0.95, top_k=64, min_p=0.02, linear=0.6, conf=0.3, quad=0.1,
         repetition_penalty=2.0, repetition_penalty_window=6),
]


def make_sampler_fixtures():
    g = torch.Generator().manual_seed(11)
    B, K, V, L = 4, 9, 1026, 12
    out = {}
    for ci, sp in enumerate(SAMPLER_CASES):
        logits = torch.randn(B, K, V, generator=g) * 3.0
        logits[..., 1025:] = -torch.inf
        logits[1, 3, 5] = -torch.inf
        gen = torch.randint(0, 1026, (B, K, L), generator=g)
        gen[..., -3:] = torch.argmax(logits, dim=-1, keepdim=True)   # make the penalty bite
        rp = torch.tensor([sp["repetition_penalty"], 1.0, sp["repetition_penalty"], sp["repetition_penalty"]])
        NoiseCtl.seed, NoiseCtl.step, NoiseCtl.draw = 77, ci + 1, 0
        kw = {k: v for k, v in sp.items() if k != "repetition_penalty"}
        tok = zs.sample_from_logits(logits.clone(), generated_tokens=gen, repetition_penalty=rp.clone(), **kw)
        # oracle
        q = torch.from_numpy(exp_noise(77, ci + 1, 0, B, K, V))
        tok_o = zonos_ref.sample(logits.clone(), q, generated_tokens=gen, repetition_penalty=rp.clone(), **kw)
        assert torch.equal(tok, tok_o), f"sampler oracle mismatch case {ci}"
        out[f"logits_{ci}"] = logits.numpy()
        out[f"gen_{ci}"] = gen.numpy().astype(np.int16)
        out[f"rp_{ci}"] = rp.numpy()
        out[f"tok_{ci}"] = tok.squeeze(-1).numpy().astype(np.int16)
        for k, v in sp.items():
            out[f"sp_{ci}_{k}"] = np.float64(v)
    out["n_cases"] = np.int32(len(SAMPLER_CASES))
    out["seed"] = np.int64(77)
    np.savez_compressed(os.path.join(HERE, "sampler.npz"), **out)
    print(f"[sampler] {len(SAMPLER_CASES)} cases ok")


def make_delay_fixtures():
    g = torch.Generator().manual_seed(5)
    codes = torch.randint(0, 1024, (2, 9, 7), generator=g)
    codes[1, :, 4:] = -1
    d = apply_delay_pattern(codes, 1025)
    r = revert_delay_pattern(d)
    assert torch.equal(d, zonos_ref.apply_delay(codes)) and torch.equal(r, zonos_ref.revert_delay(d))
    np.savez_compressed(os.path.join(HERE, "delay.npz"), codes=codes.numpy().astype(np.int16),
                        delayed=d.numpy().astype(np.int16), reverted=r.numpy().astype(np.int16))
    print("[delay] ok")


def make_dac_fixtures():
    for name, c, T, seed in (("dac_tiny", TINY_DAC, (20, 13), 4), ("dac_44k", dac_ref.DAC_44KHZ, (12, 7), 0)):
        W = dac_ref.make_dac_weights(c, seed=seed)
        hf = DacModel(DacConfig(sampling_rate=44100, hidden_size=c.hidden_size,
                                decoder_hidden_size=c.decoder_hidden_size,
                                upsampling_ratios=list(c.upsampling_ratios),
                                n_codebooks=c.n_codebooks, codebook_size=c.codebook_size,
                                codebook_dim=c.codebook_dim))
        sd = hf.state_dict()
        for k, v in W.items():
            assert sd[k].shape == v.shape, (k, sd[k].shape, v.shape)
            sd[k] = v
        hf.load_state_dict(sd)
        hf.eval()
        g = torch.Generator().manual_seed(seed + 100)
        codes = torch.randint(0, c.codebook_size, (2, c.n_codebooks, T[0]), generator=g)
        short = codes[1:, :, :T[1]].clone()
        with torch.no_grad():
            wav_b = hf.decode(audio_codes=codes).audio_values.unsqueeze(1).float()   # autoencoder.py:47 (CPU)
            wav_s = hf.decode(audio_codes=short).audio_values.unsqueeze(1).float()
        o_b = dac_ref.decode(W, c, codes)
        o_s = dac_ref.decode(W, c, short)
        eb = (o_b - wav_b).abs().max().item()
        es = (o_s - wav_s).abs().max().item()
        print(f"[{name}] rms={wav_b.pow(2).mean().sqrt().item():.4f} oracle max|d| batch={eb:.2e} short={es:.2e}")
        assert eb < 1e-5 and es < 1e-5
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), codes=codes.numpy().astype(np.int16),
                            wav=wav_b.numpy(), wav_short=wav_s.numpy(), short_len=np.int32(T[1]),
                            seed=np.int64(seed), wsum=np.array(wsum(W)),
                            cfg=np.array([c.hidden_size, c.decoder_hidden_size, *c.upsampling_ratios]))


def _q16(w: torch.Tensor):
    """int16 quantisation of a waveform, scale = max|w| / 32767: the rounding error's RMS is
    scale / sqrt(12) (~3e-6 at the fixture's amplitude), far below the 1e-4 RMS parity bar."""
    scale = max(float(w.abs().max()), 1e-30) / 32767.0
    return torch.round(w / scale).to(torch.int16).numpy(), np.float64(scale)


def make_dac_long_fixture():
    """A 44.1 kHz DacModel decode long enough that the channels-last convs stream several tiles per
    persistent workgroup (the c3 regime): 2 ragged rows of 600 / 437 frames (307,200 samples), the
    short row also decoded alone. Waveforms are stored int16-quantised with their scales (_q16)."""
    c, seed, T = dac_ref.DAC_44KHZ, 0, (600, 437)
    W = dac_ref.make_dac_weights(c, seed=seed)
    hf = DacModel(DacConfig(sampling_rate=44100, hidden_size=c.hidden_size,
                            decoder_hidden_size=c.decoder_hidden_size, upsampling_ratios=list(c.upsampling_ratios),
                            n_codebooks=c.n_codebooks, codebook_size=c.codebook_size, codebook_dim=c.codebook_dim))
    sd = hf.state_dict()
    for k, v in W.items():
        sd[k] = v
    hf.load_state_dict(sd)
    hf.eval()
    g = torch.Generator().manual_seed(seed + 300)
    codes = torch.randint(0, c.codebook_size, (2, c.n_codebooks, T[0]), generator=g)
    short = codes[1:, :, :T[1]].clone()
    with torch.no_grad():
        wav_b = hf.decode(audio_codes=codes).audio_values.unsqueeze(1).float()   # autoencoder.py:47 (CPU)
        wav_s = hf.decode(audio_codes=short).audio_values.unsqueeze(1).float()
    o_s = dac_ref.decode(W, c, short)                    # the oracle on the short row (the long one: same code)
    es = (o_s - wav_s).abs().max().item()
    print(f"[dac_44k_long] rms={wav_b.pow(2).mean().sqrt().item():.4f} oracle max|d| short={es:.2e}")
    assert es < 1e-5
    qb, sb = _q16(wav_b)
    qs, ss = _q16(wav_s)
    np.savez_compressed(os.path.join(HERE, "dac_44k_long.npz"), codes=codes.numpy().astype(np.int16),
                        wav_q=qb, wav_scale=sb, wav_short_q=qs, wav_short_scale=ss, short_len=np.int32(T[1]),
                        seed=np.int64(seed), wsum=np.array(wsum(W)))


ENC_DAC = dac_ref.DacCfg(hidden_size=64, decoder_hidden_size=64, upsampling_ratios=(8, 8, 4, 2),
                         encoder_hidden_size=32, downsampling_ratios=(2, 4, 8, 8))


def make_dac_encoder_fixture():
    """DacModel.encode (the reference's DACAutoencoder.encode, autoencoder.py:27-28) on a reduced-width
    encoder with the 44.1 kHz strides (2, 4, 8, 8): input waveform, latent and codes."""
    c, seed = ENC_DAC, 5
    W = dict(dac_ref.make_dac_weights(c, seed=seed))
    W.update(dac_ref.make_enc_weights(c, seed=seed))
    hf = DacModel(DacConfig(sampling_rate=44100, hidden_size=c.hidden_size, decoder_hidden_size=c.decoder_hidden_size,
                            upsampling_ratios=list(c.upsampling_ratios), encoder_hidden_size=c.encoder_hidden_size,
                            downsampling_ratios=list(c.downsampling_ratios), n_codebooks=c.n_codebooks,
                            codebook_size=c.codebook_size, codebook_dim=c.codebook_dim))
    sd = hf.state_dict()
    for k, v in W.items():
        assert sd[k].shape == v.shape, (k, sd[k].shape, v.shape)
        sd[k] = v
    missing = [k for k in sd if k.startswith(("encoder.", "quantizer.")) and k not in W]
    assert not missing, missing[:5]
    hf.load_state_dict(sd)
    hf.eval()
    g = torch.Generator().manual_seed(seed + 7)
    T = 512 * 24
    t = torch.arange(T) / 44100.0
    wav = (0.3 * torch.sin(2 * math.pi * 180 * t) * torch.sin(2 * math.pi * 2.5 * t)).expand(2, 1, T).clone()
    wav += 0.05 * torch.randn(2, 1, T, generator=g)
    with torch.no_grad():
        z_ref = hf.encoder(wav)
        codes = hf.encode(wav).audio_codes
        z_o, codes_o = dac_ref.encode(W, c, wav)
    print(f"[dac_enc] latent max|d| {(z_o - z_ref).abs().max().item():.2e}, codes equal "
          f"{torch.equal(codes_o, codes)}")
    assert (z_o - z_ref).abs().max().item() < 1e-4 and torch.equal(codes_o, codes)
    np.savez_compressed(os.path.join(HERE, "dac_enc.npz"), wav=wav.numpy(), z=z_ref.numpy(),
                        codes=codes.numpy().astype(np.int16), seed=np.int64(seed))


def make_cond_fixtures():
    """PrefixConditioner.forward / Zonos.prepare_conditioning (conditioning.py:373-389,
    model.py:210-218) run by the reference module, bf16, D=256; phonemize replaced by a fixed
    text -> IPA table (eSpeak is absent)."""
    import zonos.conditioning as zc
    from zonos.config import PrefixConditionerConfig

    from oracle import cond_ref
    from tests.golden_util import COND_CASES, COND_PHONEMES
    D = 256
    out = {}
    for name, (kind, proj, texts, kw, with_spk, cproj) in COND_CASES.items():
        conds = [dict(c) for c in (cond_ref.TRANSFORMER_CONDITIONERS if kind == "transformer"
                                   else cond_ref.HYBRID_CONDITIONERS)]
        for c in conds:
            if cproj and c["name"] in cproj:
                c["projection"] = cproj[c["name"]]
        W = cond_ref.make_weights(conds, D, proj, seed=3)
        pc = zc.PrefixConditioner(PrefixConditionerConfig(conds, proj), D).to(torch.bfloat16)
        sd = pc.state_dict()
        assert set(sd) == set(W), (set(sd) ^ set(W))
        pc.load_state_dict(W)
        pc.eval()
        zc.phonemize = lambda t, l: [COND_PHONEMES[x] for x in t]
        spk = (torch.randn(1, 128, generator=torch.Generator().manual_seed(9)).bfloat16() if with_spk else None)
        cd = zc.make_cond_dict(text=texts, speaker=spk, device="cpu", **kw)
        unc = {k: cd[k] for k in pc.required_keys}
        with torch.no_grad():
            y = torch.cat([pc(cd), pc(unc)])
            ids, _ = zc.tokenize_phonemes([COND_PHONEMES[x] for x in texts])
            y_o = torch.cat([cond_ref.prefix_conditioner(W, conds, cd, ids, proj),
                             cond_ref.prefix_conditioner(W, conds, unc, ids, proj)])
        print(f"[cond {name}] {tuple(y.shape)} oracle bit-exact {torch.equal(y, y_o)}")
        assert torch.equal(y, y_o)
        out[f"{name}_y"] = y.view(torch.int16).numpy()
        out[f"{name}_ids"] = ids.numpy()
        if spk is not None:
            out[f"{name}_spk"] = spk.view(torch.int16).numpy()
    np.savez_compressed(os.path.join(HERE, "cond.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1 and sys.argv[1] == "enc":
        make_dac_encoder_fixture()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "dac_long":
        make_dac_long_fixture()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "cond":
        make_cond_fixtures()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "copy":
        make_copy_fixtures()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "edge":
        make_edge_fixtures()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "full":
        make_full_fixtures(tuple(sys.argv[2:]) or ("c1", "c2", "c3"))
        sys.exit(0)
    make_delay_fixtures()
    make_sampler_fixtures()
    make_generate_fixtures()
    make_copy_fixtures()
    make_edge_fixtures()
    make_full_fixtures()
    make_dac_fixtures()
    make_dac_long_fixture()
    make_dac_encoder_fixture()
    make_cond_fixtures()
