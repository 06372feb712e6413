"""CPU: the oracle (oracle/) against golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py). These pin the checker before it is trusted."""
import hashlib
import os

import numpy as np
import pytest
import torch

from oracle import dac_ref, zonos_ref
from oracle.philox import exp_noise, philox4x32_10

from .golden_util import (CLI_SP, COND_CASES, COPY, COPY_CASES, ENC_DAC, FULL, FULL_SEED, GEN_CASES, GREEDY_SP, TINY_DAC,
                          cond_case, full_weights, load_edge_cases, load_enc_case, load_full_case, load_gen_case, wsum)

G = os.path.join(os.path.dirname(__file__), "golden")


def test_philox_known_answers():
    # Random123 KAT vectors for philox4x32-10
    assert [int(x) for x in philox4x32_10(0, 0, 0, 0, 0, 0)] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert [int(x) for x in philox4x32_10(*([0xFFFFFFFF] * 6))] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert [int(x) for x in philox4x32_10(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822,
                                          0x299f31d0)] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_noise_is_exponential():
    q = exp_noise(5, 1, 0, 8, 9, 1026)
    assert q.dtype == np.float32 and q.min() > 0
    assert abs(float(q.mean()) - 1.0) < 0.02
    # shard invariance: rows [4,8) drawn with row_base=4 equal the full draw
    assert np.array_equal(exp_noise(5, 1, 0, 4, 9, 1026, row_base=4), q[4:])


def test_delay_pattern_golden():
    d = np.load(os.path.join(G, "delay.npz"))
    codes = torch.from_numpy(d["codes"].astype(np.int64))
    dl = zonos_ref.apply_delay(codes)
    assert np.array_equal(dl.numpy(), d["delayed"])
    assert np.array_equal(zonos_ref.revert_delay(dl).numpy(), d["reverted"])
    assert torch.equal(zonos_ref.revert_delay(dl), codes)


def test_sampler_golden():
    d = np.load(os.path.join(G, "sampler.npz"))
    for ci in range(int(d["n_cases"])):
        sp = {k[len(f"sp_{ci}_"):]: float(d[k]) for k in d.files if k.startswith(f"sp_{ci}_")}
        sp["top_k"] = int(sp.get("top_k", 0))
        sp["repetition_penalty_window"] = int(sp["repetition_penalty_window"])
        sp.pop("repetition_penalty")
        logits = torch.from_numpy(d[f"logits_{ci}"])
        B, K, V = logits.shape
        q = torch.from_numpy(exp_noise(int(d["seed"]), ci + 1, 0, B, K, V))
        tok = zonos_ref.sample(logits, q, generated_tokens=torch.from_numpy(d[f"gen_{ci}"].astype(np.int64)),
                               repetition_penalty=torch.from_numpy(d[f"rp_{ci}"]), **sp)
        assert np.array_equal(tok.squeeze(-1).numpy(), d[f"tok_{ci}"]), f"case {ci}"


@pytest.mark.parametrize("name", list(GEN_CASES) + COPY_CASES)
def test_generate_golden(name):
    c = load_gen_case(name)
    assert wsum(c["W_raw"]) == c["wsum"], "synthetic weights are not reproducible on this host"
    trace = {}
    out = zonos_ref.generate(c["W"], c["cfg"], c["cond"], c["prefix"], c["max_new"], 2.0, c["B"], c["sp"],
                             seed=c["seed"], trace=trace)
    assert [int(x.shape[1]) for x in out] == c["lens"].tolist()
    for i, x in enumerate(out):
        assert np.array_equal(x.numpy(), c["codes"][i, :, :c["lens"][i]]), f"row {i}"
    assert np.array_equal(trace["delayed"].numpy(), c["delayed"])
    if c["logits"] is not None:
        got = torch.stack(trace["logits"][:len(c["logits"])]).numpy()
        assert np.array_equal(got, c["logits"])


def test_generate_edge_shapes_golden():
    """The restatement at generate()'s edge shapes (no prefix, 1 new token, fewer new tokens than
    codebooks, odd batches) reproduces the reference's codes and delayed buffer."""
    W_raw, W, ws, sp, cases = load_edge_cases()
    assert wsum(W_raw) == ws
    for i, c in enumerate(cases):
        trace = {}
        out = zonos_ref.generate(W, COPY, c["cond"], c["prefix"], c["max_new"], 2.0, c["B"], sp, seed=c["seed"],
                                 trace=trace)
        assert [int(x.shape[1]) for x in out] == c["lens"].tolist(), i
        for b, x in enumerate(out):
            assert np.array_equal(x.numpy(), c["codes"][b, :, :c["lens"][b]]), (i, b)
        assert np.array_equal(trace["delayed"].numpy(), c["delayed"]), i


@pytest.mark.parametrize("name", ["dac_tiny", "dac_44k"])
def test_dac_golden(name):
    d = np.load(os.path.join(G, f"{name}.npz"))
    c = TINY_DAC if name == "dac_tiny" else dac_ref.DAC_44KHZ
    W = dac_ref.make_dac_weights(c, seed=int(d["seed"]))
    assert wsum(W) == str(d["wsum"])
    codes = torch.from_numpy(d["codes"].astype(np.int64))
    got = dac_ref.decode(W, c, codes)
    assert (got - torch.from_numpy(d["wav"])).abs().max().item() < 1e-5
    L = int(d["short_len"])
    got_s = dac_ref.decode_list(W, c, [codes[1, :, :L]])[0]
    assert (got_s - torch.from_numpy(d["wav_short"][0])).abs().max().item() < 1e-5


def test_dac_long_golden():
    """dac_44k_long.npz (reference DacModel, 2 x 600 frames, int16-quantised): the oracle's decode of
    the short row (437 frames) within the quantisation step, and the stored scales consistent."""
    d = np.load(os.path.join(G, "dac_44k_long.npz"))
    c = dac_ref.DAC_44KHZ
    W = dac_ref.make_dac_weights(c, seed=int(d["seed"]))
    assert wsum(W) == str(d["wsum"])
    codes = torch.from_numpy(d["codes"].astype(np.int64))
    L = int(d["short_len"])
    ref_s = torch.from_numpy(d["wav_short_q"][0].astype(np.float32)) * float(d["wav_short_scale"])
    with torch.no_grad():
        got_s = dac_ref.decode_list(W, c, [codes[1, :, :L]])[0]
    assert got_s.shape == ref_s.shape == (1, L * 512)
    assert (got_s - ref_s).abs().max().item() <= 0.5 * float(d["wav_short_scale"]) + 1e-6


def test_dac_encoder_golden():
    """oracle DAC encoder + RVQ encode == transformers DacModel.encode (dac_enc.npz)."""
    W, wav, z_ref, codes_ref = load_enc_case()
    with torch.no_grad():
        z, codes = dac_ref.encode(W, ENC_DAC, wav)
    assert (z - z_ref).abs().max().item() < 1e-4
    assert torch.equal(codes, codes_ref)


@pytest.mark.parametrize("name", list(COND_CASES))
def test_prefix_conditioner_golden(name):
    """oracle PrefixConditioner (fed by zonos_amd's make_cond_dict + phoneme tokenizer) == the
    reference module's prepare_conditioning output (cond.npz), bit for bit."""
    from oracle import cond_ref
    from zonos_amd.conditioning import tokenize_phonemes
    c = cond_case(name, "cpu")
    ids, _ = tokenize_phonemes(c["phonemes"])
    assert torch.equal(ids, c["ids"])
    y = torch.cat([cond_ref.prefix_conditioner(c["W"], c["conds"], c["cond"], ids, c["proj"]),
                   cond_ref.prefix_conditioner(c["W"], c["conds"], c["uncond"], ids, c["proj"])])
    assert torch.equal(y, c["y"])


def test_full_c1_golden():
    """Full-width (1.62 B params) free-running greedy decode, B=1, Lc=24, 129 tokens: the oracle
    reproduces the reference's codes and recorded logits bit for bit (~40 s on 8 cores)."""
    c = load_full_case("c1")
    trace = {}
    out = zonos_ref.generate(full_weights("copy"), FULL, c["cond"], None, c["T"], 2.0, 1, GREEDY_SP,
                             seed=FULL_SEED, trace=trace)
    assert [int(x.shape[1]) for x in out] == c["lens"].tolist()
    assert np.array_equal(out[0].numpy(), c["codes"][0, :, :c["lens"][0]])
    got = np.stack([trace["logits"][s].numpy() for s in c["logit_steps"]])
    assert np.array_equal(got, c["logits"])
    assert c["margins"].min() > 6.0      # copy heads: every greedy decision far from a tie


@pytest.mark.parametrize("name,window", [("c2", 0), ("c3", 0)])
def test_full_forced_golden(name, window):
    """Full-width teacher-forced steps (prefill over a forced history + single-token decodes,
    CLI sampling with the engine's noise key) of utterance 0: the oracle reproduces the
    reference's logits and tokens bit for bit (first window; the late-context windows were
    cross-checked when the fixture was made)."""
    c = load_full_case(name)
    B, P = c["B"], c["P"]
    s0, n = c["windows"][window]
    cu = torch.cat([c["cond"][0:1], c["cond"][B:B + 1]])
    o = zonos_ref.forced_steps(full_weights("random"), FULL, cu, c["history"][0:1], P, [(s0, n)], CLI_SP, FULL_SEED, 0)
    steps = c["steps"].tolist()
    for s, (raw, tok, m) in o.items():
        j = steps.index(s)
        assert np.array_equal(tok[0].numpy(), c["tokens"][0, j]), s
        assert np.array_equal(m[0].numpy(), c["margins"][0, j]), s
        if s in c["logit_steps"]:
            assert np.array_equal(raw[0].numpy(), c["logits"][0, list(c["logit_steps"]).index(s)]), s
