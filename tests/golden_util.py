"""Shared loaders for the golden fixtures (no reference import; runs anywhere)."""
import hashlib
import os

import numpy as np
import torch

from oracle import dac_ref, zonos_ref

G = os.path.join(os.path.dirname(__file__), "golden")
TINY = zonos_ref.BackboneCfg(d_model=256, n_layer=2, n_heads=2, n_kv=1, d_ff=512)
TINY_DAC = dac_ref.DacCfg(hidden_size=64, decoder_hidden_size=64, upsampling_ratios=(4, 2))
ENC_DAC = dac_ref.DacCfg(hidden_size=64, decoder_hidden_size=64, upsampling_ratios=(8, 8, 4, 2),
                         encoder_hidden_size=32, downsampling_ratios=(2, 4, 8, 8))


def load_enc_case():
    """dac_enc.npz (DacModel.encode on ENC_DAC) + the oracle weights that produced it."""
    d = np.load(os.path.join(G, "dac_enc.npz"))
    seed = int(d["seed"])
    W = dict(dac_ref.make_dac_weights(ENC_DAC, seed=seed))
    W.update(dac_ref.make_enc_weights(ENC_DAC, seed=seed))
    return W, torch.from_numpy(d["wav"]), torch.from_numpy(d["z"]), torch.from_numpy(d["codes"].astype(np.int64))


GEN_CASES = ["greedy", "greedy_rep", "sampled_cli", "sampled_knobs", "eos_greedy", "eos_sampled"]
# free-running greedy fixtures on "copy" heads (zonos_ref.make_copy_weights): every decision that
# reaches the output has a top-1/top-2 margin far above the GPU-vs-CPU logit error, so the codes
# are a bit-identical target (D=1024 so the copy signal, ~sqrt(D/9), clears the cross-embedding
# noise of 1025 rows)
COPY = zonos_ref.BackboneCfg(d_model=1024, n_layer=2, n_heads=8, n_kv=2, d_ff=2048)
COPY_CASES = ["copy_greedy", "copy_rep", "copy_eos"]
FULL = zonos_ref.ZONOS_V01_TRANSFORMER
CLI_SP = dict(top_p=0, top_k=0, min_p=0, linear=0.65, conf=0.4, quad=0.0, repetition_penalty=2.5,
              repetition_penalty_window=8, temperature=1.0)
GREEDY_SP = dict(temperature=0.0, top_p=0, top_k=0, min_p=0, linear=0.0, conf=0.0, quad=0.0,
                 repetition_penalty=1.0, repetition_penalty_window=2)
# full-width (Zonos-v0.1-transformer geometry) workloads of SURVEY §8(d):
#   c1: free-running greedy on copy heads (bit-identical codes, reference-generated);
#   c2/c3: random weights (the bench's distribution), CLI sampling, teacher-forced on a seeded
#          synthetic history; windows = (first step, steps) -- one prefill over the forced history,
#          then single-token decodes; `utts` = utterances the reference computed.
FULL_CASES = {
    "c1": dict(B=1, Lc=24, P=0, T=129, emb_gain=4.0, logit_steps=(0, 1, 64, 128)),
    "c2": dict(B=1, Lc=160, P=0, T=861, windows=((0, 32), (800, 8)), utts=(0,), logit_steps=(0, 1, 31, 800, 807)),
    # c3: five utterances spread over the batch (first, last, three inside) at the first steps, the
    # mean context and the end of the 30 s workload (ctx up to Lc + P + 1 + 2567 = 2978)
    "c3": dict(B=64, Lc=400, P=10, T=2580, windows=((0, 8), (1290, 8), (2560, 8)), utts=(0, 13, 37, 50, 63),
               logit_steps=(0, 1, 1290, 1291, 2560, 2567)),
    # c4 = B=512 over 8 GPUs: the rank-7 shard (utterances 448..511 -> row_base 448, the inputs
    # bench.py gives rank 7: conditioning seed 1+7, prefix seed 3+7), five utterances, at the first
    # steps and at the last steps of the 30 s workload (context up to Lc + P + 1 + 2587 = 2998)
    "c4": dict(B=64, Lc=400, P=10, T=2580, windows=((0, 4), (2584, 4)), utts=(0, 13, 37, 50, 63), row_base=448,
               cond_seed=8, prefix_seed=10, hist_seed=14, hist_T=2590, logit_steps=(0, 1, 2584, 2587)),
}
FULL_SEED = 1234


# c5: the hybrid at the benchmark workload (bench.py --model hybrid: B = 64, Lc = 400, P = 10, 2580
# tokens), three utterances (first, middle, last of the batch), logits from the first steps to the
# last attention contexts (~2980) -- restatement-generated (tests/golden/make_hybrid_golden.py)
HYBRID_C5 = dict(B=64, Lc=400, P=10, T=2580, utts=(0, 37, 63), w_seed=0, cond_seed=1, prefix_seed=3, hist_seed=7,
                 seed=FULL_SEED,
                 logit_steps=(0, 1, 2, 256, 768, 1290, 1291, 1792, 2304, 2568, 2569, 2570))


def forced_history(B: int, P: int, T: int, prefix, seed: int = 7) -> torch.Tensor:
    """Delayed codes [B, 9, T+9] of a seeded random history after the prefix (teacher forcing)."""
    g = torch.Generator().manual_seed(seed)
    codes = torch.randint(0, 1024, (B, 9, T), generator=g)
    if P:
        codes[..., :P] = prefix
    return zonos_ref.apply_delay(codes)


_W_CACHE = {}


def full_weights(kind: str):
    """Full-width weights (cached per process): 'random' = make_weights(FULL, 0), 'copy' = c1's."""
    if kind not in _W_CACHE:
        _W_CACHE.clear()
        if kind == "random":
            W = zonos_ref.make_weights(FULL, seed=0)
        else:
            W = zonos_ref.make_copy_weights(FULL, seed=0, emb_gain=FULL_CASES["c1"]["emb_gain"])
        _W_CACHE[kind] = zonos_ref.pad_heads(W, FULL)
    return _W_CACHE[kind]


def load_full_case(name):
    """gen_full_<name>.npz + its inputs (cond, prefix, forced history) rebuilt from their seeds."""
    d = np.load(os.path.join(G, f"gen_full_{name}.npz"))
    c = dict(FULL_CASES[name])
    B, Lc, P = c["B"], c["Lc"], c["P"]
    c.setdefault("row_base", 0)
    c["cond"] = zonos_ref.synthetic_conditioning(B, Lc, FULL.d_model, seed=c.get("cond_seed", 1))
    c["prefix"] = zonos_ref.synthetic_prefix_codes(B, P, seed=c.get("prefix_seed", 3)) if P else None
    c.update({k: d[k] for k in d.files})
    if name != "c1":
        c["history"] = forced_history(B, P, c.get("hist_T", c["T"]), c["prefix"], seed=c.get("hist_seed", 7))
    return c


def wsum(W: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(W):
        h.update(k.encode())
        h.update(W[k].float().contiguous().numpy().tobytes())
    return h.hexdigest()


def load_gen_case(name):
    d = np.load(os.path.join(G, f"gen_{name}.npz"))
    sp = {k[3:]: float(d[k]) for k in d.files if k.startswith("sp_")}
    sp["top_k"] = int(sp["top_k"])
    sp["repetition_penalty_window"] = int(sp["repetition_penalty_window"])
    if name.startswith("copy"):
        cfg = COPY
        W_raw = zonos_ref.make_copy_weights(COPY, seed=int(d["wseed"]), copy_gain=float(d["copy_gain"]),
                                            eos_tokens=tuple(int(t) for t in d["eos_tokens"]))
    else:
        cfg = TINY
        W_raw = zonos_ref.make_weights(TINY, seed=0, head_scale=float(d["head_scale"]), eos_bias=float(d["eos_bias"]))
    cond = torch.from_numpy(d["cond"]).view(torch.bfloat16)
    return dict(cfg=cfg, W_raw=W_raw, W=zonos_ref.pad_heads(W_raw, cfg), wsum=str(d["wsum"]), cond=cond,
                prefix=torch.from_numpy(d["prefix"].astype(np.int64)), B=cond.shape[0] // 2,
                max_new=int(d["max_new"]), seed=int(d["seed"]), sp=sp, codes=d["codes"], lens=d["lens"],
                delayed=d["delayed"], offset=int(d["offset"]),
                logits=d["logits"] if "logits" in d.files else None,
                margins=d["margins"] if "margins" in d.files else None)


def load_edge_cases():
    """gen_edge.npz (make_golden.make_edge_fixtures): generate() at edge shapes on copy heads --
    no audio prefix, 1 / 2 / 5 / 9 / 10 / 17 new tokens, B = 1, 2, 3. Returns (W_raw, W, wsum, sp, cases)."""
    d = np.load(os.path.join(G, "gen_edge.npz"))
    sp = {k[3:]: float(d[k]) for k in d.files if k.startswith("sp_")}
    sp["top_k"] = int(sp["top_k"])
    sp["repetition_penalty_window"] = int(sp["repetition_penalty_window"])
    W_raw = zonos_ref.make_copy_weights(COPY, seed=0, copy_gain=float(d["copy_gain"]))
    cases = []
    for i in range(int(d["n"])):
        B, P, max_new, Lc, seed = (int(v) for v in d[f"e{i}_shape"])
        cases.append(dict(B=B, P=P, max_new=max_new, Lc=Lc, seed=seed,
                          cond=torch.from_numpy(d[f"e{i}_cond"]).view(torch.bfloat16),
                          prefix=torch.from_numpy(d[f"e{i}_prefix"].astype(np.int64)) if P else None,
                          codes=d[f"e{i}_codes"], lens=d[f"e{i}_lens"], margins=d[f"e{i}_margins"],
                          delayed=d[f"e{i}_delayed"]))
    return W_raw, zonos_ref.pad_heads(W_raw, COPY), str(d["wsum"]), sp, cases


EDGE_N = 6


# ---- PrefixConditioner fixtures (cond.npz; made by make_golden.make_cond_fixtures)
COND_PHONEMES = {"hello": "həlˈoʊ wˈɜːld!", "long": "ðɪs ɪz ə lˈɔŋɡɚ sˈɛntəns, wɪð pˈʌŋktʃuːˈeɪʃən… ænd ɐ ʔ",
                 "unk": "a1b"}
COND_CASES = {
    # name: (conditioner list, prefix projection, texts, cond_dict kwargs, speaker?, per-conditioner projection)
    "transformer_default": ("transformer", "none", ["hello", "long"], {}, True, None),
    "hybrid_all_cond": ("hybrid", "none", ["long"], dict(unconditional_keys=[], speaker_noised=True, fmax=24000.0,
                                                      language="ja", emotion=[0.3, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1],
                                                      pitch_std=80.0, speaking_rate=22.5, ctc_loss=3.0,
                                                      dnsmos_ovrl=3.5, vqscore_8=[0.7, 0.72, 0.74, 0.76, 0.78,
                                                                                  0.8, 0.79, 0.6]), False, None),
    "projections": ("transformer", "mlp", ["unk", "hello"], dict(unconditional_keys=["emotion"]), True,
                    {"fmax": "mlp", "language_id": "linear"}),
}


def cond_case(name: str, device="cpu"):
    """Rebuild a cond.npz case: conditioner configs, projection, weights, cond / uncond dicts (on
    ``device``, built by zonos_amd.conditioning.make_cond_dict), phoneme ids, expected [2B, L, D]."""
    from oracle import cond_ref
    from zonos_amd import conditioning as zc
    d = np.load(os.path.join(G, "cond.npz"))
    kind, proj, texts, kw, with_spk, cproj = COND_CASES[name]
    conds = [dict(c) for c in (cond_ref.TRANSFORMER_CONDITIONERS if kind == "transformer"
                               else cond_ref.HYBRID_CONDITIONERS)]
    for c in conds:
        if cproj and c["name"] in cproj:
            c["projection"] = cproj[c["name"]]
    W = cond_ref.make_weights(conds, 256, proj, seed=3)
    spk = torch.from_numpy(d[f"{name}_spk"]).view(torch.bfloat16) if with_spk else None
    cd = zc.make_cond_dict(text=texts, speaker=spk, device=device, **kw)
    required = {c["name"] for c in conds if c.get("uncond_type", "none") != "learned"}
    unc = {k: cd[k] for k in required}
    phon = [COND_PHONEMES[t] for t in texts]
    return dict(conds=conds, proj=proj, W=W, cond=cd, uncond=unc, texts=texts, phonemes=phon,
                ids=torch.from_numpy(d[f"{name}_ids"]), y=torch.from_numpy(d[f"{name}_y"]).view(torch.bfloat16))
