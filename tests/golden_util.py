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
    W_raw = zonos_ref.make_weights(TINY, seed=0, head_scale=float(d["head_scale"]), eos_bias=float(d["eos_bias"]))
    cond = torch.from_numpy(d["cond"]).view(torch.bfloat16)
    return dict(W_raw=W_raw, W=zonos_ref.pad_heads(W_raw, TINY), wsum=str(d["wsum"]), cond=cond,
                prefix=torch.from_numpy(d["prefix"].astype(np.int64)), B=cond.shape[0] // 2,
                max_new=int(d["max_new"]), seed=int(d["seed"]), sp=sp, codes=d["codes"], lens=d["lens"],
                delayed=d["delayed"], offset=int(d["offset"]),
                logits=d["logits"] if "logits" in d.files else None)
