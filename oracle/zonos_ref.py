"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the Zonos decode hot path.

This is a functional CPU restatement (PyTorch CPU ops, bf16 like the reference) of
the reference algorithm. It is the *checker* for the HIP engine in zonos_amd and the
timed CPU baseline in bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it; the product path never does.

Every function cites the reference file:line it restates (paths relative to the
coezbek/Zonos checkout). Parity of this oracle with the reference itself is pinned
by tests/test_oracle_golden.py against tests/golden/*.npz, which
tests/golden/make_golden.py produced by importing the reference in the build
container.

It uses the same torch CPU primitives at the same rounding points as the reference
(bf16 Linear / LayerNorm / SDPA, fp32 logits), so on CPU it reproduces the
reference bit for bit; the GPU engine is compared to it with tolerances.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from .philox import exp_noise

EOS, MASK, UNKNOWN = 1024, 1025, -1


@dataclass
class BackboneCfg:
    """Mirror of zonos/config.py:28-39 (BackboneConfig) restricted to the transformer."""
    d_model: int = 2048
    n_layer: int = 26
    n_heads: int = 16
    n_kv: int = 4
    d_ff: int = 8192            # attn_mlp_d_intermediate
    eps: float = 1e-5
    n_cb: int = 9
    vocab: int = 1026           # 1025 padded by pad_weight_ (zonos/utils.py:22-37)

    @property
    def head_dim(self):
        return self.d_model // self.n_heads

    @classmethod
    def from_zonos_config(cls, d: dict) -> "BackboneCfg":
        b = d["backbone"]
        return cls(d_model=b["d_model"], n_layer=b["n_layer"], n_heads=b["attn_cfg"]["num_heads"],
                   n_kv=b["attn_cfg"]["num_heads_kv"], d_ff=b["attn_mlp_d_intermediate"],
                   eps=b.get("norm_epsilon", 1e-5))

    def to_zonos_config(self) -> dict:
        """A config.json dict in the reference's format (zonos/config.py:48-62)."""
        return {
            "backbone": {"d_model": self.d_model, "d_intermediate": 0,
                         "attn_mlp_d_intermediate": self.d_ff, "n_layer": self.n_layer, "ssm_cfg": {},
                         "attn_layer_idx": list(range(self.n_layer)),
                         "attn_cfg": {"num_heads": self.n_heads, "num_heads_kv": self.n_kv},
                         "rms_norm": False, "residual_in_fp32": False, "norm_epsilon": self.eps},
            "prefix_conditioner": {"conditioners": [], "projection": "none"},
            "eos_token_id": EOS, "masked_token_id": MASK, "pad_vocab_to_multiple_of": 8,
        }


ZONOS_V01_TRANSFORMER = BackboneCfg()   # SURVEY.md §8 architecture numbers


# ----------------------------------------------------------------------------------------
# Deterministic synthetic weights (there are no trained checkpoints in this environment)
# ----------------------------------------------------------------------------------------

def weight_shapes(cfg: BackboneCfg) -> dict:
    """The reference's state-dict keys for the hot path (model.py:36-37, _torch.py:61-62,88-91,114-115,147-148)."""
    D, hd = cfg.d_model, cfg.head_dim
    s = {}
    for i in range(cfg.n_layer):
        p = f"backbone.layers.{i}."
        s[p + "norm.weight"] = (D,)
        s[p + "norm.bias"] = (D,)
        s[p + "mixer.in_proj.weight"] = ((cfg.n_heads + 2 * cfg.n_kv) * hd, D)
        s[p + "mixer.out_proj.weight"] = (D, cfg.n_heads * hd)
        s[p + "norm2.weight"] = (D,)
        s[p + "norm2.bias"] = (D,)
        s[p + "mlp.fc1.weight"] = (2 * cfg.d_ff, D)
        s[p + "mlp.fc2.weight"] = (D, cfg.d_ff)
    s["backbone.norm_f.weight"] = (D,)
    s["backbone.norm_f.bias"] = (D,)
    for k in range(cfg.n_cb):
        s[f"embeddings.{k}.weight"] = (cfg.vocab, D)
    for k in range(cfg.n_cb):
        s[f"heads.{k}.weight"] = (cfg.vocab - 1, D)   # checkpoint holds 1025 rows; padded on load
    return s


def make_weights(cfg: BackboneCfg, seed: int = 0, head_scale: float = 1.0, device="cpu",
                 eos_bias: float = 0.0) -> dict:
    """Seeded synthetic weights in the reference layout, bf16.

    Each key gets its own torch.Generator seeded from (seed, key index) so the tensors
    are reproducible on any host. ``head_scale`` widens logit margins (greedy parity
    is only meaningful when top-1/top-2 gaps exceed GEMM reduction-order noise,
    SURVEY.md §7 "Hard parts"). ``eos_bias`` tilts head 0's EOS row towards
    norm_f.bias so that EOS is sampled within a short test (exercises model.py:376-414).
    """
    out = {}
    for idx, (k, shape) in enumerate(weight_shapes(cfg).items()):
        g = torch.Generator(device="cpu").manual_seed(seed * 1_000_003 + idx)
        if k.endswith("norm.weight") or k.endswith("norm2.weight") or k.endswith("norm_f.weight"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif k.endswith(".bias"):
            t = 0.1 * torch.randn(shape, generator=g)
        elif k.startswith("embeddings"):
            t = torch.randn(shape, generator=g)
        elif k.startswith("heads"):
            t = torch.randn(shape, generator=g) * (head_scale / math.sqrt(shape[1]))
        else:
            t = torch.randn(shape, generator=g) / math.sqrt(shape[1])
        out[k] = t
    if eos_bias:
        b = out["backbone.norm_f.bias"]
        out["heads.0.weight"][EOS] += eos_bias * b / b.pow(2).sum()
    return {k: v.to(torch.bfloat16).to(device) for k, v in out.items()}


def make_copy_weights(cfg: BackboneCfg, seed: int = 0, copy_gain: float = 1.0, emb_gain: float = 1.0,
                      eos_tokens: tuple = (), noise: float = 0.0, device="cpu") -> dict:
    """Synthetic weights whose greedy decisions have LARGE margins, so that free-running greedy
    codes are a meaningful bit-identical target across CPU and GPU (test fixtures only).

    Backbone / norms / embeddings as make_weights (embeddings x ``emb_gain``). Each head k is a
    "copy" map: with pi_k a seeded permutation of 0..1023, row j = copy_gain * E_k[pi_k(j)] /
    sqrt(D) (+ ``noise`` * N(0, 1/D)), so the row whose pi_k(j) is codebook k's current input token
    gets a logit ~ copy_gain * sqrt(D / 9) above the others (the hidden state's projection on that
    embedding), while every other row sees only cross-embedding noise ~ copy_gain * N(0, 1). The
    MASK input (1025, delay-pattern fill) is folded into row pi_k^-1(0). Head 0's EOS row is a
    boosted copy of each of ``eos_tokens`` (2x, beats the -log(1024) EOS bias of model.py:333-334),
    so a greedy chain emits EOS deterministically when cb0 reaches one of them (the first EOS is
    resampled away and starts the 6-step hold-off, model.py:362-392; a later one is accepted); rows
    1024 of heads 1..8 stay small (EOS is masked there, model.py:331). The decision margins are checked on the
    reference's own run by tests/test_oracle_golden.py."""
    W = {k: v.float() for k, v in make_weights(cfg, seed=seed).items()}
    D = cfg.d_model
    g = torch.Generator(device="cpu").manual_seed(seed * 7919 + 17)
    for k in range(cfg.n_cb):
        E = W[f"embeddings.{k}.weight"]
        perm = torch.randperm(1024, generator=g)
        H = copy_gain * E[perm] / math.sqrt(D)
        H[int((perm == 0).nonzero())] += copy_gain * E[MASK] / math.sqrt(D)
        r = torch.randn(1025, D, generator=g) / math.sqrt(D)
        eos_row = 0.1 * r[EOS:EOS + 1]
        if k == 0 and eos_tokens:
            eos_row = 2.0 * copy_gain * E[list(eos_tokens)].sum(0, keepdim=True) / math.sqrt(D)
        H = torch.cat([H, eos_row]) + noise * r
        W[f"heads.{k}.weight"] = H
        W[f"embeddings.{k}.weight"] = E * emb_gain
    return {k: v.to(torch.bfloat16).to(device) for k, v in W.items()}


def copy_chain(W: dict, cfg: BackboneCfg, k: int, token: int, n: int) -> list:
    """The greedy chain of head k under make_copy_weights (test helper): next = argmax_j of the
    copy rows for input ``token``, n steps."""
    E = W[f"embeddings.{k}.weight"].float()
    H = W[f"heads.{k}.weight"].float()[:1024]
    out = []
    for _ in range(n):
        token = int(torch.argmax(H @ E[token]))
        out.append(token)
    return out


def pad_heads(W: dict, cfg: BackboneCfg) -> dict:
    """pad_weight_ (zonos/utils.py:22-37): 1025 % 8 == 1 extra zero row -> 1026 rows."""
    W = dict(W)
    for k in range(cfg.n_cb):
        w = W[f"heads.{k}.weight"]
        if w.shape[0] % 8:
            W[f"heads.{k}.weight"] = F.pad(w, (0, 0, 0, w.shape[0] % 8))
    return W


# ----------------------------------------------------------------------------------------
# Backbone (zonos/backbone/_torch.py)
# ----------------------------------------------------------------------------------------

def rope_table(seq_len: int, head_dim: int, base: float = 10000.0) -> torch.Tensor:
    """[seq_len, head_dim/2, 2] (cos, sin) fp32 -- restates precompute_freqs_cis (_torch.py:9-15)."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2)[: head_dim // 2].float() / head_dim))
    ang = torch.outer(torch.arange(seq_len, device=inv.device), inv)
    z = torch.polar(torch.ones_like(ang), ang)
    return torch.stack([z.real, z.imag], dim=-1)


def rope(x: torch.Tensor, fc: torch.Tensor) -> torch.Tensor:
    """Interleaved-pair rotation in fp32, cast back (apply_rotary_emb, _torch.py:18-30).
    x [R,S,H,hd] bf16, fc [R,S,hd/2,2]."""
    xs = x.float().reshape(*x.shape[:-1], -1, 2)
    c = fc[:, :, None, :, 0]
    s = fc[:, :, None, :, 1]
    a, b = xs[..., 0], xs[..., 1]
    y = torch.stack([a * c - b * s, b * c + a * s], dim=-1).flatten(3)
    return y.type_as(x)


class KVCache:
    """Per-layer [R, S_max, 2, Hkv, hd] bf16 cache (_torch.py:96-97) + shared offset (config.py:8-25)."""

    def __init__(self, cfg: BackboneCfg, rows: int, max_seqlen: int):
        S = max_seqlen + (-max_seqlen) % 8      # find_multiple(.., 8), model.py:205
        self.kv = [torch.zeros(rows, S, 2, cfg.n_kv, cfg.head_dim, dtype=torch.bfloat16)
                   for _ in range(cfg.n_layer)]
        self.seqlen_offset = 0
        self.lengths = torch.zeros(rows, dtype=torch.int32)


def attention(W, cfg, i, x, kv: KVCache, fc):
    """Attention.forward (_torch.py:117-141) incl. _update_kv_cache (_torch.py:33-49)."""
    R, S, _ = x.shape
    hd, H, Hk = cfg.head_dim, cfg.n_heads, cfg.n_kv
    qkv = F.linear(x, W[f"backbone.layers.{i}.mixer.in_proj.weight"])
    q, k, v = qkv.split([H * hd, Hk * hd, Hk * hd], dim=-1)
    q = rope(q.view(R, S, H, hd), fc)
    k = rope(k.view(R, S, Hk, hd), fc)
    v = v.view(R, S, Hk, hd)
    cache = kv.kv[i]
    o = kv.seqlen_offset
    cache[:, o:o + S, 0] = k
    cache[:, o:o + S, 1] = v
    kk, vv = cache[:, :o + S].unbind(dim=-3)
    y = F.scaled_dot_product_attention(q.transpose(1, 2), kk.transpose(1, 2), vv.transpose(1, 2),
                                       is_causal=S > 1, enable_gqa=True)
    y = y.transpose(1, 2).contiguous().view(R, S, H * hd)
    return F.linear(y, W[f"backbone.layers.{i}.mixer.out_proj.weight"])


def backbone(W, cfg: BackboneCfg, h: torch.Tensor, kv: KVCache, freqs: torch.Tensor) -> torch.Tensor:
    """TorchZonosBackbone.forward (_torch.py:73-80) with TransformerBlock (_torch.py:99-102)
    and FeedForward (_torch.py:150-152). Pre-LN LayerNorm *with bias*, SwiGLU (y, gate).
    A HybridCfg routes to the hybrid backbone restatement (oracle/hybrid_ref.py)."""
    from . import hybrid_ref
    if isinstance(cfg, hybrid_ref.HybridCfg):
        return hybrid_ref.backbone(W, cfg, h, kv, freqs)
    R, S, D = h.shape
    pos = torch.arange(S)[None, :] + kv.lengths[:, None]
    fc = freqs[pos]
    x = h
    for i in range(cfg.n_layer):
        p = f"backbone.layers.{i}."
        xn = F.layer_norm(x, (D,), W[p + "norm.weight"], W[p + "norm.bias"], cfg.eps)
        x = x + attention(W, cfg, i, xn, kv, fc)
        xn = F.layer_norm(x, (D,), W[p + "norm2.weight"], W[p + "norm2.bias"], cfg.eps)
        y, gate = F.linear(xn, W[p + "mlp.fc1.weight"]).chunk(2, dim=-1)
        x = x + F.linear(y * F.silu(gate), W[p + "mlp.fc2.weight"])
    return F.layer_norm(x, (D,), W["backbone.norm_f.weight"], W["backbone.norm_f.bias"], cfg.eps)


def embed_codes(W, cfg, ids: torch.Tensor) -> torch.Tensor:
    """sum_k Emb_k[ids[:, k]] with bf16 left-to-right adds (model.py:97-98). ids [B,9,S]."""
    return sum(F.embedding(ids[:, k], W[f"embeddings.{k}.weight"]) for k in range(cfg.n_cb))


def compute_logits(W, cfg, h, kv, freqs, cfg_scale):
    """_compute_logits (model.py:103-116): last position -> 9 heads -> fp32 -> CFG -> mask >= 1025."""
    last = backbone(W, cfg, h, kv, freqs)[:, -1:, :]
    logits = torch.stack([F.linear(last, W[f"heads.{k}.weight"]) for k in range(cfg.n_cb)], dim=1)
    logits = logits.squeeze(2).float()
    c, u = logits.chunk(2)
    logits = u + (c - u) * cfg_scale
    logits[..., 1025:] = -torch.inf
    return logits


# ----------------------------------------------------------------------------------------
# Sampler (zonos/sampling.py)
# ----------------------------------------------------------------------------------------

def rep_penalty(logits, generated, rp, window):
    """modify_logit_for_repetition_penalty (sampling.py:131-169): compounding factor rp^count."""
    g = generated[..., -window:].clamp_max(logits.shape[-1] - 1).to(torch.int64)
    rp = rp[:, None, None] if rp.ndim == 1 else rp
    f = torch.ones_like(logits).scatter_reduce(2, g, torch.ones_like(logits) * rp, reduce="prod")
    return torch.where(logits <= 0, logits * f, logits / f)


def shape_probs(probs, top_p=0.0, top_k=0, min_p=0.0, linear=0.0, conf=0.0, quad=0.0):
    """apply_unified / apply_top_p / apply_top_k / apply_min_p in the reference's order
    (sampling.py:54-128, call order 310-318)."""
    if linear > 0:
        lp = torch.log(probs.clamp_min(1e-20))
        ent = -torch.sum(probs * lp, dim=-1, keepdim=True)
        probs = (lp * (linear + ent * conf) - lp ** 2 * quad).softmax(dim=-1)
    if top_p > 0:
        ps, pi = torch.sort(probs, dim=-1, descending=True)
        cs = torch.cumsum(ps, dim=-1)
        ps = ps * (~(cs - ps > top_p)).float()
        probs = probs.scatter(-1, pi, ps)
        probs = probs / probs.sum(dim=-1, keepdim=True)
    if top_k > 0:
        v, _ = torch.topk(probs, min(top_k, probs.size(-1)))
        probs = torch.where(probs < v[..., -1:], 0.0, probs)
        probs = probs / probs.sum(dim=-1, keepdim=True)
    if min_p > 0:
        probs = probs.masked_fill(probs < min_p * probs.max(dim=-1, keepdim=True)[0], 0.0)
        probs = probs / probs.sum(dim=-1, keepdim=True)
    return probs


def sample(logits, noise=None, temperature=1.0, top_p=0.0, top_k=0, min_p=0.0, linear=0.0, conf=0.0,
           quad=0.0, generated_tokens=None, repetition_penalty=3.0, repetition_penalty_window=2,
           decision: list | None = None, **_):
    """sample_from_logits (sampling.py:232-328) with the Exp(1) race noise passed in explicitly
    (the reference draws it from torch's generator in multinomial, sampling.py:26-28).
    ``decision`` (test instrumentation) receives the array whose argmax is the token."""
    if not isinstance(repetition_penalty, torch.Tensor):
        repetition_penalty = torch.tensor(repetition_penalty, dtype=logits.dtype)
    if (repetition_penalty != 1.0).any() and generated_tokens is not None:
        logits = rep_penalty(logits, generated_tokens, repetition_penalty, repetition_penalty_window)
    if temperature > 0:
        probs = torch.softmax(logits / temperature, dim=-1)
        probs = shape_probs(probs, top_p, top_k, min_p, linear, conf, quad)
        if decision is not None:
            decision.append(("ratio", probs / noise))
        return torch.argmax(probs / noise, dim=-1, keepdim=True).to(torch.int64)
    if decision is not None:
        decision.append(("logit", logits.clone()))
    return torch.argmax(logits, dim=-1, keepdim=True)


# ----------------------------------------------------------------------------------------
# Delay pattern (zonos/codebook_pattern.py)
# ----------------------------------------------------------------------------------------

def apply_delay(codes: torch.Tensor, mask_token: int = MASK) -> torch.Tensor:
    """delayed[k, t] = codes[k, t-k-1], mask outside (codebook_pattern.py:5-7)."""
    B, K, T = codes.shape
    out = torch.full((B, K, T + K), mask_token, dtype=codes.dtype)
    for k in range(K):
        out[:, k, k + 1:k + 1 + T] = codes[:, k]
    return out


def revert_delay(delayed: torch.Tensor) -> torch.Tensor:
    """out[k, t] = delayed[k, t+k+1] (codebook_pattern.py:10-12)."""
    B, K, L = delayed.shape
    return torch.stack([delayed[:, k, k + 1:L - K + k + 1] for k in range(K)], dim=1)


# ----------------------------------------------------------------------------------------
# generate() (zonos/model.py:224-457)
# ----------------------------------------------------------------------------------------

DEFAULT_SAMPLING = dict(top_p=0, top_k=0, min_p=0, linear=0.55, conf=0.4, quad=0.0,
                        repetition_penalty=3.0, repetition_penalty_window=2, temperature=1.0)


def generate(W, cfg: BackboneCfg, prefix_conditioning: torch.Tensor, audio_prefix_codes=None,
             max_new_tokens: int = 86 * 30, cfg_scale: float = 2.0, batch_size: int = 1,
             sampling_params: dict = DEFAULT_SAMPLING, seed: int = 0, row_base: int = 0,
             trace: dict | None = None, force_full_length: bool = False, max_steps_run: int | None = None,
             force_delayed: torch.Tensor | None = None, noise_fn=None):
    """Restatement of Zonos.generate (model.py:224-457) on CPU.

    Noise for sampler call (step, draw) comes from oracle.philox.exp_noise(seed, step, draw, ...):
    step 0 = the prefill sample (model.py:304), step s>=1 = loop iteration s, draw 1 = the EOS
    resample (model.py:388). ``force_full_length`` adds -inf to the cb0 EOS logit so every row
    runs max_steps (the benchmark mode). ``max_steps_run`` stops the loop early
    (CPU baseline windows). ``trace`` (optional dict) receives per-step logits/tokens.
    ``force_delayed`` (test instrumentation) overwrites every written frame with the given
    delayed codes after it is sampled (teacher forcing on a recorded history). ``noise_fn(step,
    draw)`` (optional) replaces the keyed stream; it is called once per sampler call that draws
    noise (temperature > 0), in the reference's call order -- e.g. torch's own
    `exponential_` on a generator, the reference's noise (sampling.py:26-28).
    """
    assert cfg_scale != 1, "TODO: add support for cfg_scale=1"   # model.py:247
    if batch_size * 2 != prefix_conditioning.shape[0]:
        raise ValueError(f"Batch size mismatch: {batch_size} * 2 != {prefix_conditioning.shape[0]}")
    sp = dict(sampling_params)
    B = batch_size
    P = 0 if audio_prefix_codes is None else audio_prefix_codes.shape[2]
    T = P + max_new_tokens
    Lc = prefix_conditioning.shape[1]
    from . import hybrid_ref
    if isinstance(cfg, hybrid_ref.HybridCfg):          # MambaSSMZonosBackbone (model.py:204-208 cache)
        kv = hybrid_ref.HybridCache(cfg, 2 * B, Lc + T + 9)
        freqs = hybrid_ref.rotary_table(Lc + T + 16, cfg.head_dim, cfg.rotary_base)
    else:
        kv = KVCache(cfg, 2 * B, Lc + T + 9)
        freqs = rope_table(16384, cfg.head_dim)
    codes = torch.full((B, 9, T), UNKNOWN)
    if audio_prefix_codes is not None:
        codes[..., :P] = audio_prefix_codes
    delayed = apply_delay(codes, MASK)

    def noise(step, draw):
        if not float(sp.get("temperature", 1.0)) > 0:
            return None                     # greedy: the reference draws no noise (sampling.py:325-326)
        if noise_fn is not None:
            return noise_fn(step, draw)
        return torch.from_numpy(exp_noise(seed, step, draw, B, cfg.n_cb, cfg.vocab, row_base))

    ids = delayed[..., :P + 1].repeat(2, 1, 1)
    h = torch.cat([prefix_conditioning, embed_codes(W, cfg, ids)], dim=1)
    logits = compute_logits(W, cfg, h, kv, freqs, cfg_scale)
    if force_full_length:
        logits[:, 0, EOS] = -torch.inf
    dec = [] if trace is not None else None
    tok = sample(logits, noise(0, 0), decision=dec, **sp)
    if trace is not None:
        trace.setdefault("decision", []).append(dec)
        trace.setdefault("logits", []).append(logits.clone())
        trace.setdefault("tokens", []).append(tok.clone())
    offset = P + 1
    frame = delayed[..., offset:offset + 1]
    delayed[..., offset:offset + 1] = torch.where(frame == UNKNOWN, tok, frame)
    if force_delayed is not None:
        delayed[..., offset:offset + 1] = force_delayed[..., offset:offset + 1]
    kv.seqlen_offset += Lc + P + 1
    kv.lengths[:] += Lc + P + 1

    bias = torch.zeros_like(logits)
    bias[:, 1:, EOS] = -torch.inf
    bias[:, 0, EOS] -= torch.log(torch.tensor(1024.0))
    if force_full_length:
        bias[:, 0, EOS] = -torch.inf
    stopping = torch.zeros(B, dtype=torch.bool)
    max_steps = delayed.shape[2] - offset
    remaining = torch.full((B,), max_steps)
    steps_after = torch.full((B,), 6)
    eos_mode = torch.zeros(B, dtype=torch.bool)
    sp["repetition_penalty"] = torch.full((B,), float(sp["repetition_penalty"]))
    cfg_t = torch.tensor(cfg_scale)
    step = 0
    while torch.max(remaining) > 0:
        offset += 1
        step += 1
        ids = delayed[..., offset - 1:offset].repeat(2, 1, 1)
        logits = compute_logits(W, cfg, embed_codes(W, cfg, ids), kv, freqs, cfg_t)
        if trace is not None:
            trace["logits"].append(logits.clone())
        logits += bias
        sp["repetition_penalty"][eos_mode] = 1.0
        act = eos_mode & (steps_after > 0)
        logits[act, 0, EOS] = -torch.inf
        steps_after[act] -= 1
        gen = delayed[..., :offset]
        dec = [] if trace is not None else None
        tok = sample(logits, noise(step, 0), generated_tokens=gen, decision=dec, **sp)
        eos0 = tok[:, 0] == EOS
        new = eos0[:, 0] & (~eos_mode)
        if new.any():
            eos_mode[new] = True
            steps_after[new] = 6
            logits[new, 0, EOS] = -torch.inf
            tok = sample(logits, noise(step, 1), generated_tokens=gen, decision=dec, **sp)
            eos0 = tok[:, 0] == EOS
        remaining[eos0[:, 0]] = torch.minimum(remaining[eos0[:, 0]], torch.tensor(9))
        stopping |= eos0[:, 0]
        idx = torch.clamp(9 - remaining, max=8)
        for i in range(B):
            if stopping[i]:
                j = int(idx[i])
                tok[i, :j] = MASK
                tok[i, j] = EOS
        frame = delayed[..., offset:offset + 1]
        delayed[..., offset:offset + 1] = torch.where(frame == UNKNOWN, tok, frame)
        if force_delayed is not None:
            delayed[..., offset:offset + 1] = force_delayed[..., offset:offset + 1]
        if trace is not None:
            trace["tokens"].append(tok.clone())
            trace["decision"].append(dec)
        kv.seqlen_offset += 1
        kv.lengths[:] += 1
        remaining -= 1
        if max_steps_run is not None and step >= max_steps_run:
            break
    if trace is not None:
        trace["delayed"] = delayed.clone()
        trace["offset"] = offset
    return finalize(delayed, offset, P)


def forced_steps(W, cfg: BackboneCfg, cond: torch.Tensor, delayed: torch.Tensor, P: int, windows, sp: dict,
                 seed: int, row_base: int = 0, cfg_scale: float = 2.0, force_full_length: bool = True) -> dict:
    """Teacher-forced decode steps on a given delayed-code history (test instrumentation).

    For each window (s0, n): the cache is rebuilt by ONE prefill over cond + delayed[..., :P+1+s0]
    (model.py:181-202 -- the prefill path of the reference on the forced history; its logits are
    those of loop step s0), then steps s0+1 .. s0+n-1 run as single-token decodes
    (model.py:118-142) fed from the same history. At every step the logits get the loop's bias
    (model.py:332-334; step 0 = the prefill sample, no bias) and are sampled with the engine's noise
    key (seed, step, draw 0, row_base + b) (sampling.py:232-328). EOS is never accepted
    (force_full_length, the benchmark mode), so the EOS protocol does not enter. Returns {step:
    (raw CFG logits fp32 [B,9,V], token [B,9], decision margin [B,9])}.
    """
    R, Lc, _ = cond.shape
    B = R // 2
    rp = float(sp["repetition_penalty"])
    spk = {k: v for k, v in sp.items() if k != "repetition_penalty"}
    out = {}
    for s0, n in windows:
        kv = KVCache(cfg, R, Lc + delayed.shape[2] + 9)
        freqs = rope_table(16384, cfg.head_dim)
        ids = delayed[..., :P + 1 + s0].repeat(2, 1, 1)
        logits = compute_logits(W, cfg, torch.cat([cond, embed_codes(W, cfg, ids)], dim=1), kv, freqs, cfg_scale)
        kv.seqlen_offset += Lc + P + 1 + s0
        kv.lengths[:] += Lc + P + 1 + s0
        for j in range(n):
            s = s0 + j
            off = P + 1 + s
            if j > 0:
                ids = delayed[..., off - 1:off].repeat(2, 1, 1)
                logits = compute_logits(W, cfg, embed_codes(W, cfg, ids), kv, freqs, torch.tensor(cfg_scale))
                kv.seqlen_offset += 1
                kv.lengths[:] += 1
            raw = logits.clone()
            lg = logits.clone()
            if s > 0:
                lg[:, 1:, EOS] = -torch.inf
                lg[:, 0, EOS] -= torch.log(torch.tensor(1024.0))
            if force_full_length:
                lg[:, 0, EOS] = -torch.inf
            q = torch.from_numpy(exp_noise(seed, s, 0, B, cfg.n_cb, cfg.vocab, row_base))
            dec = []
            tok = sample(lg, q, generated_tokens=delayed[..., :off] if s > 0 else None,
                         repetition_penalty=torch.full((B,), rp), decision=dec, **spk)
            kind, arr = dec[-1]
            top = arr.topk(2, dim=-1).values
            m = (top[..., 0] - top[..., 1]) if kind == "logit" else torch.log(top[..., 0] / top[..., 1].clamp_min(1e-38))
            out[s] = (raw, tok[..., 0], m.float())
    return out


def finalize(delayed: torch.Tensor, offset: int, P: int):
    """Output trim (model.py:437-457)."""
    out = revert_delay(delayed)
    eos_pos = (out[:, 0, :] == EOS).int().argmax(dim=-1)
    eos_pos[eos_pos == 0] = out.shape[2]
    out = out[..., :offset - 9]
    out = out.masked_fill(out >= 1024, 0)
    return [out[i, :, P:int(eos_pos[i])].clone() for i in range(out.shape[0])]


def synthetic_conditioning(batch: int, Lc: int, D: int, seed: int = 1) -> torch.Tensor:
    """[2B, Lc, D] bf16 stand-in for PrefixConditioner output (ends in LayerNorm,
    conditioning.py:389) -- SURVEY.md §8(d) synthetic inputs."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(2 * batch, Lc, D, generator=g)
    return F.layer_norm(x, (D,)).to(torch.bfloat16)


def synthetic_prefix_codes(batch: int, P: int, seed: int = 3) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 1024, (batch, 9, P), generator=g)
