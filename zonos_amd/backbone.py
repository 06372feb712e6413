"""The reference's backbone plugin, on the MI355X kernels: ``HipZonosBackbone``.

The reference selects its backbone from a registry (zonos/backbone/__init__.py:1-12,
``BACKBONES: dict[str, type]``) and drives it through one interface
(zonos/backbone/_torch.py:52-80): ``supported_architectures``, ``__init__(BackboneConfig)``,
``allocate_inference_cache(batch_size, max_seqlen, dtype) -> {layer_idx: (kv, None)}`` and
``forward(hidden_states [B,S,D] bf16, inference_params) -> [B,S,D] bf16`` (26 pre-LN blocks +
norm_f). ``HipZonosBackbone`` implements exactly that interface -- same parameter names
(``layers.{i}.norm``, ``.mixer.in_proj``, ``.mixer.out_proj``, ``.norm2``, ``.mlp.fc1``,
``.mlp.fc2``, ``norm_f``), so ``Zonos.load_state_dict`` fills it unchanged -- and runs every
block on the engine's HIP kernels. On the first forward after a load, the weights are packed into
the engine layout (fragment-packed GEMM weights, fc1 rows interleaved for the SwiGLU epilogue).

The KV cache it allocates is the engine's (per layer and (row, kv head), 32-key slices in MFMA
fragment order, zonos_amd/kvlayout.py), handed out as ``(kv, None)`` pairs like the reference's
``[B, S, 2, Hkv, hd]`` tensors: the cache is owned by InferenceParams and only this backbone reads
it. Prefill (S > 1) must start at seqlen_offset 0 -- the reference's own SDPA with
``is_causal=True`` is only correct there too (_torch.py:139) -- and decode runs one token per call
at ``lengths_per_sample``.

This is the per-call plugin path (one forward per step, like the reference's own loop). The
engine's generate() (zonos_amd.engine.HipDecoder) runs the same kernels with the whole step --
embeddings, heads, CFG, sampler, EOS protocol -- captured in one hipGraph.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from ._lib import call, ptr
from .config import BackboneConfig, InferenceParams
from .engine import ATTN_CHUNK, EngineConfig, HipBackbone, _split_for, attn_splits_for


class _Linear(nn.Module):
    def __init__(self, n_in, n_out):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n_out, n_in), requires_grad=False)


class _LayerNorm(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(d), requires_grad=False)


class _Block(nn.Module):
    """Parameter container with TransformerBlock's names (_torch.py:84-102)."""

    def __init__(self, c: EngineConfig):
        super().__init__()
        D, hd = c.d_model, c.head_dim
        self.norm = _LayerNorm(D)
        self.mixer = nn.Module()
        self.mixer.in_proj = _Linear(D, (c.n_heads + 2 * c.n_kv) * hd)
        self.mixer.out_proj = _Linear(c.n_heads * hd, D)
        self.norm2 = _LayerNorm(D)
        self.mlp = nn.Module()
        self.mlp.fc1 = _Linear(D, 2 * c.d_ff)
        self.mlp.fc2 = _Linear(c.d_ff, D)


class HipZonosBackbone(nn.Module):
    supported_architectures = ["transformer"]

    def __init__(self, config: BackboneConfig):
        assert not config.ssm_cfg, "This backbone implementation only supports the Transformer model."
        super().__init__()
        self.config = config
        self.ecfg = EngineConfig.from_backbone_config(config)
        self.layers = nn.ModuleList([_Block(self.ecfg) for _ in range(config.n_layer)])
        self.norm_f = _LayerNorm(config.d_model)
        self._core = None
        self._ws = None
        self.register_load_state_dict_post_hook(lambda *a, **k: self._invalidate())

    def _invalidate(self):
        self._core = None
        self._ws = None

    def _apply(self, fn, *a, **k):            # .to() / .cuda() move the parameters: repack on next use
        self._invalidate()
        return super()._apply(fn, *a, **k)

    def _engine(self) -> HipBackbone:
        if self._core is None:
            dev = self.norm_f.weight.device
            _lib.require_gpu(self.norm_f.weight, "HipZonosBackbone parameters")
            self._core = HipBackbone(self.ecfg, {k: v.detach() for k, v in self.state_dict().items()}, dev,
                                     prefix="")
        return self._core

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=torch.bfloat16):
        """_torch.py:64-71: one KV cache per layer, here in the engine layout (bf16 only)."""
        assert dtype == torch.bfloat16, "the HIP attention kernels read a bf16 cache"
        c = self.ecfg
        smax = -(-max_seqlen // ATTN_CHUNK) * ATTN_CHUNK
        kv = torch.zeros(c.n_layer, 2, batch_size * c.n_kv * smax * c.head_dim, dtype=dtype,
                         device=self.norm_f.weight.device)
        return {i: (kv[i], None) for i in range(c.n_layer)}

    def _workspace(self, R: int, S: int, smax: int) -> dict:
        key = (R, S, smax)
        if self._ws is not None and self._ws["key"] == key:
            return self._ws
        c = self.ecfg
        dev = self.norm_f.weight.device
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        Nqkv = (H + 2 * Hk) * hd
        M = R * S
        f32, bf = torch.float32, torch.bfloat16
        splits = dict(qkv=_split_for(Nqkv, D, M), o=_split_for(D, H * hd, M, target_blocks=128),
                      fc2=_split_for(D, Fd, M))
        if S > 1:
            splits = dict(qkv=1, o=1, fc2=1)
        attn_splits = attn_splits_for(R, Hk, smax)
        part_n = max(M * Nqkv * splits["qkv"], M * D * max(splits["o"], splits["fc2"]))
        self._ws = dict(key=key, R=R, smax=smax, splits=splits, attn_splits=attn_splits,
                        x=torch.empty(M, D, dtype=bf, device=dev), xn=torch.empty(M, D, dtype=bf, device=dev),
                        q=torch.empty(M, H * hd, dtype=bf, device=dev), y=torch.empty(M, H * hd, dtype=bf, device=dev),
                        h=torch.empty(M, Fd, dtype=bf, device=dev), part=torch.empty(part_n, dtype=f32, device=dev),
                        attn_work=torch.empty(max(1, R * Hk * attn_splits * (8 + 4 * hd)), dtype=f32, device=dev),
                        scal=torch.zeros(16, dtype=torch.int32, device=dev))
        return self._ws

    def forward(self, hidden_states: torch.Tensor, inference_params: InferenceParams) -> torch.Tensor:
        """_torch.py:73-80: positions from lengths_per_sample, the blocks, norm_f."""
        core = self._engine()
        c = self.ecfg
        R, S, D = hidden_states.shape
        assert D == c.d_model and hidden_states.dtype == torch.bfloat16
        assert inference_params.batch_size_offset == 0
        kvd = inference_params.key_value_memory_dict
        kv0 = kvd[0][0]
        smax = kv0.shape[1] // (R * c.n_kv * c.head_dim)
        assert smax * R * c.n_kv * c.head_dim == kv0.shape[1], "cache allocated for a different batch size"
        lengths = inference_params.lengths_per_sample
        pos = int(lengths[0]) if lengths is not None else inference_params.seqlen_offset
        if lengths is not None:
            assert bool((lengths == pos).all()), "rows at different positions"
        if S > 1:
            assert pos == 0, "prefill must start at position 0 (reference SDPA is_causal semantics)"
        assert pos + S <= smax
        ws = self._workspace(R, S, smax)
        ws["kv_layers"] = [kvd[i][0] for i in range(c.n_layer)]
        stream = _lib.stream_ptr(hidden_states.device)
        M = R * S
        ws["x"].copy_(hidden_states.reshape(M, D))
        L0 = core.layers[0]
        call("zk_layernorm", ptr(ws["x"]), ptr(L0["ln1_w"]), ptr(L0["ln1_b"]), c.eps, M, D, ptr(ws["xn"]), stream)
        if S == 1:
            ws["scal"][1] = pos                     # position of the new token (ctx - 1)
        core._layers(ws, M, R, S, S > 1, stream, None)
        return ws["xn"].reshape(R, S, D).clone()
