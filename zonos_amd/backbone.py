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

import dataclasses

import torch
import torch.nn as nn

from . import _lib
from ._lib import call, ptr
from .config import BackboneConfig, InferenceParams
from .engine import ATTN_CHUNK, EngineConfig, HipBackbone, _split_for, attn_splits_for
from .hybrid import HybridBackbone, HybridEngineConfig


class _Linear(nn.Module):
    def __init__(self, n_in, n_out):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(n_out, n_in), requires_grad=False)


class _LayerNorm(nn.Module):
    def __init__(self, d, bias: bool = True):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d), requires_grad=False)
        if bias:                     # (mamba_ssm RMSNorm has no bias parameter)
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


class _Conv1d(nn.Module):
    def __init__(self, channels, k):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(channels, 1, k), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(channels), requires_grad=False)


class _Mamba2(nn.Module):
    """Parameter container with mamba_ssm Mamba2's names (ngroups 1, no projection biases)."""

    def __init__(self, c: HybridEngineConfig):
        super().__init__()
        self.in_proj = _Linear(c.d_model, c.d_in_proj)
        self.conv1d = _Conv1d(c.conv_dim, c.d_conv)
        self.dt_bias = nn.Parameter(torch.zeros(c.nheads_ssm), requires_grad=False)
        self.A_log = nn.Parameter(torch.zeros(c.nheads_ssm), requires_grad=False)
        self.D = nn.Parameter(torch.ones(c.nheads_ssm), requires_grad=False)
        self.norm = nn.Module()
        self.norm.weight = nn.Parameter(torch.ones(c.d_inner), requires_grad=False)
        self.out_proj = _Linear(c.d_inner, c.d_model)


class _HybridBlock(nn.Module):
    """mamba_ssm Block names: norm + mixer (Mamba2 or MHA); attention blocks add norm2 + mlp, and so do
    Mamba2 blocks when d_intermediate != 0 (create_block); norms are bias-free RMSNorms under rms_norm."""

    def __init__(self, c: HybridEngineConfig, attn: bool):
        super().__init__()
        D = c.d_model
        self.norm = _LayerNorm(D, bias=not c.rms_norm)
        if attn:
            self.mixer = nn.Module()
            self.mixer.in_proj = _Linear(D, (c.n_heads + 2 * c.n_kv) * c.head_dim)
            self.mixer.out_proj = _Linear(c.n_heads * c.head_dim, D)
        else:
            self.mixer = _Mamba2(c)
        width = c.d_ff if attn else c.d_mlp
        if width:
            self.norm2 = _LayerNorm(D, bias=not c.rms_norm)
            self.mlp = nn.Module()
            self.mlp.fc1 = _Linear(D, 2 * width)
            self.mlp.fc2 = _Linear(width, D)


def _has_ssm_layers(config: BackboneConfig) -> bool:
    return len(set(config.attn_layer_idx or [])) < config.n_layer and bool(config.ssm_cfg)


class HipHybridBackbone(HipZonosBackbone):
    """The reference's MambaSSMZonosBackbone plugin (_mamba_ssm.py:9-57) on the MI355X kernels:
    Mamba2 and MHA blocks per ``attn_layer_idx`` with mamba_ssm's parameter names, so
    ``Zonos.load_state_dict`` of a hybrid checkpoint fills it unchanged.

    ``allocate_inference_cache(batch_size, max_seqlen, dtype)`` returns, like mamba_ssm's
    ``layer.allocate_inference_cache``, one pair per layer: ``(kv, None)`` for attention layers (the
    engine's fragment-order KV cache, zonos_amd/kvlayout.py) and ``(conv_state, ssm_state)`` for Mamba2
    layers -- bf16 ``[2][B][conv_dim][4]`` and ``[2][B][nheads][headdim][d_state]``, double-buffered by
    position parity (the step at position p reads buffer p & 1 and writes the other; zk_mamba_step).
    ``forward(hidden_states [B,S,D] bf16, inference_params)`` returns LayerNorm(hidden + residual)
    (layer_norm_fn of _mamba_ssm.py:50-57): a prefill (S > 1) at seqlen_offset 0 runs the causal conv and
    the exact recurrence and fills the states, a decode step (S == 1) advances them by one position."""

    supported_architectures = ["transformer", "hybrid"]

    def __init__(self, config: BackboneConfig):
        self.hybrid = _has_ssm_layers(config)
        if not self.hybrid:
            # transformer architecture: the transformer blocks (same parameter names), as the reference
            # prefers its torch backbone for a transformer config (model.py:70-75)
            super().__init__(dataclasses.replace(config, ssm_cfg={}))
            self.config = config
            return
        nn.Module.__init__(self)
        self.config = config
        self.ecfg = HybridEngineConfig.from_backbone_config(config)
        attn = set(self.ecfg.attn_layer_idx)
        self.layers = nn.ModuleList([_HybridBlock(self.ecfg, i in attn) for i in range(config.n_layer)])
        self.norm_f = _LayerNorm(config.d_model)
        self._core = None
        self._ws = None
        self.register_load_state_dict_post_hook(lambda *a, **k: self._invalidate())

    def _invalidate(self):
        self._core = None
        self._ws = None

    def _apply(self, fn, *a, **k):
        self._invalidate()
        return super()._apply(fn, *a, **k)

    def _engine(self) -> HybridBackbone:
        if not self.hybrid:
            return super()._engine()
        if self._core is None:
            dev = self.norm_f.weight.device
            _lib.require_gpu(self.norm_f.weight, "HipHybridBackbone parameters")
            self._core = HybridBackbone(self.ecfg, {k: v.detach() for k, v in self.state_dict().items()}, dev,
                                        prefix="")
        return self._core

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=torch.bfloat16):
        if not self.hybrid:
            return super().allocate_inference_cache(batch_size, max_seqlen, dtype)
        assert dtype == torch.bfloat16, "the HIP kernels keep bf16 caches and states"
        c = self.ecfg
        dev = self.norm_f.weight.device
        smax = -(-max_seqlen // ATTN_CHUNK) * ATTN_CHUNK
        cache = {}
        for i in range(c.n_layer):
            if i in c.attn_layer_idx:
                kv = torch.zeros(2, batch_size * c.n_kv * smax * c.head_dim, dtype=dtype, device=dev)
                cache[i] = (kv, None)
            else:
                conv = torch.zeros(2, batch_size, c.conv_dim, c.d_conv, dtype=dtype, device=dev)
                ssm = torch.zeros(2, batch_size, c.nheads_ssm, c.headdim, c.d_state, dtype=dtype, device=dev)
                cache[i] = (conv, ssm)
        return cache

    def _workspace(self, R: int, S: int, smax: int) -> dict:
        if not self.hybrid:
            return super()._workspace(R, S, smax)
        key = (R, S, smax)
        if self._ws is not None and self._ws["key"] == key:
            return self._ws
        c = self.ecfg
        dev = self.norm_f.weight.device
        D, H, Hk, hd, Fd = c.d_model, c.n_heads, c.n_kv, c.head_dim, c.d_ff
        di, nin = c.d_inner, c.d_in_proj
        Nqkv = (H + 2 * Hk) * hd
        M = R * S
        f32, bf = torch.float32, torch.bfloat16
        if S > 1:
            splits = dict(qkv=1, o=1, fc2=1, inp=1, out=1)
        else:      # the decode engine's split rule (zonos_amd/hybrid.py HybridDecoder._alloc)
            splits = dict(qkv=_split_for(Nqkv, D, R), o=_split_for(D, H * hd, R, target_blocks=128),
                          fc2=_split_for(D, max(Fd, 64), R), inp=1, out=_split_for(D, di, R))
        attn_splits = attn_splits_for(R, Hk, smax)
        if c.d_mlp and not Fd and S == 1:
            splits["fc2"] = _split_for(D, c.d_mlp, R)
        part_n = max(M * Nqkv * splits["qkv"], M * D * max(splits["o"], splits["fc2"], splits["out"]), M * nin)
        self._ws = dict(key=key, R=R, smax=smax, splits=splits, attn_splits=attn_splits,
                        x=torch.empty(M, D, dtype=bf, device=dev), xn=torch.empty(M, D, dtype=bf, device=dev),
                        xf=torch.empty(M, D, dtype=f32, device=dev) if c.residual_in_fp32 else None,
                        q=torch.empty(M, H * hd, dtype=bf, device=dev), y=torch.empty(M, H * hd, dtype=bf, device=dev),
                        h=torch.empty(M, max(Fd, c.d_mlp, 1), dtype=bf, device=dev),
                        part=torch.empty(part_n, dtype=f32, device=dev),
                        yz=torch.empty(M, di, dtype=f32, device=dev), ym=torch.empty(M, di, dtype=bf, device=dev),
                        xc=torch.empty(M, c.conv_dim, dtype=bf, device=dev),
                        attn_work=torch.empty(max(1, R * Hk * attn_splits * (8 + 4 * hd)), dtype=f32, device=dev),
                        scal=torch.zeros(16, dtype=torch.int32, device=dev))
        return self._ws

    def forward(self, hidden_states: torch.Tensor, inference_params: InferenceParams) -> torch.Tensor:
        if not self.hybrid:
            return super().forward(hidden_states, inference_params)
        core = self._engine()
        c = self.ecfg
        R, S, D = hidden_states.shape
        assert D == c.d_model and hidden_states.dtype == torch.bfloat16
        assert inference_params.batch_size_offset == 0
        kvd = inference_params.key_value_memory_dict
        smax = 0
        for i in core.attn_ids:
            smax = kvd[i][0].shape[1] // (R * c.n_kv * c.head_dim)
            assert smax * R * c.n_kv * c.head_dim == kvd[i][0].shape[1], "cache allocated for a different batch size"
        for i in core.mamba_ids:
            assert kvd[i][0].shape[1] == R, "state allocated for a different batch size"
        lengths = inference_params.lengths_per_sample
        pos = int(lengths[0]) if lengths is not None else inference_params.seqlen_offset
        if lengths is not None:
            assert bool((lengths == pos).all()), "rows at different positions"
        if S > 1:
            assert pos == 0, "prefill must start at position 0 (Mamba2.forward fills the states from zero)"
        assert not core.attn_ids or pos + S <= smax
        ws = self._workspace(R, S, max(smax, ATTN_CHUNK))
        ws["kv_layers"] = {i: kvd[i][0] for i in core.attn_ids}
        ws["state_layers"] = {i: kvd[i] for i in core.mamba_ids}
        stream = _lib.stream_ptr(hidden_states.device)
        M = R * S
        ws["x"].copy_(hidden_states.reshape(M, D))
        L0 = core.layers[0]
        if c.norm_flags:                            # rms_norm / residual_in_fp32: layer_norm_fn, residual None
            core._prenorm(ws, M, stream, None)
        else:
            call("zk_layernorm", ptr(ws["x"]), ptr(L0["ln1_w"]), ptr(L0["ln1_b"]), c.eps, M, D, ptr(ws["xn"]),
                 stream)
        if S == 1:
            ws["scal"][1] = pos                     # position of the new token (ctx - 1; state parity)
        core._layers(ws, M, R, S, S > 1, stream, None)
        return ws["xn"].reshape(R, S, D).clone()


# The registry (reference zonos/backbone/__init__.py:1-12): the hybrid-capable class first, as
# mamba_ssm's is when installed; the reference's own keys are aliases of the same classes.
BACKBONES = {"hip_hybrid": HipHybridBackbone, "hip": HipZonosBackbone,
             "mamba_ssm": HipHybridBackbone, "torch": HipZonosBackbone}
