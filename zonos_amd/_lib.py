"""ctypes binding of libzonos_hip.so (the C ABI declared in include/zonos_hip.h).

The product path has no fallback: if the library is missing or fails to load, every
entry point raises. Device buffers are torch tensors; only their data_ptr() crosses the
ABI together with plain ints/floats and the current HIP stream.
"""
from __future__ import annotations

import ctypes as C  # noqa: N812
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZK_LIB_PATH") or os.path.join(_HERE, "lib", "libzonos_hip.so")

P = C.c_void_p
I = C.c_int
L = C.c_long
F = C.c_float
U64 = C.c_uint64
I64 = C.c_int64


class SamplingParams(C.Structure):
    _fields_ = [("temperature", F), ("top_p", F), ("min_p", F), ("linear", F), ("conf", F), ("quad", F),
                ("top_k", C.c_int32), ("rp_window", C.c_int32), ("cfg_scale", F),
                ("force_full_length", C.c_int32)]


class GenState(C.Structure):
    _fields_ = [("scal", P), ("eos_mode", P), ("steps_after", P), ("remaining", P), ("stopping", P),
                ("act", P), ("rp", P), ("tok0", P), ("tok1", P), ("delayed", P),
                ("B", C.c_int32), ("K", C.c_int32), ("Ld", C.c_int32), ("V", C.c_int32),
                ("seed", U64), ("row_base", C.c_int32), ("noise_mode", C.c_int32), ("noise_offset", U64),
                ("noise_stride", C.c_int32), ("noise_incr", C.c_int32)]


class StepLayer(C.Structure):
    _fields_ = [("ln1_w", P), ("ln1_b", P), ("wqkv", P), ("wo", P), ("ln2_w", P), ("ln2_b", P), ("fc1", P),
                ("fc2", P), ("k_cache", P), ("vt_cache", P)]


class StepDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("B", "n_layer", "d_model", "n_heads", "n_kv", "head_dim", "d_ff", "smax",
                                         "split_qkv", "split_o", "split_fc2", "split_heads", "attn_splits",
                                         "attn_merge", "rope_neox", "small")] + \
              [("eps", F), ("layers", P), ("emb", P), ("heads", P), ("lnf_w", P), ("lnf_b", P), ("freqs", P),
               ("x", P), ("xn", P), ("y", P), ("h", P), ("part", P), ("attn_work", P), ("attn_cnt", P), ("dbg", P),
               ("st", GenState), ("sp", SamplingParams)]


class HybridLayer(C.Structure):
    _fields_ = [("type", C.c_int32), ("d_mlp", C.c_int32), ("ln1_w", P), ("ln1_b", P), ("wqkv", P), ("wo", P),
                ("ln2_w", P), ("ln2_b", P), ("fc1", P), ("fc2", P), ("k_cache", P), ("vt_cache", P), ("w_in", P),
                ("conv_w", P), ("conv_b", P), ("A", P), ("dt_bias", P), ("Dskip", P), ("norm_w", P), ("w_out", P),
                ("conv_state", P * 2), ("ssm_state", P * 2)]


class HybridDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("B", "n_layer", "d_model", "n_heads", "n_kv", "head_dim", "d_ff", "smax",
                                         "d_inner", "nheads_ssm", "headdim_ssm", "d_state", "split_qkv", "split_o",
                                         "split_fc2", "split_heads", "split_inp", "split_out", "attn_splits",
                                         "norm_flags")] + \
              [("eps", F), ("gate_eps", F), ("layers", P), ("emb", P), ("heads", P), ("lnf_w", P), ("lnf_b", P),
               ("freqs", P), ("x", P), ("xn", P), ("y", P), ("h", P), ("part", P), ("attn_work", P), ("yz", P),
               ("ym", P), ("xc", P), ("dbg", P), ("st", GenState), ("sp", SamplingParams), ("xf", P)]


class DacResUnit(C.Structure):
    _fields_ = [("dil", C.c_int32), ("a1", P), ("w1", P), ("b1", P), ("a2", P), ("w2", P), ("b2", P)]


DAC_MAXB, DAC_MAXR = 6, 3


class DacBlock(C.Structure):
    _fields_ = [("stride", C.c_int32), ("cin", C.c_int32), ("cout", C.c_int32), ("nres", C.c_int32),
                ("alpha", P), ("wt", P), ("bt", P), ("res", DacResUnit * DAC_MAXR)]


class DacDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("nblocks", "ncb", "codebook_size", "hidden", "cin0", "c0")] + \
              [("tables", P), ("conv1_w", P), ("conv1_b", P), ("final_alpha", P), ("conv2_w", P), ("conv2_b", P),
               ("blocks", DacBlock * DAC_MAXB)]


# name -> argtypes (all return int status)
_SIGS = {
    "zk_version": [],
    "zk_device_sync": [],
    "zk_sample_logits": [P, I, I, I, P, I, I, P, C.POINTER(SamplingParams), U64, I, I, I, P, P],
    "zk_sample_logits_torch": [P, I, I, I, P, I, I, P, C.POINTER(SamplingParams), U64, U64, I, P, P],
    "zk_torch_exponential": [P, L, U64, U64, I, P],
    "zk_delay_apply": [P, I, I, I, I64, P, P],
    "zk_delay_revert": [P, I, I, I, P, P],
    "zk_embed_codes": [P, I, I, I, L, L, P, I, P, I, I, I, P, I, I, P, P, F, P, P, P],
    "zk_layernorm": [P, P, P, F, I, I, P, P],
    "zk_resid_ln": [P, I, P, P, P, F, I, I, P, P, I, P, P],
    "zk_gemm_bf16": [P, L, P, I, I, I, I, I, P, P, P, P],
    "zk_gemv_fused": [P, L, P, I, I, I, I, P, P, F, P, P, P, P],
    "zk_permute_fc1": [P, I, I, P, P],
    "zk_pack_weights": [P, I, I, P, P],
    "zk_qkv_rope": [P, I, I, I, I, I, I, P, I, P, P, P, P, I, P, I, P, P],
    "zk_attn_decode": [P, P, P, I, I, I, I, I, I, P, P, I, P, P, P],
    "zk_attn_decode_qkv": [P, I, P, P, P, I, I, I, I, I, I, P, P, I, P, I, P, P],
    "zk_attn_decode_qkv_sc": [P, I, P, P, P, I, I, I, I, I, I, P, P, I, P, P, I, P, P],
    "zk_attn_decode_qkv_part": [P, I, P, P, P, I, I, I, I, I, I, P, P, I, I, P, P],
    "zk_gemv_attn_out": [P, I, I, P, I, I, I, P, P, P],
    "zk_gemv_qkv_rope": [P, P, I, I, I, I, P, P, F, P, P, P, I, P, P, P, P],
    "zk_attn_decode_q_part": [P, P, P, I, I, I, I, I, I, P, P, I, P, P],
    "zk_decode_step": [C.POINTER(StepDesc), P],
    "zk_prefill": [C.POINTER(StepDesc), P, I, I, P, P],
    "zk_hybrid_decode_step": [C.POINTER(HybridDesc), P],
    "zk_hybrid_prefill": [C.POINTER(HybridDesc), P, I, I, P, P],
    "zk_dac_decode": [C.POINTER(DacDesc), P, I, I, P, P, C.c_size_t, P, P],
    "zk_mamba_step": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "zk_mamba_step_per_head": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "zk_mamba_prefill": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P],
    "zk_gated_rmsnorm": [P, I, I, P, F, P, P, P],
    "zk_attn_prefill": [P, P, P, I, I, I, I, I, I, P, P],
    "zk_sample_heads": [P, I, C.POINTER(GenState), C.POINTER(SamplingParams), I, I, P, P],
    "zk_eos_step": [C.POINTER(GenState), I, I, P],
    "zk_graph_begin": [P],
    "zk_graph_end": [P, C.POINTER(P)],
    "zk_graph_launch": [P, I, P],
    "zk_graph_destroy": [P],
    "zk_event_create": [C.POINTER(P)],
    "zk_event_record": [P, P],
    "zk_event_elapsed_ms": [P, P, C.POINTER(F)],
    "zk_event_destroy": [P],
    "zk_dac_rvq_tables": [P, P, P, I, I, I, I, P, P],
    "zk_dac_rvq_decode": [P, I, I, I, L, P, I, I, P, I, P, P],
    "zk_dac_conv": [P, I, I, I, P, P, P, I, I, I, I, I, I, I, P, I, P, I, P, I, I, P],
    "zk_dac_prep_convt": [P, I, I, I, P, P],
    "zk_dac_prep_w16": [P, I, I, I, I, I, P, P, P],
    "zk_dac_conv16": [P, I, I, I, P, P, P, P, I, I, I, I, I, I, I, P, I, P, I, P, I, I, I, P],
    "zk_dac_tail": [P, I, I, I, P, P, P, P, P, I, P],
    "zk_dac_rvq_decode_cl": [P, I, I, I, L, P, I, I, I, P, P, P],
    "zk_dac_conv_cl": [P, I, I, I, P, L, P, I, I, I, I, I, I, I, I, I, P, P, P, P, I, P, I, I, P],
    "zk_dac_tail_cl": [P, I, I, I, P, P, P, P, I, P],
    "zk_dac_resunit_cl": [P, I, I, I, P, P, I, P, P, P, P, P, P, I, P, I, P],
    "zk_dac_enc_conv1": [P, I, I, P, P, P, I, I, P, P, P],
    "zk_dac_rvq_encode": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P],
    "zk_resample": [P, I, L, P, I, I, I, I, P, L, P],
    "zk_prefix_cond": [P, I, P, P],
    "zk_loudness_gains": [P, I, L, P, I, C.c_double, P, P, P, P],
}

_lib = None


class ZonosHipError(RuntimeError):
    pass


def load():
    """Load (and type) the library. Raises ZonosHipError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZonosHipError(f"{LIB_PATH} not found: build it with `python -m zonos_amd.build` "
                            "(there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    lib.zk_last_error.restype = C.c_char_p
    lib.zk_last_error.argtypes = []
    lib.zk_loudness_max_blocks.restype = C.c_int
    lib.zk_loudness_max_blocks.argtypes = [L, I]
    lib.zk_abi_size.restype = C.c_long
    lib.zk_abi_size.argtypes = [I]
    lib.zk_dac_decode_workspace.restype = C.c_size_t
    lib.zk_dac_decode_workspace.argtypes = [C.POINTER(DacDesc), I, I]
    lib.zk_dac_resunit_supported.restype = C.c_int
    lib.zk_dac_resunit_supported.argtypes = [I]
    lib.zk_gemm_warm_tiles.restype = C.c_int
    lib.zk_gemm_warm_tiles.argtypes = [I, I, I, I, I, I]
    lib.zk_torch_noise_policy.restype = C.c_int
    lib.zk_torch_noise_policy.argtypes = [L, I, I, C.POINTER(C.c_int), C.POINTER(C.c_long)]
    _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return list(_SIGS) + ["zk_last_error", "zk_loudness_max_blocks", "zk_abi_size",
                          "zk_dac_decode_workspace", "zk_dac_resunit_supported", "zk_gemm_warm_tiles",
                          "zk_torch_noise_policy"]


def call(name: str, *args):
    lib = load()
    if len(args) != len(_SIGS[name]):
        raise TypeError(f"{name}: {len(args)} arguments given, the C ABI takes {len(_SIGS[name])}")
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise ZonosHipError(f"{name} failed ({rc}): {lib.zk_last_error().decode()}")
    return rc


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def device_index(device) -> int:
    """The GPU index a (possibly unindexed) cuda device means: torch.device("cuda") is the current
    device (torch.cuda.set_device), not GPU 0 -- the index of the generator torch itself would use."""
    device = torch.device(device)
    return device.index if device.index is not None else torch.cuda.current_device()


def require_gpu(t: torch.Tensor, name: str = "tensor"):
    if not t.is_cuda:
        raise ZonosHipError(f"{name} must be a GPU tensor (the HIP engine has no CPU path)")
