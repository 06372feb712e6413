"""Host-side view of the engine's KV-cache layout (backbone.hip k_off / v_off).

Per (row, kv head): Smax keys in 32-key slices of 8 KB, each slice stored in the order the
decode wave's MFMA fragments read it (one contiguous 1 KB load per fragment):
  K: [slice][h 2][ks 4][lane 64][8] -- lane = 16*lg + ln holds key 8*(ln>>2) + 4h + (ln&3)
     of the slice, dims 32*ks + 8*lg .. +8
  V: [slice][dt 8][lane 64][8]      -- lane holds channel 16*dt + ln, keys 8*lg .. 8*lg+7
Used by tests and tools to build / read caches; the engine never converts at run time.
"""
from __future__ import annotations

import torch


def pack_k(k: torch.Tensor) -> torch.Tensor:
    """[R][Hkv][S][128] (S % 32 == 0) -> packed [R][Hkv][S*128]."""
    R, Hk, S, hd = k.shape
    assert hd == 128 and S % 32 == 0
    # key = 32*sl + 8*grp + 4*h + i ; dim = 32*ks + 8*lg + e
    x = k.reshape(R, Hk, S // 32, 4, 2, 4, 4, 4, 8)          # sl grp h i | ks lg e
    x = x.permute(0, 1, 2, 4, 6, 7, 3, 5, 8)                 # sl h ks lg grp i e  (lane = 16lg + 4grp + i)
    return x.reshape(R, Hk, S * hd).contiguous()


def pack_v(v: torch.Tensor) -> torch.Tensor:
    """[R][Hkv][S][128] -> packed [R][Hkv][S*128]."""
    R, Hk, S, hd = v.shape
    assert hd == 128 and S % 32 == 0
    # key = 32*sl + 8*lg + e ; channel = 16*dt + ln
    x = v.reshape(R, Hk, S // 32, 4, 8, 8, 16)               # sl lg e | dt ln
    x = x.permute(0, 1, 2, 5, 3, 6, 4)                       # sl dt lg ln e
    return x.reshape(R, Hk, S * hd).contiguous()


def unpack_k(kp: torch.Tensor, S: int) -> torch.Tensor:
    R, Hk = kp.shape[:2]
    x = kp.reshape(R, Hk, S // 32, 2, 4, 4, 4, 4, 8)         # sl h ks lg grp i e
    x = x.permute(0, 1, 2, 6, 3, 7, 4, 5, 8)                 # sl grp h i ks lg e
    return x.reshape(R, Hk, S, 128)


def unpack_v(vp: torch.Tensor, S: int) -> torch.Tensor:
    R, Hk = vp.shape[:2]
    x = vp.reshape(R, Hk, S // 32, 8, 4, 16, 8)              # sl dt lg ln e
    x = x.permute(0, 1, 2, 4, 6, 3, 5)                       # sl lg e dt ln
    return x.reshape(R, Hk, S, 128)
