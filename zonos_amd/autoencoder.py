"""DAC decoder on the GPU: the decode half of zonos/autoencoder.py (DACAutoencoder.decode
44-47, codes_to_wavs 188-245, save_codes 247-268) over hand-written HIP kernels
(zonos_amd/csrc/dac.hip), restating transformers' DacModel.decode (modeling_dac.py:610-640).

Batching: codes_to_wavs in the reference decodes one utterance at a time
(autoencoder.py:219-226). Here a list of utterances is decoded as ONE zero-padded batch
with per-row valid lengths; every conv reads zeros beyond a row's length, which is
exactly the padding the standalone decode of that row would see, so each waveform equals
its per-utterance decode.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from . import _lib
from ._lib import call, ptr


class DacSpec:
    """descript/dac_44khz decoder geometry (configuration_dac.py defaults)."""

    def __init__(self, hidden_size=1024, decoder_hidden_size=1536, upsampling_ratios=(8, 8, 4, 2), n_codebooks=9,
                 codebook_size=1024, codebook_dim=8, sampling_rate=44100):
        self.hidden_size = hidden_size
        self.decoder_hidden_size = decoder_hidden_size
        self.upsampling_ratios = tuple(upsampling_ratios)
        self.n_codebooks = n_codebooks
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.sampling_rate = sampling_rate

    @property
    def hop_length(self):
        return int(math.prod(self.upsampling_ratios))

    @classmethod
    def from_hf_config(cls, d: dict) -> "DacSpec":
        return cls(d.get("hidden_size", 1024), d.get("decoder_hidden_size", 1536),
                   tuple(d.get("upsampling_ratios", (8, 8, 4, 2))), d.get("n_codebooks", 9),
                   d.get("codebook_size", 1024), d.get("codebook_dim", 8), d.get("sampling_rate", 44100))


def _fold_weight_norm(sd: dict) -> dict:
    """Accept weight-normalised checkpoints (weight_g/weight_v or parametrizations.*.original0/1)."""
    out = dict(sd)
    for k in list(sd):
        for g_suf, v_suf, base in ((".weight_g", ".weight_v", ".weight"),
                                   (".parametrizations.weight.original0", ".parametrizations.weight.original1",
                                    ".weight")):
            if k.endswith(g_suf):
                stem = k[: -len(g_suf)]
                g, v = sd[k].float(), sd[stem + v_suf].float()
                norm = v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
                out[stem + base] = g * v / norm
                out.pop(k, None)
                out.pop(stem + v_suf, None)
    return out


class HipDacDecoder:
    """Decoder weights on the device + the launch sequence of the DAC decoder.

    precision: "fp16" (default; the reference's own GPU numerics -- autocast fp16 around
    DacModel.decode, autoencoder.py:46 -- on the channels-last pipeline of dac_cl.hip: fp16
    conv operands, fp32 accumulation and fp32 residual stream), "fp16x3" (split-precision
    fp16 MFMA, ~fp32 accuracy) or "fp32" (exact-fp32 MFMA kernel); the last two match the
    reference's CPU fp32 decode to ~1e-6 RMS and run channels-first."""

    def __init__(self, spec: DacSpec, state_dict: dict, device="cuda", precision: str = "fp16"):
        _lib.load()
        assert precision in ("fp16x3", "fp16", "fp32"), precision
        self.precision = precision
        self.spec = spec
        self.device = torch.device(device)
        sd = _fold_weight_norm(state_dict)
        dev = self.device

        def t(k):
            return sd[k].to(device=dev, dtype=torch.float32).contiguous()

        s = spec
        stream = _lib.stream_ptr(dev)
        cbs = torch.stack([t(f"quantizer.quantizers.{k}.codebook.weight") for k in range(s.n_codebooks)])
        ows = torch.stack([t(f"quantizer.quantizers.{k}.out_proj.weight").reshape(s.hidden_size, s.codebook_dim)
                           for k in range(s.n_codebooks)])
        obs = torch.stack([t(f"quantizer.quantizers.{k}.out_proj.bias") for k in range(s.n_codebooks)])
        self.tables = torch.empty(s.n_codebooks, s.codebook_size, s.hidden_size, device=dev)
        call("zk_dac_rvq_tables", ptr(cbs.contiguous()), ptr(ows.contiguous()), ptr(obs.contiguous()),
             s.n_codebooks, s.codebook_size, s.codebook_dim, s.hidden_size, ptr(self.tables), stream)
        self.conv1_w, self.conv1_b = t("decoder.conv1.weight"), t("decoder.conv1.bias")
        self.blocks = []
        self._convt_raw = []
        for i, st in enumerate(s.upsampling_ratios):
            p = f"decoder.block.{i}."
            wt = t(p + "conv_t1.weight")                      # [Cin][Cout][2s]
            self._convt_raw.append(wt)
            cin, cout = wt.shape[0], wt.shape[1]
            wprep = torch.empty(st, cout, cin, 2, device=dev)
            call("zk_dac_prep_convt", ptr(wt), cin, cout, st, ptr(wprep), stream)
            blk = dict(stride=st, cin=cin, cout=cout, alpha=t(p + "snake1.alpha").reshape(-1), wt=wprep,
                       bt=t(p + "conv_t1.bias"), res=[])
            for r, dil in ((1, 1), (2, 3), (3, 9)):
                u = p + f"res_unit{r}."
                blk["res"].append(dict(dil=dil, a1=t(u + "snake1.alpha").reshape(-1), w1=t(u + "conv1.weight"),
                                       b1=t(u + "conv1.bias"), a2=t(u + "snake2.alpha").reshape(-1),
                                       w2=t(u + "conv2.weight"), b2=t(u + "conv2.bias")))
            self.blocks.append(blk)
        self.final_alpha = t("decoder.snake1.alpha").reshape(-1)
        self.conv2_w, self.conv2_b = t("decoder.conv2.weight"), t("decoder.conv2.bias")
        if precision == "fp16":
            self._prep_cl(stream)
        elif precision != "fp32":
            self.w16 = {}
            self._prep16("conv1", self.conv1_w, 0, stream)
            for i, blk in enumerate(self.blocks):
                self._prep16(f"b{i}.t", t(f"decoder.block.{i}.conv_t1.weight"), 1, stream, s=blk["stride"])
                for j, ru in enumerate(blk["res"]):
                    self._prep16(f"b{i}.r{j}.1", ru["w1"], 0, stream)
                    self._prep16(f"b{i}.r{j}.2", ru["w2"], 0, stream)
        torch.cuda.synchronize(dev)

    # ---------------------------------------------------------------- channels-last fp16 path
    @staticmethod
    def _pad32(c):
        return (c + 31) // 32 * 32

    def _prep_cl(self, stream):
        """Weights for dac_cl.hip: channels zero-padded to multiples of 32, fp16 [tap][Cout][Cin]
        (ConvTranspose1d: [phase][2][Cout][Cin]); biases padded with 0, Snake alphas with 1."""
        dev, s, P = self.device, self.spec, self._pad32

        def wconv(w):                       # [Cout][Cin][ks] -> fp16 [ks][Cout_p][Cin_p]
            co, ci, ks = w.shape
            wp = torch.zeros(P(co), P(ci), ks, device=dev)
            wp[:co, :ci] = w
            out = torch.empty(ks * P(co) * P(ci), dtype=torch.int16, device=dev)
            call("zk_dac_prep_w16", ptr(wp), P(co), P(ci), ks, 1, 0, ptr(out), None, stream)
            return out

        def wconvt(w, st):                  # [Cin][Cout][2s] -> fp16 [s][2][Cout_p][Cin_p]
            ci, co, _ = w.shape
            wp = torch.zeros(P(ci), P(co), 2 * st, device=dev)
            wp[:ci, :co] = w
            out = torch.empty(st * 2 * P(co) * P(ci), dtype=torch.int16, device=dev)
            call("zk_dac_prep_w16", ptr(wp), P(co), P(ci), 2, st, 1, ptr(out), None, stream)
            return out

        def vec(v, fill):
            out = torch.full((P(v.numel()),), fill, device=dev)
            out[:v.numel()] = v.reshape(-1)
            return out

        cl = {"cin0": P(s.hidden_size), "c0": P(self.conv1_w.shape[0]), "conv1_w": wconv(self.conv1_w),
              "conv1_b": vec(self.conv1_b, 0.0), "blocks": []}
        for blk in self.blocks:
            st = blk["stride"]
            b = {"stride": st, "cin": P(blk["cin"]), "cout": P(blk["cout"]), "alpha": vec(blk["alpha"], 1.0),
                 "wt": wconvt(self._convt_raw[len(cl["blocks"])], st), "bt": vec(blk["bt"], 0.0), "res": []}
            for ru in blk["res"]:
                b["res"].append({"dil": ru["dil"], "a1": vec(ru["a1"], 1.0), "w1": wconv(ru["w1"]),
                                 "b1": vec(ru["b1"], 0.0), "a2": vec(ru["a2"], 1.0), "w2": wconv(ru["w2"]),
                                 "b2": vec(ru["b2"], 0.0)})
            cl["blocks"].append(b)
        cl["final_alpha"] = vec(self.final_alpha, 1.0)
        cw = torch.zeros(P(self.conv2_w.shape[1]), 7, device=dev)
        cw[:self.conv2_w.shape[1]] = self.conv2_w[0]
        cl["conv2_w"], cl["conv2_b"] = cw.contiguous(), self.conv2_b.contiguous()
        self.cl = cl

    # the decode's launch sequence is enqueued by the C ABI (zk_dac_decode); False issues the
    # same sequence from Python (bit-identical; the reference for the test)
    c_dac = True
    # Python-issued sequence: residual units fused where zk_dac_resunit_supported says so, as in
    # zk_dac_decode; False = every unit as two convs (tests only)
    fuse_units = True

    def _dac_desc(self):
        if getattr(self, "_desc", None) is None:
            s, cl = self.spec, self.cl
            d = _lib.DacDesc()
            d.nblocks, d.ncb, d.codebook_size = len(cl["blocks"]), s.n_codebooks, s.codebook_size
            d.hidden, d.cin0, d.c0 = s.hidden_size, cl["cin0"], cl["c0"]
            d.tables, d.conv1_w, d.conv1_b = ptr(self.tables), ptr(cl["conv1_w"]), ptr(cl["conv1_b"])
            d.final_alpha, d.conv2_w, d.conv2_b = ptr(cl["final_alpha"]), ptr(cl["conv2_w"]), ptr(cl["conv2_b"])
            assert len(cl["blocks"]) <= _lib.DAC_MAXB
            for i, blk in enumerate(cl["blocks"]):
                b = d.blocks[i]
                b.stride, b.cin, b.cout, b.nres = blk["stride"], blk["cin"], blk["cout"], len(blk["res"])
                b.alpha, b.wt, b.bt = ptr(blk["alpha"]), ptr(blk["wt"]), ptr(blk["bt"])
                assert len(blk["res"]) <= _lib.DAC_MAXR
                for j, ru in enumerate(blk["res"]):
                    b.res[j] = _lib.DacResUnit(ru["dil"], ptr(ru["a1"]), ptr(ru["w1"]), ptr(ru["b1"]), ptr(ru["a2"]),
                                               ptr(ru["w2"]), ptr(ru["b2"]))
            self._desc = d
        return self._desc

    def _decode_cl(self, codes, lens, stream):
        s, cl, dev = self.spec, self.cl, self.device
        B, K, T = codes.shape
        if self.c_dac and cl["blocks"]:
            d = self._dac_desc()
            d.ncb = K
            nbytes = _lib.load().zk_dac_decode_workspace(C.byref(d), B, T)
            if nbytes == 0:
                raise _lib.ZonosHipError("zk_dac_decode_workspace: bad descriptor")
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            hop = 1
            for blk in cl["blocks"]:
                hop *= blk["stride"]
            out = torch.empty(B, 1, T * hop, device=dev)
            call("zk_dac_decode", C.byref(d), ptr(codes.contiguous()), B, T, ptr(lens), ptr(ws), nbytes, ptr(out),
                 stream)
            self._ws_keep = ws          # freed at the next decode (stream-ordered reuse)
            return out
        f16 = torch.int16
        z = torch.empty(B, T, cl["cin0"], dtype=f16, device=dev)
        call("zk_dac_rvq_decode_cl", ptr(codes), B, K, T, K * T, ptr(self.tables), s.codebook_size, s.hidden_size,
             cl["cin0"], ptr(z), ptr(lens), stream)
        blocks = cl["blocks"]
        a_next = blocks[0]["alpha"] if blocks else cl["final_alpha"]
        act = torch.empty(B, T, cl["c0"], dtype=f16, device=dev)
        call("zk_dac_conv_cl", ptr(z), B, cl["cin0"], T, ptr(cl["conv1_w"]), 0, ptr(cl["conv1_b"]), cl["c0"], 7, 1, 3,
             T, 1, 1, 0, T, None, None, ptr(a_next), ptr(act), 0, ptr(lens), 1, 1, stream)
        del z
        L, scale = T, 1
        for bi, blk in enumerate(blocks):
            st, cin, cout = blk["stride"], blk["cin"], blk["cout"]
            Lo = L * st
            x = torch.empty(B, Lo, cout, device=dev)
            s_new = torch.empty(B, Lo, cout, dtype=f16, device=dev)
            a1 = blk["res"][0]["a1"]
            call("zk_dac_conv_cl", ptr(act), B, cin, L, ptr(blk["wt"]), 2 * cout * cin, ptr(blk["bt"]), cout, 2, 1, 1,
                 L + 1, st, st, -((st + 1) // 2), Lo, None, ptr(x), ptr(a1), ptr(s_new), 0, ptr(lens), scale,
                 scale * st, stream)
            act = s_new
            scale *= st
            L = Lo
            tmp = torch.empty_like(act)
            nres = len(blk["res"])
            for j, ru in enumerate(blk["res"]):
                d = ru["dil"]
                if j + 1 < nres:
                    a_next = blk["res"][j + 1]["a1"]
                elif bi + 1 < len(blocks):
                    a_next = blocks[bi + 1]["alpha"]
                else:
                    a_next = cl["final_alpha"]
                last = j + 1 == nres and bi + 1 == len(blocks)
                fm = _lib.load().zk_dac_resunit_supported(cout) if self.fuse_units else 0
                if fm == 2 or (fm == 1 and not last):
                    # the whole unit in one launch, into the other buffer (the k7 reads its input's halo)
                    out = torch.empty(B, L, cout, device=dev) if last else tmp
                    call("zk_dac_resunit_cl", ptr(act), B, cout, L, ptr(ru["w1"]), ptr(ru["b1"]), d, ptr(ru["a2"]),
                         ptr(ru["w2"]), ptr(ru["b2"]), ptr(x), ptr(a_next), ptr(out), int(last), ptr(lens), scale,
                         stream)
                    act, tmp = out, act
                    continue
                call("zk_dac_conv_cl", ptr(act), B, cout, L, ptr(ru["w1"]), 0, ptr(ru["b1"]), cout, 7, d, 3 * d, L,
                     1, 1, 0, L, None, None, ptr(ru["a2"]), ptr(tmp), 0, ptr(lens), scale, scale, stream)
                if last:       # the tail's input: fp32 Snake output (keeps the waveform at fp32-level error)
                    act = torch.empty(B, L, cout, device=dev)
                call("zk_dac_conv_cl", ptr(tmp), B, cout, L, ptr(ru["w2"]), 0, ptr(ru["b2"]), cout, 1, 1, 0, L,
                     1, 1, 0, L, ptr(x), ptr(x), ptr(a_next), ptr(act), int(last), ptr(lens), scale, scale, stream)
            del tmp, x
        out = torch.empty(B, 1, L, device=dev)
        call("zk_dac_tail_cl", ptr(act), B, act.shape[2], L, ptr(cl["conv2_w"]), ptr(cl["conv2_b"]), ptr(out),
             ptr(lens), scale, stream)
        return out

    def _prep16(self, key, w, mode, stream, s=1):
        if mode == 0:
            cout, cin, ks = w.shape
            n = cout * cin * ks
        else:
            cin, cout, k2 = w.shape
            ks = 2
            n = s * 2 * cout * cin
        hi = torch.empty(n, dtype=torch.int16, device=self.device)
        lo = torch.empty(n, dtype=torch.int16, device=self.device)
        call("zk_dac_prep_w16", ptr(w), cout, cin, ks, s, mode, ptr(hi), ptr(lo), stream)
        self.w16[key] = (hi, lo, cout * cin)

    def _conv(self, x, B, Cin, Tin, alpha, w, b, Cout, ks, dil, pad, Qn, ostride, ooff, out, Tout, resid, tanh,
              lens, in_scale, out_scale, stream, key=None, phase=0):
        if self.precision != "fp32" and key is not None and Cin % 32 == 0:
            hi, lo, per = self.w16[key]
            off = phase * 2 * per * 2          # bytes: phase r of a ConvTranspose1d pack
            npass = 3 if self.precision == "fp16x3" else 1
            call("zk_dac_conv16", ptr(x), B, Cin, Tin, ptr(alpha), hi.data_ptr() + off, lo.data_ptr() + off, ptr(b),
                 Cout, ks, dil, pad, Qn, ostride, ooff, ptr(out), Tout, ptr(resid), int(tanh), ptr(lens), in_scale,
                 out_scale, npass, stream)
            return
        call("zk_dac_conv", ptr(x), B, Cin, Tin, ptr(alpha), ptr(w), ptr(b), Cout, ks, dil, pad, Qn, ostride, ooff,
             ptr(out), Tout, ptr(resid), int(tanh), ptr(lens), in_scale, out_scale, stream)

    @torch.inference_mode()
    def decode_padded(self, codes: torch.Tensor, lens: torch.Tensor | None = None) -> torch.Tensor:
        """codes int64 [B][9][T] on device -> waveform fp32 [B][1][hop*T].
        lens (int32 [B], frames) marks each row's valid length; None = all T."""
        s = self.spec
        dev = self.device
        codes = codes.to(device=dev, dtype=torch.int64).contiguous()
        B, K, T = codes.shape
        assert K == s.n_codebooks, f"Expected {s.n_codebooks} codebooks, got {K}"   # autoencoder.py:45
        stream = _lib.stream_ptr(dev)
        if lens is not None:
            lens = lens.to(device=dev, dtype=torch.int32).contiguous()
        if self.precision == "fp16":
            return self._decode_cl(codes, lens, stream)
        z = torch.empty(B, s.hidden_size, T, device=dev)
        call("zk_dac_rvq_decode", ptr(codes), B, K, T, K * T, ptr(self.tables), s.codebook_size, s.hidden_size,
             ptr(z), T, ptr(lens), stream)
        C0 = self.conv1_w.shape[0]
        x = torch.empty(B, C0, T, device=dev)
        self._conv(z, B, s.hidden_size, T, None, self.conv1_w, self.conv1_b, C0, 7, 1, 3, T, 1, 0, x, T, None,
                   False, lens, 1, 1, stream, key="conv1")
        del z
        L, scale = T, 1
        for bi, blk in enumerate(self.blocks):
            st, cin, cout = blk["stride"], blk["cin"], blk["cout"]
            Lo = L * st
            y = torch.empty(B, cout, Lo, device=dev)
            p = math.ceil(st / 2)
            for r in range(st):
                self._conv(x, B, cin, L, blk["alpha"], blk["wt"][r], blk["bt"], cout, 2, 1, 1, L + 1, st, r - p, y,
                           Lo, None, False, lens, scale, scale * st, stream, key=f"b{bi}.t", phase=r)
            del x
            scale *= st
            L = Lo
            tmp = torch.empty_like(y)
            for j, ru in enumerate(blk["res"]):
                d = ru["dil"]
                self._conv(y, B, cout, L, ru["a1"], ru["w1"], ru["b1"], cout, 7, d, 3 * d, L, 1, 0, tmp, L, None,
                           False, lens, scale, scale, stream, key=f"b{bi}.r{j}.1")
                self._conv(tmp, B, cout, L, ru["a2"], ru["w2"], ru["b2"], cout, 1, 1, 0, L, 1, 0, y, L, y, False,
                           lens, scale, scale, stream, key=f"b{bi}.r{j}.2")
            del tmp
            x = y
        out = torch.empty(B, 1, L, device=dev)
        cl = x.shape[1]
        if self.precision == "fp32":
            self._conv(x, B, cl, L, self.final_alpha, self.conv2_w, self.conv2_b, 1, 7, 1, 3, L, 1, 0, out, L, None,
                       True, lens, scale, scale, stream)
        else:
            call("zk_dac_tail", ptr(x), B, cl, L, ptr(self.final_alpha), ptr(self.conv2_w), ptr(self.conv2_b),
                 ptr(out), ptr(lens), scale, stream)
        return out

    def decode_list(self, codes_list, max_batch_bytes: float = 64e9) -> list:
        """Per-utterance waveforms for a list of [9, T_i] / [1, 9, T_i] code tensors, decoded as
        zero-padded batches (chunks bounded by activation memory, default 64 GB of HBM)."""
        items = []
        for c in codes_list:
            c = c.unsqueeze(0) if c.dim() == 2 else c
            for j in range(c.shape[0]):
                items.append(c[j])
        results = [None] * len(items)
        order = [i for i in range(len(items)) if items[i].shape[1] > 0]
        order.sort(key=lambda i: -items[i].shape[1])
        hop = self.spec.hop_length
        width = self.blocks[-1]["cout"] if self.blocks else self.spec.decoder_hidden_size
        i = 0
        while i < len(order):
            Tmax = items[order[i]].shape[1]
            # live activations at the widest-time stage: channels-last fp32 x + 2 fp16 (+ the
            # previous stage's fp16 input) ~ 10 B per (position, channel); channels-first fp32 ~ 12 B
            per_bytes = (10 if self.precision == "fp16" else 12) * self._pad32(width) * hop * Tmax
            per = max(1, int(max_batch_bytes // per_bytes))
            grp = order[i:i + per]
            codes = torch.zeros(len(grp), self.spec.n_codebooks, Tmax, dtype=torch.int64, device=self.device)
            lens = torch.tensor([items[g].shape[1] for g in grp], dtype=torch.int32)
            for j, g in enumerate(grp):
                codes[j, :, :items[g].shape[1]] = items[g].to(self.device)
            wav = self.decode_padded(codes, lens)
            for j, g in enumerate(grp):
                results[g] = wav[j, :, : int(lens[j]) * hop]
            i += per
        return [r for r in results if r is not None]


class HipDacEncoder:
    """DAC encoder + residual-VQ encode on the GPU: DACAutoencoder.encode (autoencoder.py:27-28)
    -> DacModel.encode (modeling_dac DacEncoder, DacResidualVectorQuantizer eval path).

    Channels-last, on the same conv kernel as the decoder (zk_dac_conv_cl: fp16 operands, fp32
    accumulation, fp32 residual stream -- the reference runs this fp32 under cuDNN's default
    TF32 convolutions, a comparable 10-bit-mantissa operand precision). The strided
    Conv1d(k=2s, stride s, pad s/2) of each block runs as a stride-1 3-tap convolution over the
    activation viewed as [T/s][s*C] (a free reshape of channels-last memory) with host-repacked
    weights W'[tap][co][j*C+ci] = W[co][ci][(tap-1)s + j + s/2]."""

    def __init__(self, spec: "DacSpec", state_dict: dict, device="cuda"):
        _lib.load()
        self.spec = spec
        self.device = dev = torch.device(device)
        sd = _fold_weight_norm(state_dict)
        P = HipDacDecoder._pad32
        stream = _lib.stream_ptr(dev)

        def t(k):
            return sd[k].to(device=dev, dtype=torch.float32).contiguous()

        def w16(w):                          # fp32 [Cout][Cin][ks] (padded) -> fp16 [ks][Cout][Cin]
            co, ci, ks = w.shape
            out = torch.empty(ks * co * ci, dtype=torch.int16, device=dev)
            call("zk_dac_prep_w16", ptr(w.contiguous()), co, ci, ks, 1, 0, ptr(out), None, stream)
            return out

        def wconv(w):
            co, ci, ks = w.shape
            wp = torch.zeros(P(co), P(ci), ks, device=dev)
            wp[:co, :ci] = w
            return w16(wp)

        def wstrided(w, st):                 # [Cout][Cin][2s] -> folded 3-tap [Cout_p][s*Cin_p][3]
            co, ci, k2 = w.shape
            assert k2 == 2 * st and st % 2 == 0, "strided encoder conv: k = 2*stride, even stride"
            cip = P(ci)
            wf = torch.zeros(P(co), st, cip, 3, device=dev)
            for tap in range(3):
                for j in range(st):
                    k = (tap - 1) * st + j + st // 2
                    if 0 <= k < k2:
                        wf[:co, j, :ci, tap] = w[:, :, k]
            return w16(wf.reshape(P(co), st * cip, 3))

        def vec(v, fill):
            out = torch.full((P(v.numel()),), fill, device=dev)
            out[:v.numel()] = v.reshape(-1)
            return out

        w1 = t("encoder.conv1.weight")
        self.c0 = w1.shape[0]
        self.conv1_w, self.conv1_b = w1.reshape(self.c0, 7), t("encoder.conv1.bias")
        self.blocks = []
        i = 0
        while f"encoder.block.{i}.conv1.weight" in sd:
            p = f"encoder.block.{i}."
            wb = t(p + "conv1.weight")
            st = wb.shape[2] // 2
            blk = {"stride": st, "cin": P(wb.shape[1]), "cout": P(wb.shape[0]), "alpha": vec(t(p + "snake1.alpha"), 1.0),
                   "w": wstrided(wb, st), "b": vec(t(p + "conv1.bias"), 0.0), "res": []}
            for r, dil in ((1, 1), (2, 3), (3, 9)):
                u = p + f"res_unit{r}."
                blk["res"].append({"dil": dil, "a1": vec(t(u + "snake1.alpha"), 1.0), "w1": wconv(t(u + "conv1.weight")),
                                   "b1": vec(t(u + "conv1.bias"), 0.0), "a2": vec(t(u + "snake2.alpha"), 1.0),
                                   "w2": wconv(t(u + "conv2.weight")), "b2": vec(t(u + "conv2.bias"), 0.0)})
            self.blocks.append(blk)
            i += 1
        self.final_alpha = vec(t("encoder.snake1.alpha"), 1.0)
        w2 = t("encoder.conv2.weight")
        self.hidden = w2.shape[0]
        self.conv2_w, self.conv2_b = wconv(w2), vec(t("encoder.conv2.bias"), 0.0)
        self.cd = spec.codebook_dim
        K = spec.n_codebooks
        q = "quantizer.quantizers.{}."
        self.in_w = torch.stack([t(q.format(k) + "in_proj.weight").reshape(self.cd, self.hidden) for k in range(K)])
        self.in_b = torch.stack([t(q.format(k) + "in_proj.bias") for k in range(K)])
        self.cb = torch.stack([t(q.format(k) + "codebook.weight") for k in range(K)])
        self.cbn = torch.nn.functional.normalize(self.cb, dim=2).contiguous()   # one-time weight prep
        self.cbn2 = self.cbn.pow(2).sum(2).contiguous()
        self.out_w = torch.stack([t(q.format(k) + "out_proj.weight").reshape(self.hidden, self.cd) for k in range(K)])
        self.out_b = torch.stack([t(q.format(k) + "out_proj.bias") for k in range(K)])
        self.hop = int(math.prod(b["stride"] for b in self.blocks))
        torch.cuda.synchronize(dev)

    def latents(self, wav: torch.Tensor) -> torch.Tensor:
        """DacEncoder.forward: wav [B, 1, T] (T a multiple of the hop) -> z fp32 [B, T/hop, hidden]."""
        assert wav.dim() == 3 and wav.shape[1] == 1, "expected [B, 1, T]"
        B, _, T = wav.shape
        assert T % self.hop == 0, f"T={T} must be a multiple of the hop {self.hop} (see preprocess)"
        dev, P, f16 = self.device, HipDacDecoder._pad32, torch.int16
        stream = _lib.stream_ptr(dev)
        wav = wav.to(dev, torch.float32).contiguous()
        C = P(self.c0)
        first_alpha = self.blocks[0]["res"][0]["a1"] if self.blocks else self.final_alpha
        x = torch.empty(B, T, C, device=dev)
        act = torch.empty(B, T, C, dtype=f16, device=dev)
        call("zk_dac_enc_conv1", ptr(wav), B, T, ptr(self.conv1_w), ptr(self.conv1_b), ptr(first_alpha), self.c0, C,
             ptr(x), ptr(act), stream)
        L = T
        for bi, blk in enumerate(self.blocks):
            C = blk["cin"]
            tmp = torch.empty_like(act)
            for j, ru in enumerate(blk["res"]):
                d = ru["dil"]
                a_next = blk["res"][j + 1]["a1"] if j + 1 < len(blk["res"]) else blk["alpha"]
                call("zk_dac_conv_cl", ptr(act), B, C, L, ptr(ru["w1"]), 0, ptr(ru["b1"]), C, 7, d, 3 * d, L,
                     1, 1, 0, L, None, None, ptr(ru["a2"]), ptr(tmp), 0, None, 1, 1, stream)
                call("zk_dac_conv_cl", ptr(tmp), B, C, L, ptr(ru["w2"]), 0, ptr(ru["b2"]), C, 1, 1, 0, L,
                     1, 1, 0, L, ptr(x), ptr(x), ptr(a_next), ptr(act), 0, None, 1, 1, stream)
            del tmp
            st, Co = blk["stride"], blk["cout"]
            Lo = L // st
            a_next = self.blocks[bi + 1]["res"][0]["a1"] if bi + 1 < len(self.blocks) else self.final_alpha
            x = torch.empty(B, Lo, Co, device=dev)
            s_new = torch.empty(B, Lo, Co, dtype=f16, device=dev)
            call("zk_dac_conv_cl", ptr(act), B, st * C, Lo, ptr(blk["w"]), 0, ptr(blk["b"]), Co, 3, 1, 1, Lo,
                 1, 1, 0, Lo, None, ptr(x), ptr(a_next), ptr(s_new), 0, None, 1, 1, stream)
            act, L = s_new, Lo
        Hp = P(self.hidden)
        z = torch.empty(B, L, Hp, device=dev)
        call("zk_dac_conv_cl", ptr(act), B, act.shape[2], L, ptr(self.conv2_w), 0, ptr(self.conv2_b), Hp, 3, 1, 1, L,
             1, 1, 0, L, None, ptr(z), None, None, 0, None, 1, 1, stream)
        return z[:, :, :self.hidden] if Hp != self.hidden else z

    def quantize(self, z: torch.Tensor) -> torch.Tensor:
        """DacResidualVectorQuantizer (eval, all codebooks): z fp32 [B, T, hidden] -> int64 [B, K, T]."""
        z = z.contiguous()
        B, T, H = z.shape
        K = self.in_w.shape[0]
        codes = torch.empty(B, K, T, dtype=torch.int64, device=self.device)
        call("zk_dac_rvq_encode", ptr(z), B, T, H, K, self.cb.shape[1], self.cd, ptr(self.in_w), ptr(self.in_b),
             ptr(self.cbn), ptr(self.cbn2), ptr(self.cb), ptr(self.out_w), ptr(self.out_b), ptr(codes),
             _lib.stream_ptr(self.device))
        return codes

    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        return self.quantize(self.latents(wav))


class DACAutoencoder:
    """API mirror of zonos/autoencoder.py:12-268 (prefix encode + decode + post-processing).

    Weights: ``DACAutoencoder(state_dict=...)``, ``DACAutoencoder.from_local(dir_or_file)``
    (a HF-format DacModel safetensors), or the local HF cache of "descript/dac_44khz"
    (autoencoder.py:15 fetches it by name; offline only the cache is consulted)."""

    def __init__(self, state_dict: dict | None = None, spec: DacSpec | None = None, device="cuda"):
        self.spec = spec or DacSpec()
        if state_dict is None:
            state_dict, cfg = _load_hf_cache("descript/dac_44khz")
            if cfg is not None:
                self.spec = DacSpec.from_hf_config(cfg)
        self.decoder = HipDacDecoder(self.spec, state_dict, device)
        self._encoder = None
        self._state_dict = state_dict if any(k.startswith("encoder.") for k in state_dict) else None
        self.codebook_size = self.spec.codebook_size
        self.num_codebooks = self.spec.n_codebooks
        self.sampling_rate = self.spec.sampling_rate

    @classmethod
    def from_local(cls, path: str, device="cuda") -> "DACAutoencoder":
        sd, cfg = _load_safetensors_dir(path)
        return cls(sd, DacSpec.from_hf_config(cfg) if cfg else None, device)

    # ---- prefix-audio side (autoencoder.py:21-42)
    @property
    def encoder(self) -> HipDacEncoder:
        if self._encoder is None:
            if self._state_dict is None:
                raise ValueError("the DAC state dict has no encoder.* weights; encode() needs the full DacModel")
            self._encoder = HipDacEncoder(self.spec, self._state_dict, self.decoder.device)
            self._state_dict = None
        return self._encoder

    def preprocess(self, wav: torch.Tensor, sr: int) -> torch.Tensor:
        """autoencoder.py:21-25: resample to 44.1 kHz (windowed-sinc, on the GPU), left-pad to a
        multiple of 512 samples."""
        from . import audio
        wav = audio.resample(wav.to(self.decoder.device, torch.float32), sr, self.sampling_rate)
        return audio.left_pad(wav, 512)

    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """autoencoder.py:27-28 (DacModel.encode(wav).audio_codes): [B, 1, T] -> int64 [B, 9, T/512]."""
        return self.encoder.encode(wav)

    def load_prefix_audio(self, audio_path: str, device=None) -> torch.Tensor:
        """autoencoder.py:30-42: read, average channels to mono, preprocess, encode -> [1, 9, T]."""
        from . import audio
        wav, sr = audio.read_wav(audio_path)
        wav = wav.mean(dim=0, keepdim=True)
        wav = self.preprocess(wav, sr)
        codes = self.encode(wav.unsqueeze(0))
        return codes if device is None else codes.to(device)

    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        """autoencoder.py:44-47: [B, 9, T] -> fp32 [B, 1, 512*T] (all rows full length)."""
        assert codes.shape[1] == self.num_codebooks, \
            f"Expected {self.num_codebooks} codebooks, got {codes.shape[1]}"
        return self.decoder.decode_padded(codes)

    def decode_list(self, codes) -> list:
        return self.decoder.decode_list(codes)

    # ---- post-processing of codes_to_wavs (autoencoder.py:49-90, 172-245)
    @staticmethod
    def trim_silence(wav: torch.Tensor, threshold: float = 1e-5, frame_size: int = 512) -> torch.Tensor:
        """autoencoder.py:49-90 as written: the tail loop's first frame is wav[:, -512:-0] (empty,
        its mean is nan and never above the threshold), a found tail frame cuts at -(i+1)*512."""
        assert wav.ndim == 2 and wav.shape[0] == 1, "Expected mono audio tensor"
        n = min((wav.shape[1] // frame_size) // 4, 16)
        start, end = 0, wav.shape[1]
        for i in range(n):
            if wav[:, i * frame_size:(i + 1) * frame_size].pow(2).mean() > threshold:
                start = i * frame_size
                break
        for i in range(n):
            if wav[:, -((i + 1) * frame_size): -i * frame_size].pow(2).mean() > threshold:
                end = -((i + 1) * frame_size)
                break
        return wav[:, start:end] if (start > 0 or end < wav.shape[1]) else wav

    def loudness_gains(self, wavs: list, target_lufs: float = -23.0) -> list:
        """Per-utterance gains of normalize_loudness (pyloudnorm BS.1770 integrated loudness),
        measured for the whole list in one batched GPU pass (zk_loudness_gains)."""
        wavs = [w for w in wavs]
        if not wavs:
            return []
        dev = self.decoder.device
        T = max(int(w.shape[-1]) for w in wavs)
        T = (T + 3) // 4 * 4
        B = len(wavs)
        batch = torch.zeros(B, T, device=dev)
        for i, w in enumerate(wavs):
            batch[i, :w.shape[-1]] = w.reshape(-1).to(dev, torch.float32)
        lens = torch.tensor([int(w.shape[-1]) for w in wavs], dtype=torch.int32, device=dev)
        nb = _lib.load().zk_loudness_max_blocks(T, int(self.sampling_rate))
        scratch = torch.empty(B * T + B * max(nb, 1), dtype=torch.float64, device=dev)
        gains = torch.empty(B, dtype=torch.float64, device=dev)
        loud = torch.empty(B, dtype=torch.float64, device=dev)
        call("zk_loudness_gains", ptr(batch), B, T, ptr(lens), int(self.sampling_rate), float(target_lufs),
             ptr(scratch), ptr(gains), ptr(loud), _lib.stream_ptr(dev))
        return gains.cpu().tolist()

    def normalize_loudness(self, audio, sr, target_lufs=-19.0):
        """autoencoder.py:172-186: audio * 10^((target - loudness)/20); unchanged if too short."""
        assert sr == self.sampling_rate
        return audio * self.loudness_gains([audio], target_lufs)[0]

    def codes_to_wavs(self, codes) -> list:
        """autoencoder.py:188-245: decode (one batched, length-masked GPU pass instead of one
        decode per utterance), loudness to -23 LUFS (batched GPU measurement), silence trim,
        512-sample linear fade-in, log fade-out over up to 20 blocks. Returns CPU [1, n] fp32."""
        if isinstance(codes, list):
            code_list = [c if c.dim() == 3 else c.unsqueeze(0) for c in codes]
            items = [c[i] for c in code_list for i in range(c.shape[0])]
        elif codes.dim() == 2:
            items = [codes]
        elif codes.dim() == 3:
            items = [codes[i] for i in range(codes.shape[0])]
        else:
            raise ValueError(f"Invalid shape for codes: {codes.shape}. Expected [num_codebooks, num_codes] or "
                             f"[batch_size, num_codebooks, num_codes]")
        wavs = self.decode_list(items)                     # empty utterances skipped (autoencoder.py:221-223)
        gains = self.loudness_gains(wavs, -23.0)
        out = []
        for wav, g in zip(wavs, gains):
            wav = wav.cpu() * g
            wav = self.trim_silence(wav)
            blocksize = 512
            wav[:, :blocksize] *= torch.linspace(0, 1, blocksize, device=wav.device).unsqueeze(0)
            nb = min((wav.shape[1] // blocksize) // 4, 20)
            if nb > 0:
                wav[:, -(nb * blocksize):] *= torch.logspace(0, -10, nb * blocksize, device=wav.device).unsqueeze(0)
            out.append(wav)
        return out

    def save_codes(self, paths, codes) -> None:
        """autoencoder.py:247-268: codes_to_wavs + one file per waveform. torchaudio.save of a
        float32 tensor writes a 32-bit IEEE-float WAV; the same format is written here
        (torchaudio is not a dependency of this package)."""
        if isinstance(paths, str):
            paths = [paths]
        wavs = self.codes_to_wavs(codes)
        assert len(paths) == len(wavs), f"Number of paths ({len(paths)}) must match number of codes ({len(wavs)})"
        for p, w in zip(paths, wavs):
            write_wav_f32(p, w, self.sampling_rate)


def write_wav_f32(path: str, wav: torch.Tensor, sr: int) -> None:
    """RIFF/WAVE, WAVE_FORMAT_IEEE_FLOAT (3), 32 bit, channels = wav.shape[0] (interleaved)."""
    import struct

    x = wav.detach().to("cpu", torch.float32)
    x = x.unsqueeze(0) if x.dim() == 1 else x
    ch, n = x.shape
    data = x.t().contiguous().numpy().tobytes()
    fmt = struct.pack("<HHIIHH", 3, ch, sr, sr * ch * 4, ch * 4, 32)
    fact = struct.pack("<I", n)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + (8 + len(fmt)) + (8 + len(fact)) + (8 + len(data))) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt)
        f.write(b"fact" + struct.pack("<I", len(fact)) + fact)
        f.write(b"data" + struct.pack("<I", len(data)) + data)


def _load_safetensors_dir(path: str):
    import json

    from safetensors.torch import load_file
    cfg = None
    if os.path.isdir(path):
        cj = os.path.join(path, "config.json")
        if os.path.exists(cj):
            cfg = json.load(open(cj))
        files = [os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors")]
    else:
        files = [path]
    sd = {}
    for f in files:
        sd.update(load_file(f))
    return sd, cfg


def _load_hf_cache(repo_id: str):
    """The DAC weights the reference fetches by name (autoencoder.py:15): $ZONOS_DAC_PATH (a local
    HF-format directory or .safetensors file) if set, else the local Hugging Face cache."""
    local = os.environ.get("ZONOS_DAC_PATH")
    if local:
        return _load_safetensors_dir(local)
    from huggingface_hub import snapshot_download
    try:
        d = snapshot_download(repo_id, local_files_only=True)
    except Exception as e:   # no network in this environment
        raise FileNotFoundError(
            f"{repo_id} is not in the local Hugging Face cache; pass state_dict= or use "
            f"DACAutoencoder.from_local(path)") from e
    return _load_safetensors_dir(d)
