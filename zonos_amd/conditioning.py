"""Prefix conditioning (zonos/conditioning.py): ``make_cond_dict``, phoneme tokenisation and
``PrefixConditioner`` whose forward pass is ONE HIP launch (csrc/cond.hip, zk_prefix_cond).

The eSpeak front end (number/Japanese normalisation, ``phonemize``) stays on the CPU and is not
part of this engine: the ``phonemizer``/espeak-ng stack is absent here. ``phonemize`` uses a
callable installed with ``set_phonemizer(fn)`` (``fn(texts, languages) -> list[str]`` of IPA
strings), or the ``phonemizer`` package's EspeakBackend when it is importable.

Config and weights follow the reference: ``PrefixConditionerConfig.conditioners`` is the list
of dicts from config.json, the state-dict keys are the module's (``conditioners.{i}.*``,
``project.*``, ``norm.*`` under ``prefix_conditioner.``).
"""
from __future__ import annotations

import ctypes as C  # noqa: N812
import warnings
from typing import Iterable, Union

import torch

from . import _lib
from ._lib import call

# ---------------------------------------------------------------- phoneme vocabulary (conditioning.py:140-191)
PAD_ID, UNK_ID, BOS_ID, EOS_ID = 0, 1, 2, 3
SPECIAL_TOKEN_IDS = [PAD_ID, UNK_ID, BOS_ID, EOS_ID]
_PUNCT = ';:,.!?¡¿—…"«»“”() *~-/\\&'
_LETTERS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
_IPA = ("ɑɐɒæɓʙβɔɕçɗɖðʤəɘɚɛɜɝɞɟʄɡɠɢʛɦɧħɥʜɨɪʝɭɬɫɮʟɱɯɰŋɳɲɴøɵɸθœɶʘɹɺɾɻʀʁɽʂʃʈʧʉʊʋⱱʌɣɤʍχʎʏʑʐʒʔʡʕʢǀǁǂǃˈˌːˑʼʴʰʱʲʷˠˤ˞↓↑→↗↘"
        "'̩'ᵻ")
symbols = [*_PUNCT, *_LETTERS, *_IPA]
# a symbol listed twice maps to its last position, as the reference's dict comprehension does
_symbol_to_id = {sym: i for i, sym in enumerate(symbols, start=len(SPECIAL_TOKEN_IDS))}
N_PHONEME_IDS = len(SPECIAL_TOKEN_IDS) + len(symbols)


def get_symbol_ids(text: str) -> list[int]:
    ids = []
    for ch in text:
        i = _symbol_to_id.get(ch)
        if i is None:
            warnings.warn(f"Character ' {ch} ' not recognized; using UNK_ID.", stacklevel=2)
            i = UNK_ID
        ids.append(i)
    return ids


def tokenize_phonemes(phonemes: list[str]) -> tuple[torch.Tensor, list[int]]:
    """[BOS, ids..., EOS] per string, LEFT-padded with PAD to the longest (conditioning.py:186-191)."""
    seqs = [[BOS_ID, *get_symbol_ids(p), EOS_ID] for p in phonemes]
    lengths = [len(s) for s in seqs]
    longest = max(lengths)
    return torch.tensor([[PAD_ID] * (longest - len(s)) + s for s in seqs]), lengths


_phonemizer = None


def set_phonemizer(fn) -> None:
    """Install the text -> IPA front end: ``fn(texts, languages) -> list[str]``."""
    global _phonemizer
    _phonemizer = fn


def phonemize(texts: list[str], languages: list[str]) -> list[str]:
    if _phonemizer is not None:
        return list(_phonemizer(texts, languages))
    try:
        from phonemizer.backend import EspeakBackend
    except ImportError as e:
        raise RuntimeError("no phonemizer: install phonemizer + espeak-ng, or call "
                           "zonos_amd.conditioning.set_phonemizer(fn)") from e
    out = []
    for text, lang in zip(texts, languages):
        be = EspeakBackend(lang, preserve_punctuation=True, with_stress=True, punctuation_marks=_PUNCT)
        out.append(be.phonemize([text], strip=True)[0])
    return out


# ---------------------------------------------------------------- make_cond_dict (conditioning.py:406-495)
supported_language_codes = [
    'af', 'am', 'an', 'ar', 'as', 'az', 'ba', 'bg', 'bn', 'bpy', 'bs', 'ca', 'cmn', 'cs', 'cy', 'da', 'de', 'el',
    'en-029', 'en-gb', 'en-gb-scotland', 'en-gb-x-gbclan', 'en-gb-x-gbcwmd', 'en-gb-x-rp', 'en-us', 'eo', 'es',
    'es-419', 'et', 'eu', 'fa', 'fa-latn', 'fi', 'fr-be', 'fr-ch', 'fr-fr', 'ga', 'gd', 'gn', 'grc', 'gu', 'hak',
    'hi', 'hr', 'ht', 'hu', 'hy', 'hyw', 'ia', 'id', 'is', 'it', 'ja', 'jbo', 'ka', 'kk', 'kl', 'kn', 'ko', 'kok',
    'ku', 'ky', 'la', 'lfn', 'lt', 'lv', 'mi', 'mk', 'ml', 'mr', 'ms', 'mt', 'my', 'nb', 'nci', 'ne', 'nl', 'om',
    'or', 'pa', 'pap', 'pl', 'pt', 'pt-br', 'py', 'quc', 'ro', 'ru', 'ru-lv', 'sd', 'shn', 'si', 'sk', 'sl', 'sq',
    'sr', 'sv', 'sw', 'ta', 'te', 'tn', 'tr', 'tt', 'ur', 'uz', 'vi', 'vi-vn-x-central', 'vi-vn-x-south', 'yue',
]


def make_cond_dict(text: Union[str, list[str]] = "Zonos uses eSpeak for text to phoneme conversion!",
                   language: str = "en-us", speaker: torch.Tensor | None = None,
                   emotion: list[float] = [1.0, 0.05, 0.05, 0.05, 0.05, 0.05, 0.1, 0.2], fmax: float = 22050.0,
                   pitch_std: float = 20.0, speaking_rate: float = 15.0, vqscore_8: list[float] = [0.78] * 8,
                   ctc_loss: float = 0.0, dnsmos_ovrl: float = 4.0, speaker_noised: bool = False,
                   unconditional_keys: Iterable[str] = {"emotion", "vqscore_8", "dnsmos_ovrl"},
                   device=None) -> dict:
    """Same keys, defaults and tensor shapes ([1, 1, n]) as the reference; emotion normalised to sum 1."""
    from .utils import DEFAULT_DEVICE
    device = DEFAULT_DEVICE if device is None else device
    texts = [text] if isinstance(text, str) else list(text)
    language = language.lower().replace("_", "-")
    assert language in supported_language_codes, \
        f"Language code {language} isn't supported. Please pick a supported language code from the list: " \
        f"{supported_language_codes}"
    cond = {"espeak": (texts, [language] * len(texts)), "speaker": speaker, "emotion": emotion, "fmax": fmax,
            "pitch_std": pitch_std, "speaking_rate": speaking_rate,
            "language_id": supported_language_codes.index(language), "vqscore_8": vqscore_8,
            "ctc_loss": ctc_loss, "dnsmos_ovrl": dnsmos_ovrl, "speaker_noised": int(speaker_noised)}
    for k in unconditional_keys:
        cond.pop(k, None)
    for k, v in list(cond.items()):
        if isinstance(v, (float, int, list)):
            v = torch.tensor(v)
        if isinstance(v, torch.Tensor):
            cond[k] = v.view(1, 1, -1).to(device)
        if k == "emotion":
            cond[k] /= cond[k].sum(dim=-1)
    return cond


# ---------------------------------------------------------------- the C plan (include/zonos_hip.h)
MAXSEG = 16
SEG_VECTOR, SEG_EMBED, SEG_FOURIER, SEG_PASS = 0, 1, 2, 3
_PROJ = {"none": 0, "linear": 1, "mlp": 2}


class ZkCondSeg(C.Structure):
    _fields_ = [("type", C.c_int), ("len", C.c_int), ("cin", C.c_int), ("in_dim", C.c_int), ("bin", C.c_int),
                ("proj", C.c_int), ("in_bstride", C.c_long), ("id_min", C.c_long), ("vmin", C.c_float),
                ("vden", C.c_float), ("table", C.c_void_p), ("input", C.c_void_p), ("pw0", C.c_void_p),
                ("pb0", C.c_void_p), ("pw1", C.c_void_p), ("pb1", C.c_void_p)]


class ZkCondPlan(C.Structure):
    _fields_ = [("nseg", C.c_int), ("D", C.c_int), ("L", C.c_int), ("proj", C.c_int), ("eps", C.c_float),
                ("pw0", C.c_void_p), ("pb0", C.c_void_p), ("pw1", C.c_void_p), ("pb1", C.c_void_p),
                ("norm_w", C.c_void_p), ("norm_b", C.c_void_p), ("seg", ZkCondSeg * MAXSEG)]


class PrefixConditioner:
    """conditioning.py:373-389 on the GPU. ``state_dict`` holds the module's own keys
    (``conditioners.{i}.…``, ``project.…``, ``norm.…``); ``conditioners`` the config dicts."""

    def __init__(self, config, output_dim: int, state_dict: dict, device="cuda"):
        _lib.load()
        self.conditioners = [dict(c) for c in config.conditioners]
        assert len(self.conditioners) <= MAXSEG
        self.projection = config.projection
        self.D = int(output_dim)
        self.device = dev = torch.device(device)
        self.w = {k: v.to(device=dev, dtype=torch.bfloat16).contiguous() for k, v in state_dict.items()}
        for c in self.conditioners:
            if c["type"] == "FourierConditioner":
                assert self.D % 2 == 0
            elif c["type"] not in ("EspeakPhonemeConditioner", "IntegerConditioner", "PassthroughConditioner"):
                raise ValueError(f"unknown conditioner type {c['type']}")
        self.required_keys = {c["name"] for i, c in enumerate(self.conditioners)
                              if f"conditioners.{i}.uncond_vector" not in self.w}

    def _proj_ptrs(self, pre, kind):
        w = self.w
        if kind == "linear":
            return w[pre + "project.weight"].data_ptr(), w[pre + "project.bias"].data_ptr(), None, None
        if kind == "mlp":
            return (w[pre + "project.0.weight"].data_ptr(), w[pre + "project.0.bias"].data_ptr(),
                    w[pre + "project.2.weight"].data_ptr(), w[pre + "project.2.bias"].data_ptr())
        return None, None, None, None

    def _plan(self, cond_dict: dict):
        """Segments for one cond_dict; returns (plan, batch, keep-alive tensors)."""
        if not set(cond_dict).issuperset(self.required_keys):
            raise ValueError(f"Missing required keys: {self.required_keys - set(cond_dict)}")
        dev, D = self.device, self.D
        plan = ZkCondPlan()
        plan.nseg, plan.D, plan.eps = len(self.conditioners), D, 1e-5
        plan.proj = _PROJ[self.projection]
        plan.pw0, plan.pb0, plan.pw1, plan.pb1 = self._proj_ptrs("", self.projection)
        plan.norm_w, plan.norm_b = self.w["norm.weight"].data_ptr(), self.w["norm.bias"].data_ptr()
        keep, batches, L = [], [], 0
        for i, c in enumerate(self.conditioners):
            pre = f"conditioners.{i}."
            g = plan.seg[i]
            value = cond_dict.get(c["name"])
            if value is None:
                assert pre + "uncond_vector" in self.w, f"conditioner {c['name']} has no learned uncond vector"
                g.type, g.len, g.cin, g.bin = SEG_VECTOR, 1, D, 1
                g.table = self.w[pre + "uncond_vector"].data_ptr()
                batches.append(1)
                L += 1
                continue
            proj = c.get("projection", "none")
            g.proj = _PROJ[proj]
            g.pw0, g.pb0, g.pw1, g.pb1 = self._proj_ptrs(pre, proj)
            if c["type"] == "EspeakPhonemeConditioner":
                texts, langs = value
                ids, _ = tokenize_phonemes(phonemize(list(texts), list(langs)))
                ids = ids.to(dev, torch.int64).contiguous()
                assert int(ids.max()) < N_PHONEME_IDS
                keep.append(ids)
                g.type, g.len, g.cin, g.bin, g.in_bstride = SEG_EMBED, ids.shape[1], D, ids.shape[0], ids.shape[1]
                g.table, g.input = self.w[pre + "phoneme_embedder.weight"].data_ptr(), ids.data_ptr()
            else:
                x = value if value.dim() == 3 else value.reshape(1, *value.shape[-2:])
                nb, seq = x.shape[0], x.shape[1]
                if c["type"] == "FourierConditioner":
                    in_dim = c.get("input_dim", 1)
                    assert x.shape[-1] == in_dim
                    x = x.to(dev, torch.float32).contiguous()
                    lo, hi = c.get("min_val", 0.0), c.get("max_val", 1.0)
                    g.type, g.cin, g.in_dim, g.vmin, g.vden = SEG_FOURIER, D, in_dim, float(lo), float(hi - lo)
                    g.table = self.w[pre + "weight"].data_ptr()
                    g.in_bstride = seq * in_dim
                elif c["type"] == "IntegerConditioner":
                    assert x.shape[-1] == 1
                    x = x.reshape(nb, seq).to(dev, torch.int64).contiguous()
                    lo, hi = c.get("min_val", 0), c.get("max_val", 512)
                    if int(x.min()) < lo or int(x.max()) > hi:
                        raise IndexError(f"{c['name']}: value outside [{lo}, {hi}]")
                    g.type, g.cin, g.id_min, g.in_bstride = SEG_EMBED, D, int(lo), seq
                    g.table = self.w[pre + "int_embedder.weight"].data_ptr()
                else:                               # PassthroughConditioner
                    cin = c.get("cond_dim") or D
                    assert x.shape[-1] == cin
                    x = x.to(dev, torch.bfloat16).contiguous()
                    g.type, g.cin, g.in_bstride = SEG_PASS, cin, seq * cin
                keep.append(x)
                g.len, g.bin, g.input = seq, nb, x.data_ptr()
            batches.append(g.bin)
            L += g.len
        B = max(batches)
        assert all(b in (1, B) for b in batches), f"conditioner batch sizes {batches} do not broadcast"
        plan.L = L
        return plan, B, keep

    def __call__(self, cond_dict: dict) -> torch.Tensor:
        return self.forward(cond_dict)

    def forward(self, cond_dict: dict) -> torch.Tensor:
        """[B, L, D] bf16 = LayerNorm(project(cat(conditioner rows)))."""
        plan, B, keep = self._plan(cond_dict)
        out = torch.empty(B, plan.L, self.D, dtype=torch.bfloat16, device=self.device)
        call("zk_prefix_cond", C.addressof(plan), B, out.data_ptr(), _lib.stream_ptr(self.device))
        del keep            # stream-ordered reuse by the caching allocator keeps this safe
        return out

    def prepare_conditioning(self, cond_dict: dict, uncond_dict: dict | None = None) -> torch.Tensor:
        """Zonos.prepare_conditioning (model.py:210-218): cat([cond, uncond]) -> [2B, L, D]."""
        if uncond_dict is None:
            uncond_dict = {k: cond_dict[k] for k in self.required_keys}
        return torch.cat([self.forward(cond_dict), self.forward(uncond_dict)])
