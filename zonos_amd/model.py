"""Zonos model API mirror (zonos/model.py:22-457) backed by the HIP engine.

Kept from the reference: ``Zonos.from_pretrained`` / ``from_local`` / ``generate`` /
``autoencoder`` / ``embed_codes`` semantics and the same safetensors key names
(backbone.layers.{i}.{norm,mixer.in_proj,mixer.out_proj,norm2,mlp.fc1,mlp.fc2},
backbone.norm_f, embeddings.{k}, heads.{k}). The text/speaker front end
``prepare_conditioning`` runs the PrefixConditioner as one HIP launch (zonos_amd/conditioning.py);
the eSpeak phonemizer and the speaker-embedding network (make_speaker_embedding) are outside this
engine's scope.
"""
from __future__ import annotations

import json
from typing import Callable

import torch

from .autoencoder import DACAutoencoder
from .config import ZonosConfig
from .engine import EngineConfig, HipDecoder
from .utils import DEFAULT_DEVICE, hub_download


def is_hybrid(bc) -> bool:
    """A backbone with SSM layers (ssm_cfg set and some layer not in attn_layer_idx)."""
    return bool(bc.ssm_cfg) and len(set(bc.attn_layer_idx or [])) < bc.n_layer


class Zonos:
    def __init__(self, config: ZonosConfig, state_dict: dict, device=DEFAULT_DEVICE,
                 autoencoder: DACAutoencoder | None = None):
        self.config = config
        self.eos_token_id = config.eos_token_id
        self.masked_token_id = config.masked_token_id
        self.device = torch.device(device)
        bc = config.backbone
        if is_hybrid(bc):
            # Zonos-v0.1-hybrid: mamba_ssm backbone (zonos/backbone/_mamba_ssm.py)
            from .hybrid import HybridDecoder, HybridEngineConfig
            self.engine = HybridDecoder(HybridEngineConfig.from_backbone_config(bc), state_dict, self.device)
        else:
            self.engine = HipDecoder(EngineConfig.from_backbone_config(bc), state_dict, self.device)
        self._autoencoder = autoencoder
        pc = {k[len("prefix_conditioner."):]: v for k, v in state_dict.items() if k.startswith("prefix_conditioner.")}
        self.prefix_conditioner = None
        if pc:
            from .conditioning import PrefixConditioner
            self.prefix_conditioner = PrefixConditioner(config.prefix_conditioner, bc.d_model, pc, self.device)

    @property
    def autoencoder(self) -> DACAutoencoder:
        if self._autoencoder is None:
            self._autoencoder = DACAutoencoder(device=self.device)
        return self._autoencoder

    @autoencoder.setter
    def autoencoder(self, ae):
        self._autoencoder = ae

    @classmethod
    def from_pretrained(cls, repo_id: str, revision: str | None = None, device=DEFAULT_DEVICE, **kwargs) -> "Zonos":
        config_path = hub_download(repo_id=repo_id, filename="config.json", revision=revision)
        model_path = hub_download(repo_id=repo_id, filename="model.safetensors", revision=revision)
        return cls.from_local(config_path, model_path, device, **kwargs)

    @classmethod
    def from_local(cls, config_path: str, model_path: str, device=DEFAULT_DEVICE, backbone: str | None = None,
                   autoencoder: DACAutoencoder | None = None) -> "Zonos":
        """model.py:65-88. ``backbone`` names a class of the registry (zonos_amd.backbone.BACKBONES,
        the reference's keys included) and is **validated only**: an unknown name raises KeyError, and a
        class whose ``supported_architectures`` lacks the checkpoint's architecture raises ValueError
        (the reference's torch backbone asserts on a hybrid config, _torch.py:56). The model is then
        built on the engine of the checkpoint's architecture whatever the name -- ``HipDecoder`` for a
        transformer, ``HybridDecoder`` for a hybrid -- because every registered plugin runs exactly those
        kernels for that architecture (``HipHybridBackbone`` on a transformer config runs the transformer
        blocks, zonos_amd/backbone.py), so generate() does not depend on the selection. The name is kept
        in ``model.backbone_name``. (One deviation: the reference's mamba_ssm backbone, selected
        explicitly for a transformer checkpoint, would build mamba_ssm MHA blocks; here the transformer
        blocks run, as with the reference's default choice for a transformer config, model.py:70-75.)"""
        from safetensors import safe_open

        from .backbone import BACKBONES
        config = ZonosConfig.from_dict(json.load(open(config_path)))
        if backbone:
            bcls = BACKBONES[backbone]
            arch = "hybrid" if is_hybrid(config.backbone) else "transformer"
            if arch not in bcls.supported_architectures:
                raise ValueError(f"backbone {backbone!r} ({bcls.__name__}) does not support the {arch} "
                                 f"architecture (supported: {bcls.supported_architectures})")
        sd = {}
        with safe_open(model_path, framework="pt") as f:
            for k in f.keys():
                if k.startswith(("backbone.", "embeddings.", "heads.", "prefix_conditioner.")):
                    sd[k] = f.get_tensor(k)
        model = cls(config, sd, device, autoencoder)
        if backbone:
            model.backbone_name = backbone
        return model

    def prepare_conditioning(self, cond_dict: dict, uncond_dict: dict | None = None) -> torch.Tensor:
        """model.py:210-218: [2B, L, d_model] bf16 = cat(PrefixConditioner(cond), PrefixConditioner(uncond))."""
        if self.prefix_conditioner is None:
            raise ValueError("this model was loaded without prefix_conditioner.* weights")
        return self.prefix_conditioner.prepare_conditioning(cond_dict, uncond_dict)

    def make_speaker_embedding(self, wav, sr):
        raise NotImplementedError("speaker embedding (zonos/speaker_cloning.py) is outside the HIP engine's scope")

    @torch.inference_mode()
    def generate(self, prefix_conditioning: torch.Tensor, audio_prefix_codes: torch.Tensor | None = None,
                 max_new_tokens: int = 86 * 30, cfg_scale: float = 2.0, batch_size: int = 1,
                 sampling_params: dict = dict(top_p=0, top_k=0, min_p=0, linear=0.55, conf=0.4, quad=0.0,
                                              repetition_penalty=3.0, repetition_penalty_window=2, temperature=1.0),
                 progress_bar: bool = True, disable_torch_compile: bool = False,
                 callback: Callable[[torch.Tensor, int, int], bool] | None = None, *, seed: int | None = None,
                 row_base: int = 0, force_full_length: bool = False, pad_rows: int = 0):
        """model.py:224-457. ``disable_torch_compile`` is accepted and ignored (the step is a
        captured hipGraph). Sampling noise: by default (``seed`` None) the reference's own -- every
        sampler call takes the values `torch.empty_like(probs).exponential_(1)` would draw from torch's
        CUDA generator (sampling.py:26-28) and advances that generator as the reference does, so
        ``torch.manual_seed(s)`` (sample.py:19) gives the reference's noise on the same GPU. An
        integer ``seed`` selects the engine's keyed stream instead (independent of batch sharding).

        ``row_base`` (the global index of this batch's first utterance, for sharded batches) keys the
        keyed stream only, so it needs an explicit ``seed``: with ``seed=None`` and ``row_base != 0``
        this raises ValueError. (Before round 5 ``seed=None`` drew a keyed-stream seed from torch and
        accepted any ``row_base``; ``generate_sharded`` always passes a seed and is unaffected.)
        ``pad_rows``: trailing padding utterances kept out of the EOS protocol (HipDecoder.generate)."""
        noise = "torch" if seed is None else "keyed"
        if noise == "torch" and row_base:
            raise ValueError("row_base needs an explicit seed (the keyed noise stream)")
        prog = None
        if progress_bar:
            try:
                from tqdm import tqdm
                Ld = (0 if audio_prefix_codes is None else audio_prefix_codes.shape[2]) + max_new_tokens + 9
                prog = tqdm(total=Ld - 1 - (0 if audio_prefix_codes is None else audio_prefix_codes.shape[2]),
                            desc="Generating")
            except ImportError:
                prog = None
        out = self.engine.generate(prefix_conditioning.to(self.device), audio_prefix_codes, max_new_tokens,
                                   cfg_scale, batch_size, sampling_params, seed=seed or 0, row_base=row_base,
                                   force_full_length=force_full_length, callback=callback, progress=prog,
                                   noise=noise, pad_rows=pad_rows)
        if prog is not None:
            prog.close()
        return out
