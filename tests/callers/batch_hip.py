"""The generation core of the reference's zonos_batch_cli.py (generate_audio, :106-186: import
lines, make_cond_dict / prepare_conditioning / generate / codes_to_wavs / sampling_rate calls with
the CLI's argument names) against the `zonos` import surface. Prefix audio goes through
model.autoencoder.encode like the CLI's load_audio (:19-56); the waveform is synthetic and
torchaudio (absent) is replaced by this repo's WAV reader/writer. Speaker: precomputed tensor."""
import os

import torch
import torch.nn.functional as F

from zonos.model import Zonos
from zonos.conditioning import make_cond_dict
from zonos.utils import DEFAULT_DEVICE as device

from zonos_amd.audio import read_wav
from zonos_amd.autoencoder import write_wav_f32


class Args:
    text = ["Hello, world!", "Zonos uses eSpeak for text to phoneme conversion!"]
    language = "en-us"
    emotion = [0.3077, 0.0256, 0.0256, 0.0256, 0.0256, 0.0256, 0.2564, 0.3077]
    fmax = 22050.0
    pitch_std = 20.0
    speaking_rate = 15.0
    vqscore_8 = [0.78] * 8
    ctc_loss = 0.0
    dnsmos_ovrl = 4.0
    speaker_noised = False
    unconditional_keys = ["emotion"]
    max_new_tokens = int(os.environ.get("ZONOS_MAX_NEW", 86 * 3))
    cfg_scale = 2.0
    top_p, top_k, min_p = 0.0, 0, 0.0
    linear, conf, quad = 0.65, 0.40, 0.00
    repetition_penalty, repetition_penalty_window, temperature = 2.5, 8, 1.0
    seed = 423
    progress_bar = False
    output = os.environ["ZONOS_OUT"]


def load_audio(file_paths, model):
    wavs = []
    for file_path in file_paths:
        wav, sr = read_wav(file_path)
        if wav.shape[0] == 2:
            wav = wav.mean(0, keepdim=True)
        if sr != 44_100:
            wav = model.autoencoder.preprocess(wav, sr)[0]
        wavs.append(wav)
    max_length = max(-(-w.shape[-1] // 512) * 512 for w in wavs)
    padded = [F.pad(w, (max_length - w.shape[-1], 0), value=0) for w in wavs]
    batch_wav = torch.stack(padded).to(device, dtype=torch.float32)
    return model.autoencoder.encode(batch_wav)


args = Args()
model = Zonos.from_pretrained(os.environ["ZONOS_CKPT"], device=device)
speaker_embedding = torch.load(os.environ["ZONOS_SPEAKER"], weights_only=True)
prefix_audio_codes = load_audio([os.environ["ZONOS_PREFIX_WAV"]] * len(args.text), model)

torch.manual_seed(args.seed)
cond_dict = make_cond_dict(
    text=args.text,
    speaker=speaker_embedding,
    language=args.language,
    emotion=args.emotion,
    fmax=args.fmax,
    pitch_std=args.pitch_std,
    speaking_rate=args.speaking_rate,
    vqscore_8=args.vqscore_8,
    ctc_loss=args.ctc_loss,
    dnsmos_ovrl=args.dnsmos_ovrl,
    speaker_noised=args.speaker_noised,
    unconditional_keys=args.unconditional_keys,
)
prefix_conditioning = model.prepare_conditioning(cond_dict)
codes = model.generate(
    prefix_conditioning,
    audio_prefix_codes=prefix_audio_codes,
    max_new_tokens=args.max_new_tokens,
    cfg_scale=args.cfg_scale,
    batch_size=len(args.text),
    disable_torch_compile=True,
    sampling_params={
        "top_p": args.top_p,
        "top_k": args.top_k,
        "min_p": args.min_p,
        "linear": args.linear,
        "conf": args.conf,
        "quad": args.quad,
        "repetition_penalty": args.repetition_penalty,
        "repetition_penalty_window": args.repetition_penalty_window,
        "temperature": args.temperature,
    },
    progress_bar=args.progress_bar,
)
written = []
for i, code in enumerate(codes):
    output_file = f"{args.output.rstrip('.wav')}_{i}.wav"
    wavs = model.autoencoder.codes_to_wavs(code)
    if len(wavs) == 0:
        continue
    wav = wavs[0]
    sr = model.autoencoder.sampling_rate
    write_wav_f32(output_file, wav, sr)
    written.append(output_file)
RESULT = dict(codes=codes, prefix_audio_codes=prefix_audio_codes, written=written)
