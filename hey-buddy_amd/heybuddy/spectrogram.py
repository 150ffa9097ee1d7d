"""Drop-in for heybuddy.spectrogram (reference src/python/heybuddy/spectrogram.py).

``MelSpectrogramModel.__call__`` keeps the reference contract (numpy
[b, t] int16-range audio in, numpy [b, frames, 32] log-mel out, already
``/10 + 2``-scaled, squeezed) but runs the fused STFT + mel HIP kernel
(hbk_mel_frames) instead of an ONNX Runtime session. The mel parameters are
runtime data (window, filterbank); the defaults are hypothesis H0 of
SURVEY.md §8a-3 (torchaudio MelSpectrogram, n_fft 512, win 400, hop 160,
60-3800 Hz, 32 HTK mels, 10 log10(max(P, 1e-10))).
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from heybuddy import _native
from heybuddy.kernels import MelPlan

__all__ = ["MelSpectrogramModel", "get_mel_spectrogram_model", "mel_parameters",
           "default_mel_plan"]

SAMPLE_RATE = 16000
N_FFT = 512
WIN_LENGTH = 400
HOP = 160
F_MIN = 60.0
F_MAX = 3800.0
N_MELS = 32


def _hann_window(win_length: int = WIN_LENGTH, n_fft: int = N_FFT) -> np.ndarray:
    n = np.arange(win_length, dtype=np.float64)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / win_length)  # periodic Hann
    out = np.zeros(n_fft, dtype=np.float64)
    left = (n_fft - win_length) // 2                         # torch.stft centring
    out[left:left + win_length] = w
    return out.astype(np.float32)


def _mel_fbank(n_freqs: int = N_FFT // 2 + 1, f_min: float = F_MIN, f_max: float = F_MAX,
               n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE) -> np.ndarray:
    hz2mel = lambda f: 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)  # noqa: E731
    mel2hz = lambda m: 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)  # noqa: E731
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    f_pts = mel2hz(np.linspace(hz2mel(f_min), hz2mel(f_max), n_mels + 2))
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    fb = np.maximum(0.0, np.minimum(-slopes[:, :-2] / f_diff[:-1], slopes[:, 2:] / f_diff[1:]))
    return fb.astype(np.float32)


def mel_parameters() -> Tuple[np.ndarray, np.ndarray]:
    """(window [512], filterbank [257, 32]) of the mel graph (H0)."""
    return _hann_window(), _mel_fbank()


_PLANS: Dict[Tuple[int, float], MelPlan] = {}


def default_mel_plan(device: torch.device, in_scale: float = 32767.0) -> MelPlan:
    """Cached plan per (device, input scale)."""
    key = (device.index, float(in_scale))
    if key not in _PLANS:
        window, fbank = mel_parameters()
        _PLANS[key] = MelPlan(window, fbank, hop=HOP, in_scale=in_scale, log_floor=1e-10,
                              out_div=10.0, out_add=2.0, device=device)
    return _PLANS[key]


class MelSpectrogramModel:
    """Compute the log-mel spectrogram of int16-range audio (spectrogram.py:11-32).

    ``device_id`` picks the HIP device (None = the current one); there is no
    CPU execution provider: without a GPU the call raises HBKUnavailable.
    """

    def __init__(self, device_id: Optional[int] = None, load: bool = False) -> None:
        self.device_id = device_id
        self.loaded = False
        if load:
            self.load()

    @property
    def device(self) -> torch.device:
        return _native.require_device(self.device_id)

    def load(self) -> None:
        default_mel_plan(self.device, 1.0)
        self.loaded = True

    def unload(self) -> None:
        self.loaded = False

    def __call__(self, audio: np.ndarray[Any, Any]) -> np.ndarray[Any, Any]:
        assert isinstance(audio, np.ndarray)
        if audio.ndim == 1:
            audio = audio[np.newaxis, :]
        assert audio.ndim == 2, f"Audio must be a 1D or 2D array, got {audio.ndim}D"
        dev = self.device
        plan = default_mel_plan(dev, 1.0)  # input already in int16 range
        x = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(dev)
        out = plan(x)
        return np.squeeze(out.cpu().numpy())


GLOBAL_MEL_MODELS: Dict[Optional[int], MelSpectrogramModel] = {}


def get_mel_spectrogram_model(device_id: Optional[int] = None) -> MelSpectrogramModel:
    if device_id not in GLOBAL_MEL_MODELS:
        GLOBAL_MEL_MODELS[device_id] = MelSpectrogramModel(device_id=device_id, load=True)
    return GLOBAL_MEL_MODELS[device_id]
