"""Input normalisation of the featurizer.

Mirrors ``audio_to_bct_tensor`` (reference util/audio_util.py:73-145) for the
in-memory inputs the hot path receives (lists, numpy arrays, torch tensors);
file / URI / bytes decoding is outside this build's scope. ``resample`` is
the band-limited resampler the extract path needs (torchaudio's, restated).
Quirks kept on purpose: a list is cropped to its shortest member; a 2-D
array/tensor [C, T] is ONE clip with C channels (it gets a batch dim, not a
channel dim), which SpeechEmbeddings then averages (embeddings.py:183-184).
"""
from __future__ import annotations

from typing import Any, Optional, Sequence, Tuple, Union

import math
from functools import lru_cache

import numpy as np
import torch

from heybuddy.util.log_util import logger

AudioType = Union[np.ndarray, torch.Tensor, Sequence[Any]]


def audio_to_bct_tensor(input_data: AudioType, sample_rate: Optional[int] = None,
                        target_sample_rate: Optional[int] = None
                        ) -> Tuple[torch.Tensor, Optional[int]]:
    if isinstance(input_data, (list, tuple)):
        parts = [audio_to_bct_tensor(x, sample_rate) for x in input_data]
        min_frames = min(p.shape[-1] for p, _ in parts)
        rates = [sr for _, sr in parts if sr is not None]
        if rates and sample_rate is None:
            sample_rate = rates[0]
        return torch.cat([p[..., :min_frames] for p, _ in parts], dim=0), sample_rate
    if isinstance(input_data, np.ndarray):
        if sample_rate is None:
            logger.warning("No sample rate provided for numpy array input. Assuming 44100 Hz.")
            sample_rate = 44100
        waveform = torch.from_numpy(np.ascontiguousarray(input_data))
    elif isinstance(input_data, torch.Tensor):
        if sample_rate is None:
            logger.warning("No sample rate provided for torch tensor input. Assuming 44100 Hz.")
            sample_rate = 44100
        waveform = input_data
    else:
        raise ValueError(f"Unsupported input type {type(input_data)}")
    if waveform.dtype is torch.int16:
        waveform = waveform.float() / 32768.0
    elif waveform.dtype is torch.int8:
        waveform = (waveform.float() - 128) / 128.0
    if target_sample_rate is not None and sample_rate != target_sample_rate:
        waveform = resample(waveform.float(), int(sample_rate), int(target_sample_rate))
        sample_rate = target_sample_rate
    if waveform.dim() == 1:
        waveform = waveform.unsqueeze(0)
    if waveform.dim() == 2:
        waveform = waveform.unsqueeze(0)
    return waveform, sample_rate


@lru_cache(maxsize=16)
def _sinc_kernel(orig: int, new: int, width_zc: int = 6, rolloff: float = 0.99) -> Tuple[torch.Tensor, int]:
    """Polyphase windowed-sinc filters [new, 1, taps] of torchaudio's
    Resample(orig, new) (sinc_interp_hann, lowpass_filter_width 6, rolloff
    0.99; torchaudio is not installed here, so parity is unpinned): one row per
    output phase, cut off at rolloff x the lower Nyquist frequency."""
    base = min(orig, new) * rolloff
    width = math.ceil(width_zc * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    # torchaudio builds the phase offsets with arange(dtype=None), i.e. float32, before adding idx (float64)
    t = ((torch.arange(0, -new, -1, dtype=torch.float32)[:, None, None] / new).double() + idx) * base
    t = t.clamp(-width_zc, width_zc)
    window = torch.cos(t * math.pi / width_zc / 2) ** 2
    t = t * math.pi
    k = torch.where(t == 0, torch.ones_like(t), torch.sin(t) / torch.where(t == 0, torch.ones_like(t), t))
    return (k * window * (base / orig)).float(), width


def resample(waveform: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """Resample the last axis from orig_freq to new_freq (any leading shape),
    on the tensor's device: pad, strided conv with the polyphase filters,
    interleave phases, keep ceil(new * T / orig) samples."""
    if orig_freq == new_freq:
        return waveform
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    kernel, width = _sinc_kernel(orig, new)
    kernel = kernel.to(waveform.device)
    shape = waveform.shape
    x = waveform.reshape(-1, shape[-1]).float()
    n = x.shape[-1]
    x = torch.nn.functional.pad(x, (width, width + orig))
    y = torch.nn.functional.conv1d(x[:, None], kernel, stride=orig)  # [b, new, steps]
    y = y.transpose(1, 2).reshape(x.shape[0], -1)[:, :math.ceil(new * n / orig)]
    return y.reshape(*shape[:-1], y.shape[-1])
