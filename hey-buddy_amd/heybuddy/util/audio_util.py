"""Input normalisation of the featurizer.

Mirrors ``audio_to_bct_tensor`` (reference util/audio_util.py:73-145) for the
in-memory inputs the hot path receives (lists, numpy arrays, torch tensors);
file / URI / bytes decoding and resampling are outside this build's scope.
Quirks kept on purpose: a list is cropped to its shortest member; a 2-D
array/tensor [C, T] is ONE clip with C channels (it gets a batch dim, not a
channel dim), which SpeechEmbeddings then averages (embeddings.py:183-184).
"""
from __future__ import annotations

from typing import Any, Optional, Sequence, Tuple, Union

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
        raise NotImplementedError("resampling is outside the MI355X hot path")
    if waveform.dim() == 1:
        waveform = waveform.unsqueeze(0)
    if waveform.dim() == 2:
        waveform = waveform.unsqueeze(0)
    return waveform, sample_rate
