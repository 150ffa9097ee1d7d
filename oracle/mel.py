"""Mel spectrogram oracle (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates the mel ONNX graph called by ``MelSpectrogramModel.__call__``
(reference src/python/heybuddy/spectrogram.py:23-32). The docstring there
(spectrogram.py:14-18) says the graph is "an ONNX version of the PyTorch model
from the torchaudio library"; the graph itself is absent offline, so its
parameters are hypothesis H0, pinned only by the frame
count formula ``ceil(t/160 - 3)`` (embeddings.py:67) and the shape KATs
(tests/test_embeddings.py:9-15, src/js/src/models/mel-spectrogram.js:37-49):

    torchaudio.transforms.MelSpectrogram(sample_rate=16000, n_fft=512,
        win_length=400, hop_length=160, f_min=60, f_max=3800, n_mels=32,
        power=2, center=False, mel_scale="htk", norm=None)
    -> AmplitudeToDB(stype="power", top_db=None): 10 log10(max(P, 1e-10))

followed by the host post-scale ``x / 10 + 2`` (spectrogram.py:32).
Parity of the HIP kernel is against this restatement (fp64 FFT).
"""
from __future__ import annotations

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 512
WIN_LENGTH = 400
HOP = 160
F_MIN = 60.0
F_MAX = 3800.0
N_MELS = 32
LOG_FLOOR = 1e-10
IN_SCALE = 32767.0  # embeddings.py:182


def hann_window(win_length: int = WIN_LENGTH, n_fft: int = N_FFT) -> np.ndarray:
    """torch.hann_window(win_length, periodic=True), zero-padded and centred in
    n_fft exactly as torch.stft does for win_length < n_fft."""
    n = np.arange(win_length, dtype=np.float64)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / win_length)
    out = np.zeros(n_fft, dtype=np.float64)
    left = (n_fft - win_length) // 2
    out[left:left + win_length] = w
    return out.astype(np.float32)


def _hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def _mel_to_hz_htk(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def mel_fbank(n_freqs: int = N_FFT // 2 + 1, f_min: float = F_MIN, f_max: float = F_MAX,
              n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE) -> np.ndarray:
    """torchaudio.functional.melscale_fbanks(..., norm=None, mel_scale="htk"):
    triangular filters, layout [n_freqs, n_mels], float32."""
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    m_pts = np.linspace(_hz_to_mel_htk(f_min), _hz_to_mel_htk(f_max), n_mels + 2)
    f_pts = _mel_to_hz_htk(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up)).astype(np.float32)


def n_frames_for(t: int, n_fft: int = N_FFT, hop: int = HOP) -> int:
    """Unique frames of a t-sample signal with no centre padding; equals the
    reference's ceil(t/160 - 3) (embeddings.py:67) for t = 17,280."""
    return (t - n_fft) // hop + 1


def power_mel(frames: np.ndarray, window: np.ndarray, fbank: np.ndarray, energy: bool = False):
    """|rFFT(frames * window)|^2 @ fbank in float64. frames: [..., n_fft].
    With energy=True also returns sum_k |X_k|^2 per frame."""
    x = frames.astype(np.float64) * window.astype(np.float64)
    spec = np.fft.rfft(x, axis=-1)
    p = spec.real ** 2 + spec.imag ** 2
    mel = p @ fbank.astype(np.float64)
    if energy:
        return mel, p.sum(axis=-1)
    return mel


def mel_graph(audio: np.ndarray, window=None, fbank=None, hop: int = HOP,
              log_floor: float = LOG_FLOOR) -> np.ndarray:
    """The ONNX mel graph (H0): audio [b, t] (int16-range f32) ->
    [b, 1, frames, n_mels] = 10 log10(max(mel, 1e-10))."""
    window = hann_window() if window is None else window
    fbank = mel_fbank() if fbank is None else fbank
    audio = np.asarray(audio)
    if audio.ndim == 1:
        audio = audio[None]
    n_fft = window.shape[0]
    nf = n_frames_for(audio.shape[1], n_fft, hop)
    idx = np.arange(nf)[:, None] * hop + np.arange(n_fft)[None, :]
    mel = power_mel(audio[:, idx], window, fbank)
    out = 10.0 * np.log10(np.maximum(mel, log_floor))
    return out[:, None].astype(np.float32)


def mel_spectrogram_model(audio: np.ndarray, **kw) -> np.ndarray:
    """MelSpectrogramModel.__call__ (spectrogram.py:23-32): graph output
    squeezed, then /10 + 2."""
    audio = np.asarray(audio)
    if audio.ndim == 1:
        audio = audio[np.newaxis, :]
    assert audio.ndim == 2
    pred = mel_graph(audio.astype(np.float32), **kw)
    return np.squeeze(pred) / np.float32(10) + np.float32(2)


def mel_frames(pcm: np.ndarray, n_frames: int | None = None, in_scale: float = IN_SCALE,
               window=None, fbank=None, hop: int = HOP, log_floor: float = LOG_FLOOR,
               out_div: float = 10.0, out_add: float = 2.0) -> np.ndarray:
    """What hbk_mel_frames computes: the unique frames of every clip.

    pcm: [B, T] float in [-1, 1]; frame f of clip b covers samples
    [hop f, hop f + n_fft) of pcm * in_scale. Returns [B, n_frames, n_mels] f32.
    """
    window = hann_window() if window is None else window
    fbank = mel_fbank() if fbank is None else fbank
    pcm = np.asarray(pcm, dtype=np.float32)
    n_fft = window.shape[0]
    if n_frames is None:
        n_frames = n_frames_for(pcm.shape[1], n_fft, hop)
    scaled = pcm * np.float32(in_scale)  # f32 rounding, as the reference (embeddings.py:182)
    idx = np.arange(n_frames)[:, None] * hop + np.arange(n_fft)[None, :]
    mel, energy = power_mel(scaled[:, idx], window, fbank, energy=True)
    out = 10.0 * np.log10(np.maximum(mel, log_floor)) / out_div + out_add
    return out.astype(np.float32), mel, energy


def fp32_noise_tolerance(mel_pow: np.ndarray, frames_energy: np.ndarray, base: float = 1e-4,
                         c: float = 64.0) -> np.ndarray:
    """Tolerance on the log10 mel output of an fp32 FFT.

    An fp32 FFT carries an absolute error of ~c * 2^-24 * ||X|| per bin, so a
    mel bin whose power sits far below the frame's energy is only resolved to
    delta log10 ~ 2 sqrt(P_floor / P) / ln 10. ``mel_pow`` [..., n_mels] is the
    (fp64) mel power, ``frames_energy`` [...] the frame's total spectral energy
    sum_k |X_k|^2 (c absorbs the filter width and the FFT depth). Bins within ~60 dB of the
    frame energy get the flat 1e-4 bound; DC / pure-tone frames get the
    physically achievable one.
    """
    eps = c * 2.0 ** -24
    floor = (eps ** 2) * frames_energy[..., None]
    ratio = floor / np.maximum(mel_pow, 1e-30)
    return base + (2.0 * np.sqrt(ratio) + ratio) / np.log(10.0)
