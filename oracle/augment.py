"""Augmentation oracle (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates three batch augmentations of AugmentedAudioGenerator.execute_augment_batch
(reference src/python/heybuddy/dataset/augmented.py:114-118, :383-392). Both live in
third-party packages that are not installed here, so they are restated from
their published algorithms at the versions environment.yml pins
(PARITY UNPINNED at the third-party boundary; the reference holds no fixture):

* torch_audiomentations.Gain (min -18 dB, max 6 dB, mode per_batch, p
  DEFAULT_AUGMENT_GAIN_PROB = 1.0, constants.py:136): y = 10^(g/20) x with
  g ~ U[-18, 6] dB; the last transform of the torch_audiomentations chain, so
  it precedes the noise mix and the reverb;
* torchaudio.functional.add_noise (torchaudio >= 2.3, environment.yml:28),
  called by add_background_noise_to_batch (augmented.py:234-276):
      E_x = ||x||^2, E_n = ||n||^2 (per clip)
      snr_0 = 10 (log10 E_x - log10 E_n)
      y = x + 10^((snr_0 - snr) / 20) * n
  with the noise of clip b = samples [b T, (b+1) T) of the concatenation of
  consecutive background clips (augmented.py:246-267).
* speechbrain.processing.signal_processing.reverberate(x, ir, rescale_amp="avg")
  (speechbrain >= 1.0, environment.yml:24), one IR per batch (augmented.py:389-392):
      a_in = mean |x|  (per clip)
      d = argmax |ir|; if L > T: ir = ir[:T]
      k = [ir[d:], zeros(T - L), ir[:d]]
      y = irfft(rfft(x) * rfft(k), n=T)          (circular, length T)
      y = a_in * y / (mean |y| + 1e-14)
* torch_audiomentations.AddColoredNoise (min/max SNR 10/30 dB, f_decay -1..2,
  mode per_batch, p 0.25; augmented.py:107-113, constants.py:128-132), between
  band-stop and gain in the batch chain. per_batch mode: torch_audiomentations'
  BaseWaveformTransform.forward reshapes the batch to (1, batch * channels, T)
  before randomize_parameters / apply_transform, so ONE (snr, f_decay) and ONE
  noise vector serve the whole batch (the same holds for Gain, BandStopFilter
  and PitchShift: one parameter set per batch); rms(x) stays per clip:
      w ~ N(0, 1) [T];  S = rfft(w) / linspace(1, sqrt(sr / 2), T/2 + 1)^f_decay
      n = irfft(S);  n = n / (rms(n) + 1e-8)                 (Audio.rms_normalize)
      y = x + rms(x) / 10^(snr / 20) * n                     (calculate_rms)
  The white noise is an explicit input (torch.randn's stream is not reproduced).
* audiomentations.TanhDistortion (p 0.25 per clip, distortion ~ U[1e-4, 0.1];
  augmented.py:79-90, constants.py:122-124), in the per-clip Compose before H2D:
      th = np.percentile(|x|, 100 - 99 amount);  y = tanh(0.5 / (th + 1e-6) x)
      if rms(x) > 1e-9: y *= rms(x) / rms(y)
* audiomentations.SevenBandParametricEQ (p 0.25 per clip, gains +-6 dB;
  augmented.py:79-84, constants.py:120-121), first in the per-clip Compose:
  a low shelf, five peaking filters and a high shelf (RBJ audio-EQ-cookbook
  biquads, each applied with scipy sosfilt = direct form II transposed in
  float64, its output cast back to float32 before the next filter). Per filter
  k: center frequency mel-uniform in the band's range (low shelf 42-95 Hz,
  peaks 91-204, 196-441, 421-948, 909-2045, 1957-4404 Hz, high shelf
  4216-9486 Hz, clamped to 0.95 Nyquist), gain ~ U[-g, g] dB, Q ~ U[0.5, 1.33];
      A = 10^(gain/40), w0 = 2 pi f0 / sr, alpha = sin(w0) / (2 Q)
  (the band ranges, Q range and draw distributions are restated from the
  package's documentation: PARITY UNPINNED, no fixture exists).
* torch_audiomentations.BandStopFilter (torch_audiomentations >= 0.11,
  environment.yml:27; p 0.25, mode per_batch: one coin AND one parameter set
  per batch (the (1, batch * channels, T) reshape above); augmented.py:101-105,
  constants.py:127), second in the batch chain (after PitchShift, before
  AddColoredNoise). Per batch: center frequency
  mel-uniform in [200, 4000] Hz, bandwidth fraction ~ U[0.5, 1.99],
      cut_lo = f_c (1 - bw/2) / sr,  cut_hi = f_c (1 + bw/2) / sr   (float32)
  and y = x - julius.bandpass_filter(x, cut_lo, cut_hi) with julius's
  LowPassFilters([cut_lo, cut_hi], zeros=8): half_size h = int(8 / cut_lo / 2),
  taps t in [-h, h], window hann(2h + 1, periodic=False),
      f_c[t] = 2 c w[t] sinc(2 pi c t),  f_c /= sum(f_c)        (float32 math)
      bandpass = conv1d(pad(x, h, 'replicate'), f_hi) - (same with f_lo)
  (julius switches to an FFT convolution for h > 32: the same linear
  convolution up to rounding). PARITY UNPINNED: neither package is installed.
"""
from __future__ import annotations

import numpy as np
from scipy.signal import sosfilt


def add_noise(x: np.ndarray, noise: np.ndarray, snr_db: np.ndarray, dtype=np.float64) -> np.ndarray:
    x = np.asarray(x, dtype=dtype)
    n = np.asarray(noise, dtype=dtype)
    with np.errstate(divide="ignore", invalid="ignore"):
        ex = (x * x).sum(axis=-1)
        en = (n * n).sum(axis=-1)
        snr0 = 10.0 * (np.log10(ex) - np.log10(en))
        scale = 10.0 ** ((snr0 - np.asarray(snr_db, dtype=dtype)) / 20.0)
        return x + scale[..., None] * n


def noise_segments(bank: list, start_clip: int, batch: int, T: int):
    """augmented.py:246-267: concatenate background clips from ``start_clip``
    (cycling) until >= batch*T samples, split into ``batch`` segments of T.
    Returns (segments [batch, T], next clip index)."""
    parts, total, i = [], 0, start_clip
    while total < batch * T:
        c = np.asarray(bank[i % len(bank)], dtype=np.float64)
        parts.append(c)
        total += c.shape[0]
        i += 1
    cat = np.concatenate(parts)[:batch * T]
    return cat.reshape(batch, T), i


def reverb_kernel(ir: np.ndarray, T: int) -> np.ndarray:
    """The rotated length-T kernel of speechbrain's convolve1d(use_fft=True,
    rotation_index=argmax|ir|)."""
    ir = np.asarray(ir, dtype=np.float64)
    d = int(np.argmax(np.abs(ir)))
    if ir.shape[0] > T:
        ir = ir[:T]
    zeros = np.zeros(T - ir.shape[0])
    return np.concatenate([ir[d:], zeros, ir[:d]])


def reverberate(x: np.ndarray, ir: np.ndarray, dtype=np.float64) -> np.ndarray:
    x = np.asarray(x, dtype=dtype)
    T = x.shape[-1]
    a_in = np.abs(x).mean(axis=-1, keepdims=True)
    k = reverb_kernel(ir, T)
    y = np.fft.irfft(np.fft.rfft(x, axis=-1) * np.fft.rfft(k), n=T, axis=-1)
    return a_in * y / (np.abs(y).mean(axis=-1, keepdims=True) + 1e-14)


def gen_colored_noise(white, f_decay, num_samples: int, sample_rate: int = 16000, dtype=np.float64):
    """torch_audiomentations' _gen_noise (AddColoredNoise, the reference's batch
    chain, augmented.py:107-113) with the white noise given: ``sample_rate``
    N(0,1) samples (ONE second), rfft, mask 1 / linspace(1, sqrt(sr/2),
    sr/2 + 1)^f_decay, irfft (n = sr), RMS-normalise (/ (rms + 1e-8)), then
    TILE to num_samples (ceil(num_samples / sr) copies, cut). torch_audiomentations
    is not installed here: restated from its published source (lower bound pinned
    by the reference's environment.yml); parity unpinned against the package."""
    w = np.asarray(white, dtype=dtype)[..., :sample_rate]
    spec = np.fft.rfft(w, axis=-1)
    lin = np.linspace(1.0, np.sqrt(sample_rate / 2.0), spec.shape[-1])
    fd = np.asarray(f_decay, dtype=dtype).reshape(-1, 1)
    n = np.fft.irfft(spec / lin[None, :] ** fd, n=sample_rate, axis=-1)
    n = n / (np.sqrt((n * n).mean(axis=-1, keepdims=True)) + 1e-8)
    reps = -(-num_samples // sample_rate)
    return np.concatenate([n] * reps, axis=-1)[..., :num_samples]


def colored_noise(x, white, f_decay, snr_db, sample_rate: int = 16000, dtype=np.float64) -> np.ndarray:
    """AddColoredNoise.apply_transform with the white noise given:
    y = x + rms(x) / 10^(snr/20) * noise, rms over the clip (calculate_rms)."""
    x = np.asarray(x, dtype=dtype)
    n = gen_colored_noise(white, f_decay, x.shape[-1], sample_rate, dtype)
    rms_x = np.sqrt((x * x).mean(axis=-1, keepdims=True))
    return x + rms_x / 10.0 ** (np.asarray(snr_db, dtype=dtype).reshape(-1, 1) / 20.0) * n


def tanh_distortion(x, amount) -> np.ndarray:
    """TanhDistortion.apply on float32 clips (audiomentations computes in the clip dtype)."""
    x = np.asarray(x, dtype=np.float32)
    out = np.empty_like(x)
    for i, a in enumerate(np.asarray(amount, dtype=np.float64).reshape(-1)):
        th = np.percentile(np.abs(x[i]), 100 - 99 * a)
        y = np.tanh((0.5 / (th + 1e-6)) * x[i]).astype(np.float32)
        rb = np.sqrt(np.mean(np.square(x[i])))
        if rb > 1e-9:
            y = (rb / np.sqrt(np.mean(np.square(y)))) * y
        out[i] = y
    return out


def db_to_amplitude(db) -> np.ndarray:
    """torch_audiomentations.utils.dsp.convert_decibels_to_amplitude_ratio."""
    return 10.0 ** (np.asarray(db, dtype=np.float64) / 20.0)


def augment_batch(x, noise=None, snr_db=None, ir=None, dtype=np.float64, gain=None):
    """gain (linear factor per clip, if given), noise mix (if noise is given),
    then reverb (if ir is given), as execute_augment_batch applies them
    (augmented.py:114-118 inside augment_batch, then :383-392)."""
    y = np.asarray(x, dtype=dtype)
    if gain is not None:
        y = y * np.asarray(gain, dtype=dtype).reshape(-1, 1)
    if noise is not None:
        y = add_noise(y, noise, snr_db, dtype)
    if ir is not None:
        y = reverberate(y, ir, dtype)
    return y


# --------------------------------------------------------------------------
# SevenBandParametricEQ
EQ_BANDS = ((42.0, 95.0), (91.0, 204.0), (196.0, 441.0), (421.0, 948.0), (909.0, 2045.0),
            (1957.0, 4404.0), (4216.0, 9486.0))  # low shelf, 5 peaks, high shelf
EQ_Q = (0.5, 1.33)


def hz_to_mel(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_to_hz(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def eq_draw(rng, n: int, gain_db: float, sample_rate: int = 16000):
    """(center Hz, gain dB, Q) [n, 7, 3] for n clips."""
    lo = hz_to_mel([b[0] for b in EQ_BANDS])
    hi = hz_to_mel([b[1] for b in EQ_BANDS])
    f0 = mel_to_hz(rng.uniform(lo, hi, (n, 7)))
    f0[:, 6] = np.minimum(f0[:, 6], (sample_rate // 2) * 0.95)
    g = rng.uniform(-gain_db, gain_db, (n, 7))
    q = rng.uniform(EQ_Q[0], EQ_Q[1], (n, 7))
    return np.stack([f0, g, q], axis=-1)


def eq_sos(params, sample_rate: int = 16000) -> np.ndarray:
    """RBJ biquads [..., 7, 6] (b0, b1, b2, 1, a1, a2; normalised by a0) from
    eq_draw parameters [..., 7, 3]: filter 0 low shelf, 1-5 peaking, 6 high shelf."""
    params = np.asarray(params, dtype=np.float64)
    f0, gdb, q = params[..., 0], params[..., 1], params[..., 2]
    A = 10.0 ** (gdb / 40.0)
    w0 = 2.0 * np.pi * f0 / sample_rate
    c, al = np.cos(w0), np.sin(w0) / (2.0 * q)
    sA = np.sqrt(A)
    # peaking
    pb = np.stack([1 + al * A, -2 * c, 1 - al * A], -1)
    pa = np.stack([1 + al / A, -2 * c, 1 - al / A], -1)
    # low shelf
    lb = np.stack([A * ((A + 1) - (A - 1) * c + 2 * sA * al), 2 * A * ((A - 1) - (A + 1) * c),
                   A * ((A + 1) - (A - 1) * c - 2 * sA * al)], -1)
    la = np.stack([(A + 1) + (A - 1) * c + 2 * sA * al, -2 * ((A - 1) + (A + 1) * c),
                   (A + 1) + (A - 1) * c - 2 * sA * al], -1)
    # high shelf
    hb = np.stack([A * ((A + 1) + (A - 1) * c + 2 * sA * al), -2 * A * ((A - 1) + (A + 1) * c),
                   A * ((A + 1) + (A - 1) * c - 2 * sA * al)], -1)
    ha = np.stack([(A + 1) - (A - 1) * c + 2 * sA * al, 2 * ((A - 1) - (A + 1) * c),
                   (A + 1) - (A - 1) * c - 2 * sA * al], -1)
    k = np.arange(7)
    b = np.where((k == 0)[:, None], lb, np.where((k == 6)[:, None], hb, pb))
    a = np.where((k == 0)[:, None], la, np.where((k == 6)[:, None], ha, pa))
    a0 = a[..., :1]
    return np.concatenate([b / a0, np.ones_like(a0), a[..., 1:] / a0], axis=-1)


def seven_band_eq(x, sos) -> np.ndarray:
    """The cascade on float32 clips x [n, T] with per-clip sos [n, 7, 6]; a NaN
    b0 in filter 0 leaves the clip unchanged (the transform's coin came up
    tails). Each stage: DF2T in float64 on the float32 input, output cast to
    float32 (audiomentations: sosfilt(...).astype(np.float32))."""
    x = np.asarray(x, dtype=np.float32)
    out = x.copy()
    sos = np.asarray(sos, dtype=np.float64)
    for i in range(x.shape[0]):
        if np.isnan(sos[i, 0, 0]):
            continue
        y = x[i]
        for k in range(7):  # scipy.signal.sosfilt: the DF2T recursion audiomentations calls
            y = sosfilt(sos[i, k][None], y).astype(np.float32)
        out[i] = y
    return out


# --------------------------------------------------------------------------
# BandStopFilter
BANDSTOP_CENTER = (200.0, 4000.0)
BANDSTOP_BANDWIDTH = (0.5, 1.99)


def bandstop_draw(rng, n: int, sample_rate: int = 16000):
    """(cut_lo, cut_hi) [n] float32 fractions of the sample rate: f_c
    mel-uniform in BANDSTOP_CENTER, bandwidth fraction uniform (float32 math,
    as torch_audiomentations' tensors)."""
    lo, hi = hz_to_mel(BANDSTOP_CENTER)
    fc = mel_to_hz(rng.uniform(lo, hi, n)).astype(np.float32)
    bw = rng.uniform(*BANDSTOP_BANDWIDTH, n).astype(np.float32)
    sr = np.float32(sample_rate)
    return (fc * (np.float32(1) - bw / np.float32(2)) / sr).astype(np.float32), \
        (fc * (np.float32(1) + bw / np.float32(2)) / sr).astype(np.float32)


def bandstop_half_size(cut_lo) -> int:
    """julius LowPassFilters.half_size = int(zeros / min(cutoffs) / 2), zeros 8."""
    return int(8 / float(cut_lo) / 2)


def lowpass_taps(cutoff, half: int) -> np.ndarray:
    """julius' windowed-sinc lowpass [2 half + 1] in float32 arithmetic:
    2 c hann[t] sinc(2 pi c t), normalised to unit sum."""
    n = 2 * half + 1
    k = np.arange(n, dtype=np.float32)
    hann = (np.float32(0.5) - np.float32(0.5) * np.cos(k * np.float32(2.0 * np.pi / (n - 1)))).astype(np.float32) \
        if n > 1 else np.ones(1, np.float32)
    t = np.arange(-half, half + 1).astype(np.float32)
    arg = (np.float32(2.0 * float(cutoff) * np.pi) * t).astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        sinc = np.where(arg == 0, np.float32(1), (np.sin(arg) / arg).astype(np.float32))
    f = (np.float32(2.0 * float(cutoff)) * hann * sinc).astype(np.float32)
    return (f / f.astype(np.float64).sum().astype(np.float32)).astype(np.float32)


def band_stop(x, cut_lo, cut_hi) -> np.ndarray:
    """x [n, T] float32 -> x - bandpass(x), per-clip cutoffs (float64
    convolution of the float32 taps; a NaN cut_lo leaves the clip unchanged)."""
    from scipy.signal import fftconvolve
    x = np.asarray(x, dtype=np.float32)
    out = x.copy()
    for i in range(x.shape[0]):
        if np.isnan(cut_lo[i]):
            continue
        h = bandstop_half_size(cut_lo[i])
        g = lowpass_taps(cut_hi[i], h).astype(np.float64) - lowpass_taps(cut_lo[i], h).astype(np.float64)
        xp = np.pad(x[i].astype(np.float64), h, mode="edge")
        bp = fftconvolve(xp, g[::-1], mode="valid")  # conv1d is a correlation; g is symmetric anyway
        out[i] = (x[i] - bp).astype(np.float32)
    return out


# PitchShift (torch_audiomentations PitchShift, mode per_batch, p 0.25, +-3
# semitones; augmented.py:93-100, constants.py:125-126) -> torch_pitch_shift
# (>= 1.2, unpinned: not in environment.yml's explicit list) -> torch.stft /
# torchaudio TimeStretch (phase_vocoder) / torch.istft / torchaudio Resample.
# PARITY UNPINNED: none of these packages is installed; the restatement below
# follows their published algorithms and computes in float64 throughout (the
# reference runs them in float32, whose phase cumsum alone carries ~1e-2 rad of
# rounding at the top bins).

def _prime_factors(n: int) -> list:
    out, d = [], 2
    while n > 1:
        while n % d == 0:
            out.append(d)
            n //= d
        d += 1
    return out


def pitch_fast_shifts(sample_rate: int = 16000, semitones: float = 3.0) -> list:
    """torch_pitch_shift.get_fast_shifts(sample_rate, lo <= f <= hi and f != 1)
    with lo / hi = Fraction(2 ** (-+semitones / 12)) (semitones_to_ratio): the
    ratios i / j of products of sample_rate's prime factors. At 16 kHz and +-3
    semitones that is {125/128, 128/125} (+-0.41 semitones)."""
    from fractions import Fraction
    from itertools import combinations
    from math import prod
    fac = _prime_factors(sample_rate)
    products = {prod(c) for r in range(1, len(fac) + 1) for c in combinations(fac, r)}
    lo, hi = Fraction(2.0 ** (-semitones / 12.0)), Fraction(2.0 ** (semitones / 12.0))
    return sorted({Fraction(i, j) for i in products for j in products if lo <= Fraction(i, j) <= hi} - {1})


def pitch_shift_geometry(length: int, num: int, den: int, sample_rate: int = 16000) -> dict:
    """Frame counts and resampler shape of pitch_shift(x, Fraction(num, den))."""
    from math import ceil, gcd
    n_fft = sample_rate // 64
    hop = n_fft // 32
    f_in = 1 + length // hop                       # torch.stft, center=True
    rate = float(den) / float(num)                 # TimeStretch(fixed_rate = float(1 / shift))
    f_out = int(ceil(f_in / rate))                 # torch.arange(0, f_in, rate).numel()
    l1 = hop * (f_out - 1)                         # torch.istft, center=True, length=None
    new_sr = (sample_rate * den) // num            # int(sample_rate / shift)
    g = gcd(sample_rate, new_sr)
    orig, new = sample_rate // g, new_sr // g
    width = int(ceil(6 * orig / (min(orig, new) * 0.99)))
    target = int(ceil(new * l1 / orig))
    return dict(n_fft=n_fft, hop=hop, f_in=f_in, rate=rate, f_out=f_out, l1=l1, orig=orig, new=new,
                width=width, target=target)


def resample_taps(orig: int, new: int) -> tuple:
    """torchaudio _get_sinc_resample_kernel (sinc_interp_hann, lowpass_filter_width
    6, rolloff 0.99, dtype None: float64 math, float32 taps) -> ([new, 2w + orig], w)."""
    from math import ceil
    lpw = 6.0
    base = min(orig, new) * 0.99
    width = int(ceil(lpw * orig / base))
    idx = np.arange(-width, width + orig, dtype=np.float64)[None] / orig
    t = (np.arange(0, -new, -1) / new).astype(np.float32).astype(np.float64)[:, None] + idx
    t = np.clip(t * base, -lpw, lpw)
    window = np.cos(t * np.pi / lpw / 2) ** 2
    t = t * np.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    return (k * window * (base / orig)).astype(np.float32), width


def pitch_shift(x, num: int, den: int, sample_rate: int = 16000) -> np.ndarray:
    """torch_pitch_shift.pitch_shift(x, Fraction(num, den), sample_rate) per clip
    (rows of x), float64:
      X = stft(x, n_fft = sr // 64, hop = n_fft // 32)   rectangular window,
          center, reflect padding, onesided
      phase_vocoder(X, rate = den / num, adv_k = linspace(0, pi hop, n_fft/2 + 1)):
          ts = arange(0, F, rate) (float32), i0 = int(ts), a = ts % 1
          X padded with 2 zero frames; ph = angle(X[i0+1]) - angle(X[i0]) - adv
          ph -= 2 pi round(ph / 2 pi); ph += adv
          acc = cumsum([angle(X[0]), ph[:-1]]);  Y = (a |X[i0+1]| + (1-a) |X[i0]|) e^(i acc)
      y = istft(Y)  (overlap-add / frame count, trimmed by n_fft // 2)
      y = Resample(sr, int(sr / shift))(y), cropped or zero-padded to len(x)."""
    x = np.atleast_2d(np.asarray(x, dtype=np.float64))
    n, L = x.shape
    g = pitch_shift_geometry(L, num, den, sample_rate)
    n_fft, hop, f_in, f_out = g["n_fft"], g["hop"], g["f_in"], g["f_out"]
    pad = n_fft // 2
    nb = n_fft // 2 + 1
    xp = np.pad(x, ((0, 0), (pad, pad)), mode="reflect")
    fidx = hop * np.arange(f_in)[:, None] + np.arange(n_fft)[None]
    X = np.fft.rfft(xp[:, fidx], axis=-1)                                # [n, f_in, nb]
    ts = (np.arange(f_out, dtype=np.float64) * g["rate"]).astype(np.float32)
    i0 = ts.astype(np.int64)
    alpha = (ts - np.floor(ts)).astype(np.float64)[None, :, None]
    Xp = np.concatenate([X, np.zeros((n, 2, nb), X.dtype)], axis=1)
    X0, X1 = Xp[:, i0], Xp[:, i0 + 1]
    adv = np.linspace(0.0, np.pi * hop, nb)
    ph = np.angle(X1) - np.angle(X0) - adv
    ph = ph - 2 * np.pi * np.round(ph / (2 * np.pi)) + adv
    ph = np.concatenate([np.angle(X[:, :1]), ph[:, :-1]], axis=1)
    acc = np.cumsum(ph, axis=1)
    Y = (alpha * np.abs(X1) + (1.0 - alpha) * np.abs(X0)) * np.exp(1j * acc)
    frames = np.fft.irfft(Y, n=n_fft, axis=-1)                           # [n, f_out, n_fft]
    full = np.zeros((n, n_fft + hop * (f_out - 1)))
    env = np.zeros(full.shape[1])
    for t in range(f_out):
        full[:, hop * t:hop * t + n_fft] += frames[:, t]
        env[hop * t:hop * t + n_fft] += 1.0
    y = full[:, pad:pad + g["l1"]] / env[pad:pad + g["l1"]]
    taps, w = resample_taps(g["orig"], g["new"])
    orig, new = g["orig"], g["new"]
    ypad = np.pad(y, ((0, 0), (w, w + orig)))
    nfr = g["l1"] // orig + 1
    win = orig * np.arange(nfr)[:, None] + np.arange(2 * w + orig)[None]
    res = np.einsum("nfq,pq->nfp", ypad[:, win], taps.astype(np.float64)).reshape(n, -1)[:, :g["target"]]
    out = np.zeros((n, L))
    m = min(L, res.shape[1])
    out[:, :m] = res[:, :m]
    return out


def pitch_shift_torch(x, num: int, den: int, sample_rate: int = 16000) -> np.ndarray:
    """pitch_shift in float32 torch CPU ops, as the reference's packages run it
    (torch.stft / torch.istft, torchaudio's phase_vocoder and Resample written
    out): the timed CPU baseline's pitch shift (bench.py config 5); the float64
    pitch_shift above stays the parity oracle."""
    import math
    import torch
    import torch.nn.functional as F
    x = torch.as_tensor(np.atleast_2d(np.asarray(x, dtype=np.float32)))
    n, L = x.shape
    g = pitch_shift_geometry(L, num, den, sample_rate)
    n_fft, hop = g["n_fft"], g["hop"]
    X = torch.stft(x, n_fft, hop, window=torch.ones(n_fft), center=True, pad_mode="reflect",
                   return_complex=True)  # [n, nb, f_in]; torch_pitch_shift passes no window: rectangular
    nb = X.shape[1]
    adv = torch.linspace(0, math.pi * hop, nb)[:, None]
    ts = torch.arange(0, X.shape[-1], g["rate"], dtype=torch.float32)
    alpha = ts % 1.0
    ph0 = X[..., :1].angle()
    Xp = F.pad(X, [0, 2])
    X0, X1 = Xp.index_select(-1, ts.long()), Xp.index_select(-1, (ts + 1).long())
    ph = X1.angle() - X0.angle() - adv
    ph = ph - 2 * math.pi * torch.round(ph / (2 * math.pi)) + adv
    acc = torch.cumsum(torch.cat([ph0, ph[..., :-1]], -1), -1)
    Y = torch.polar(alpha * X1.abs() + (1 - alpha) * X0.abs(), acc)
    y = torch.istft(Y, n_fft, hop, window=torch.ones(n_fft), center=True)
    taps, w = resample_taps(g["orig"], g["new"])
    orig = g["orig"]
    yp = F.pad(y[:, None], (w, w + orig))
    res = F.conv1d(yp, torch.from_numpy(taps)[:, None], stride=orig).transpose(1, 2).reshape(n, -1)[:, :g["target"]]
    out = torch.zeros((n, L))
    m = min(L, res.shape[1])
    out[:, :m] = res[:, :m]
    return out.numpy()


# --------------------------------------------------------------------------
# The whole chain of AugmentedAudioGenerator.execute_augment_batch
# (augmented.py:297-394), used as bench.py's CPU baseline (config 5) and by
# tests: placement (to_target_length, :200-232), per clip [7-band EQ p .25,
# tanh p .25] (:79-90, :314-328), per batch [pitch shift p .25, band-stop
# p .25, colored noise p .25, gain p 1.0] (:93-121, :368-380), background
# noise p .75 (:383-384), reverb p .75 (:386-392).
def place(clip, length: int, T: int, rng) -> np.ndarray:
    """to_target_length: crop to T, or pad with U[S/4, 3S/4) leading zeros."""
    x = np.asarray(clip[:length], dtype=np.float32)
    if length >= T:
        return x[:T].copy()
    out = np.zeros(T, np.float32)
    s = T - length
    pre = int(rng.integers(s // 4, max(s // 4 + 1, 3 * s // 4)))
    out[pre:pre + length] = x
    return out


COIN_KINDS = ("pitch", "bandstop", "colored", "gain", "noise", "reverb")


def stratified_coins(rng, nb: int, p_pitch=0.25, p_bandstop=0.25, p_colored=0.25, p_gain=1.0, p_noise=0.75,
                     p_reverb=0.75):
    """augment_chain's per-batch coins for nb batches, each kind on exactly
    round(p * nb) batches (a random subset)."""
    out = {}
    for k, p in zip(COIN_KINDS, (p_pitch, p_bandstop, p_colored, p_gain, p_noise, p_reverb)):
        on = np.zeros(nb, bool)
        on[rng.permutation(nb)[:int(round(p * nb))]] = True
        out[k] = on
    return out


def augment_chain(src, lengths, rng, noise_bank, irs, T: int = 23040, batch: int = 128,
                  p_eq=0.25, p_tanh=0.25, p_pitch=0.25, p_bandstop=0.25, p_colored=0.25, p_gain=1.0,
                  p_noise=0.75, p_reverb=0.75, stratify: bool = False, fast_pitch: bool = False,
                  coins_given=None, batch0: int = 0):
    """src [n, >= T] utterances with valid lengths -> augmented [n, T] float32.
    Per-batch coins from ``rng``; stratify=True turns each per-batch coin into
    exactly round(p * n_batches) batches (a random subset), so a small sample
    carries the chain's expected cost; fast_pitch: the float32 torch pitch
    shift (the reference's own cost) instead of the float64 restatement.
    coins_given: {"pitch", "bandstop", "colored", "gain", "noise", "reverb"} ->
    per-batch booleans decided by the caller (a worker's share of a larger
    sample, whose first batch is global batch ``batch0``; stratified_coins).
    Returns (y, counts of applied stages)."""
    n = len(src)
    x = np.stack([place(src[i], int(lengths[i]), T, rng) for i in range(n)])
    cnt = {}
    e_on = rng.random(n) < p_eq
    if e_on.any():
        sos = np.full((n, 7, 6), np.nan)
        sos[e_on] = eq_sos(eq_draw(rng, int(e_on.sum()), 6.0))
        x = seven_band_eq(x, sos)
    t_on = rng.random(n) < p_tanh
    for i in np.flatnonzero(t_on):
        x[i] = tanh_distortion(x[i:i + 1], rng.uniform(1e-4, 0.1))[0]
    cnt["eq_clips"], cnt["tanh_clips"] = int(e_on.sum()), int(t_on.sum())
    nb = (n + batch - 1) // batch

    def coins(p):
        if stratify:
            on = np.zeros(nb, bool)
            on[rng.permutation(nb)[:int(round(p * nb))]] = True
            return on
        return rng.random(nb) < p

    if coins_given is not None:
        c_pitch, c_bs, c_col, c_gain, c_noise, c_rev = (np.asarray(coins_given[k], bool)[:nb] for k in COIN_KINDS)
    else:
        c_pitch, c_bs, c_col, c_gain, c_noise, c_rev = (coins(p) for p in (p_pitch, p_bandstop, p_colored, p_gain,
                                                                           p_noise, p_reverb))
    ring = np.concatenate([np.asarray(v, np.float32) for v in noise_bank])
    ring_pos = (batch0 * batch * T) % ring.size
    shifts = ((125, 128), (128, 125))
    for b in range(nb):
        sl = slice(b * batch, min(n, (b + 1) * batch))
        y = x[sl].astype(np.float64)
        m = y.shape[0]
        if c_pitch[b]:
            num, den = shifts[int(rng.integers(0, 2))]
            for s in range(0, m, 32):
                y[s:s + 32] = (pitch_shift_torch if fast_pitch else pitch_shift)(y[s:s + 32], num, den)
        if c_bs[b]:
            lo, hi = bandstop_draw(rng, 1)
            y = band_stop(y.astype(np.float32), np.repeat(lo, m), np.repeat(hi, m)).astype(np.float64)
        if c_col[b]:
            w = np.repeat(rng.standard_normal((1, 16000)), m, axis=0)
            y = colored_noise(y, w, np.full(m, rng.uniform(-1, 2)), np.full(m, rng.uniform(10, 30)))
        gain = db_to_amplitude(np.full(m, rng.uniform(-18, 6))) if c_gain[b] else None
        noise = snr = ir = None
        if c_noise[b]:
            idx = (ring_pos + np.arange(m * T)) % ring.size
            noise = ring[idx].reshape(m, T)
            ring_pos = (ring_pos + m * T) % ring.size
            snr = rng.uniform(-10, 15, m)
        if c_rev[b]:
            ir = np.asarray(irs[(batch0 + b) % len(irs)], np.float64)
        x[sl] = augment_batch(y, noise, snr, ir, gain=gain).astype(np.float32)
    for k, v in (("pitch", c_pitch), ("bandstop", c_bs), ("colored", c_col), ("gain", c_gain),
                 ("noise", c_noise), ("reverb", c_rev)):
        cnt[k + "_batches"] = int(v.sum())
    cnt["batches"] = nb
    return x, cnt
