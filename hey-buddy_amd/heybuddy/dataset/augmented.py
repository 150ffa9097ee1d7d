"""Batch augmentation on the device (replaces the noise-mix and reverb steps of
AugmentedAudioGenerator.execute_augment_batch, reference
src/python/heybuddy/dataset/augmented.py:297-394).

Semantics kept from the reference:
* one coin flip per BATCH for background noise (p 0.75, :383) and one for
  reverb (p 0.75, :387), from numpy's global RNG (drawn for all batches of a
  call at once: the coins are the same Bernoulli draws, the stream order differs);
* background noise: consecutive noise clips (cycling through the bank) are
  concatenated until they cover batch * T samples and cut into consecutive
  T-sample segments (:246-267); SNR ~ U[min, max] dB per clip (:269-270);
* reverb: ONE impulse response per batch, taken in order (:188-192);
* gain: torch_audiomentations Gain in per_batch mode (:116-120), one factor
  10^(g/20), g ~ U[-18, 6] dB, per batch with probability gain_prob (1.0),
  applied before the noise mix (it is the last transform of augment_batch);
* colored noise: torch_audiomentations AddColoredNoise in per_batch mode
  (:107-113), before the gain: per batch with probability colored_noise_prob
  (0.25) one snr ~ U[10, 30] dB and one f_decay ~ U[-1, 2]; torch_audiomentations
  runs a per_batch transform on the batch reshaped to (1, batch * channels, T)
  (BaseWaveformTransform.forward), so ONE parameter set and ONE noise vector
  serve the whole batch, scaled per clip by its own rms; the white noise comes
  from the kernel's counter-based normal stream (seeded from numpy's global RNG),
  one vector per batch;
* seven-band EQ: audiomentations SevenBandParametricEQ, per CLIP with
  probability seven_band_prob (0.25), gains ~ U[-6, 6] dB (:79-84): first in the
  per-clip Compose; the per-clip filter parameters (center mel-uniform in each
  band's range, gain, Q ~ U[0.5, 1.33]) are drawn here and turned into RBJ
  biquad coefficients (eq_coefficients), the cascade runs on the device;
* tanh distortion: audiomentations TanhDistortion, per CLIP with probability
  tanh_distortion_prob (0.25), amount ~ U[1e-4, 0.1] (:79-90), after the EQ: the
  reference applies both on the host before the batch chain (:325-328).
* band-stop: torch_audiomentations BandStopFilter in per_batch mode (:101-105),
  second in the batch chain (before the colored noise): per batch with
  probability band_stop_prob (0.25) one center frequency (mel-uniform in
  [200, 4000] Hz) and one bandwidth fraction (U[0.5, 1.99]); julius'
  windowed-sinc band-pass subtracted from each clip of the batch on the device
  (hbk_band_stop).
Differences (by design): the IR spectra are computed once for the whole bank
instead of once per batch, every batch of a call is one kernel launch, and
clips never leave the device (the reference copies each clip back to host,
:419).
* pitch shift: torch_audiomentations PitchShift in per_batch mode (:93-100),
  first in the batch chain: per batch with probability pitch_shift_prob (0.25)
  one of torch_pitch_shift's fast shifts within +-pitch_shift_semitones (at
  16 kHz and 3 semitones: 125/128 and 128/125), drawn uniformly; stft, phase
  vocoder, istft and the sinc resampler on the device (hbk_pitch_shift).
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Sequence

import os
import numpy as np
import torch

from heybuddy.constants import (DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB, DEFAULT_AUGMENT_BAND_STOP_PROB,
                                DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB, DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                                DEFAULT_AUGMENT_PITCH_SHIFT_PROB, DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
                                DEFAULT_AUGMENT_TANH_DISTORTION_PROB, DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                                DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB, DEFAULT_AUGMENT_GAIN_MAX_DB,
                                DEFAULT_AUGMENT_GAIN_MIN_DB, DEFAULT_AUGMENT_GAIN_PROB,
                                DEFAULT_AUGMENT_REVERB_PROB, DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                                DEFAULT_AUGMENT_SEVEN_BAND_PROB)
from heybuddy.kernels import ReverbPlan, pitch_shift, place_clips, seven_band_eq, tanh_distortion

__all__ = ["AugmentedAudioGenerator", "BatchAugmenter", "SourceOrder", "bandstop_cutoffs", "eq_coefficients",
           "eq_parameters", "hf_shuffle_permutation", "source_plan", "target_length_offset", "target_length_offsets",
           "to_target_length"]

T = 23040

# Random streams. numpy's global RNG carries exactly the draws the reference's
# own code makes from it, in its order: the leading silence of each placed clip
# (augmented.py:219-223), the re-shuffle of a dataset iterator when it runs out
# (augmented.py:148-162 -> datasets.Dataset.shuffle(), seeded from numpy's
# state), and the background-noise and reverb coins of every batch
# (augmented.py:370-392). The augmentation parameters come from torch's CPU
# generator (torch_audiomentations draws from torch; audiomentations from
# Python's random): with a seeded numpy the clip placement and dataset order
# equal the reference's for any augmentation probabilities.


def _u(shape, lo: float = 0.0, hi: float = 1.0) -> np.ndarray:
    """Uniform [lo, hi) float64 draws from torch's CPU generator."""
    return (torch.rand(shape, dtype=torch.float64) * (hi - lo) + lo).numpy()


def hf_shuffle_permutation(n: int) -> np.ndarray:
    """The permutation datasets.Dataset.shuffle() (no seed) applies: a seed
    taken from numpy's global state (key[pos]), one np.random.random() step,
    then default_rng(seed).permutation(n) (datasets 5.x arrow_dataset.shuffle)."""
    _, keys, pos, *_ = np.random.get_state()
    seed = keys[pos] if pos < 624 else keys[0]
    np.random.random()
    return np.random.default_rng(seed).permutation(n)


class SourceOrder:
    """The row order of AudioDatasetGenerator.get_next_dataset_value
    (augmented.py:148-162) over a dataset of n rows: in order first
    (shuffle_first=False), then a fresh shuffle() each time it runs out."""

    def __init__(self, n: int) -> None:
        if n <= 0:
            raise ValueError("source dataset is empty")
        self.n = int(n)
        self.perm = np.arange(self.n)
        self.pos = 0

    def take(self, m: int) -> np.ndarray:
        out = np.empty(int(m), dtype=np.int64)
        for i in range(int(m)):
            if self.pos == self.n:
                self.perm = hf_shuffle_permutation(self.n)
                self.pos = 0
            out[i] = self.perm[self.pos]
            self.pos += 1
        return out

# SevenBandParametricEQ: low shelf, five peaking filters, high shelf; center
# frequency ranges (Hz) and the Q range of audiomentations' documentation
EQ_BANDS = ((42.0, 95.0), (91.0, 204.0), (196.0, 441.0), (421.0, 948.0), (909.0, 2045.0),
            (1957.0, 4404.0), (4216.0, 9486.0))
EQ_Q_RANGE = (0.5, 1.33)


def eq_parameters(n: int, gain_db: float, sample_rate: int = 16000) -> np.ndarray:
    """(center Hz, gain dB, Q) [n, 7, 3] from torch's CPU generator: centers
    uniform on the mel scale within each band (the high shelf clamped to 0.95
    Nyquist), gains ~ U[-gain_db, gain_db], Q ~ U[0.5, 1.33]."""
    mel = lambda f: 2595.0 * np.log10(1.0 + np.asarray(f) / 700.0)  # noqa: E731
    lo, hi = mel([b[0] for b in EQ_BANDS]), mel([b[1] for b in EQ_BANDS])
    f0 = 700.0 * (10.0 ** ((lo + _u((n, 7)) * (hi - lo)) / 2595.0) - 1.0)
    f0[:, 6] = np.minimum(f0[:, 6], (sample_rate // 2) * 0.95)
    g = _u((n, 7), -gain_db, gain_db)
    q = _u((n, 7), *EQ_Q_RANGE)
    return np.stack([f0, g, q], axis=-1)


def eq_coefficients(params: np.ndarray, sample_rate: int = 16000) -> np.ndarray:
    """RBJ audio-EQ-cookbook biquads (b0, b1, b2, a1, a2) / a0, float64 [..., 7, 5]:
    filter 0 low shelf, 1-5 peaking, 6 high shelf; A = 10^(gain / 40),
    w0 = 2 pi f0 / sr, alpha = sin(w0) / (2 Q)."""
    p = np.asarray(params, dtype=np.float64)
    A = 10.0 ** (p[..., 1] / 40.0)
    w0 = 2.0 * np.pi * p[..., 0] / sample_rate
    c, al = np.cos(w0), np.sin(w0) / (2.0 * p[..., 2])
    r = 2.0 * np.sqrt(A) * al
    Ap, Am = A + 1.0, A - 1.0
    peak = (1 + al * A, -2 * c, 1 - al * A, 1 + al / A, -2 * c, 1 - al / A)
    low = (A * (Ap - Am * c + r), 2 * A * (Am - Ap * c), A * (Ap - Am * c - r),
           Ap + Am * c + r, -2 * (Am + Ap * c), Ap + Am * c - r)
    high = (A * (Ap + Am * c + r), -2 * A * (Am + Ap * c), A * (Ap + Am * c - r),
            Ap - Am * c + r, 2 * (Am - Ap * c), Ap - Am * c - r)
    kind = np.arange(7)
    b0, b1, b2, a0, a1, a2 = (np.where(kind == 0, lo_, np.where(kind == 6, hi_, pk_))
                              for lo_, hi_, pk_ in zip(low, high, peak))
    return np.stack([b0 / a0, b1 / a0, b2 / a0, a1 / a0, a2 / a0], axis=-1)


def bandstop_cutoffs(n: int, sample_rate: int = 16000):
    """n (cut_lo, cut_hi) pairs of torch_audiomentations BandStopFilter (float32
    fractions of the sample rate): center mel-uniform in [200, 4000] Hz (its
    convert_frequencies_to_mels: 2595 log10(1 + f / 700)), bandwidth fraction
    U[0.5, 1.99], cut = f_c (1 -+ bw / 2) / sr; torch's CPU generator."""
    def mel(f):
        return 2595.0 * np.log10(1.0 + f / 700.0)
    m = _u(n, mel(200.0), mel(4000.0)).astype(np.float32)
    fc = (np.float32(700.0) * (np.float32(10.0) ** (m / np.float32(2595.0)) - np.float32(1.0))).astype(np.float32)
    bw = _u(n, 0.5, 1.99).astype(np.float32)
    sr = np.float32(sample_rate)
    lo = (fc * (np.float32(1.0) - bw / np.float32(2.0)) / sr).astype(np.float32)
    hi = (fc * (np.float32(1.0) + bw / np.float32(2.0)) / sr).astype(np.float32)
    return lo, hi


def _pinned(t: torch.Tensor) -> torch.Tensor:
    """Page-locked copy for an asynchronous upload (as is on a GPU-less host)."""
    return t.pin_memory() if torch.cuda.is_available() else t


def fast_shifts(sample_rate: int = 16000, semitones: float = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES) -> list:
    """torch_pitch_shift.get_fast_shifts as torch_audiomentations PitchShift
    calls it: every ratio i / j (i, j products of sample_rate's prime factors)
    in [2^(-semitones/12), 2^(semitones/12)] except 1, ascending."""
    from fractions import Fraction
    from itertools import combinations
    from math import prod
    fac, n, d = [], int(sample_rate), 2
    while n > 1:
        while n % d == 0:
            fac.append(d)
            n //= d
        d += 1
    products = {prod(c) for r in range(1, len(fac) + 1) for c in combinations(fac, r)}
    lo, hi = Fraction(2.0 ** (-semitones / 12.0)), Fraction(2.0 ** (semitones / 12.0))
    return sorted({Fraction(i, j) for i in products for j in products if lo <= Fraction(i, j) <= hi} - {1})


class BatchAugmenter:
    def __init__(self, noise: Optional[Sequence[torch.Tensor]] = None,
                 impulse_responses: Optional[Sequence[torch.Tensor]] = None,
                 device: Optional[torch.device] = None, batch_size: int = 128,
                 background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                 background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                 background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                 reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB,
                 gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
                 min_gain_in_db: float = DEFAULT_AUGMENT_GAIN_MIN_DB,
                 max_gain_in_db: float = DEFAULT_AUGMENT_GAIN_MAX_DB,
                 colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                 colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
                 colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                 colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                 colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                 tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
                 tanh_min_distortion: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                 tanh_max_distortion: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                 seven_band_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
                 seven_band_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                 band_stop_prob: float = DEFAULT_AUGMENT_BAND_STOP_PROB,
                 sample_rate: int = 16000,
                 pitch_shift_prob: float = DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
                 pitch_shift_semitones: float = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES) -> None:
        self.plan = ReverbPlan(device)
        self.device = self.plan.device
        if background_noise_prob > 0 and not noise:
            raise ValueError("Background noise is enabled but no augmentation dataset is provided")
        if reverb_prob > 0 and not impulse_responses:
            raise ValueError("Reverb is enabled but no impulse response dataset is provided")
        self.batch_size = int(batch_size)
        self.p_noise = float(background_noise_prob)
        self.p_reverb = float(reverb_prob)
        self.snr_min = float(background_noise_min_snr_db)
        self.snr_max = float(background_noise_max_snr_db)
        self.p_gain = float(gain_prob)
        self.gain_min_db = float(min_gain_in_db)
        self.gain_max_db = float(max_gain_in_db)
        self.p_colored = float(colored_noise_prob)
        self.colored_snr = (float(colored_noise_min_snr_db), float(colored_noise_max_snr_db))
        self.colored_decay = (float(colored_noise_min_f_decay), float(colored_noise_max_f_decay))
        self.sample_rate = int(sample_rate)
        self.p_tanh = float(tanh_distortion_prob)
        self.tanh_range = (float(tanh_min_distortion), float(tanh_max_distortion))
        self.p_eq = float(seven_band_prob)
        self.eq_gain_db = float(seven_band_gain_db)
        self.p_bandstop = float(band_stop_prob)
        self.p_pitch = float(pitch_shift_prob)
        self.pitch_shifts = fast_shifts(self.sample_rate, pitch_shift_semitones) if self.p_pitch > 0 else []
        if self.p_pitch > 0 and not self.pitch_shifts:
            raise ValueError(f"no fast pitch shift within +-{pitch_shift_semitones} semitones at {sample_rate} Hz")
        self.ring = None
        self.lengths: List[int] = []
        self.starts: List[int] = []
        if noise:
            parts = [n.reshape(-1).to(self.device, torch.float32) for n in noise]
            self.ring = torch.cat(parts)
            self.lengths = [p.numel() for p in parts]
            self.starts = list(np.cumsum([0] + self.lengths[:-1]))
        self.spectra = None
        if impulse_responses:
            ks = torch.stack([ReverbPlan.rotated_kernel(ir.to(self.device), T) for ir in impulse_responses])
            self.spectra = self.plan.spectra(ks)
        self.noise_idx = 0
        self.ir_idx = 0
        self._advance = {}
        # a list: __call__ appends (sub-stage, start event, end event) per stage it
        # launches (timing events on the current stream; bench.py's per-kernel rooflines)
        self.timing: Optional[list] = None

    def _tick(self, name: str, start: Optional[Any]) -> Optional[Any]:
        """Close the sub-stage started by ``start`` (an event or None) as
        ``name`` and open the next one; no-op unless self.timing is a list."""
        if self.timing is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if start is not None and name:
            self.timing.append((name, start, ev))
        return ev

    def _noise_advance(self, idx: int, nb: int) -> int:
        """Index of the noise clip after a batch of nb clips starting at clip idx:
        whole clips are consumed until they cover nb * T samples
        (augmented.py:249-254). Memoised: full batches repeat the same few."""
        key = (idx, nb)
        nxt = self._advance.get(key)
        if nxt is None:
            need, covered, nxt = nb * T, 0, idx
            while covered < need:
                covered += self.lengths[nxt]
                nxt = (nxt + 1) % len(self.lengths)
            self._advance[key] = nxt
        return nxt

    def plan_batches(self, n: int, coins: Optional[np.ndarray] = None):
        """Per-clip noise offsets, spectrum indices and gains (dB) for n clips
        (host bookkeeping that mirrors the reference's dataset iteration).
        coins [nbat, 2]: each batch's background-noise and reverb draws from
        numpy's global RNG (augmented.py:370-392; AugmentedAudioGenerator
        interleaves them with the batches' placement draws, as the reference
        does); drawn here, batch by batch, when not given. Every other draw
        comes from torch's CPU generator, only for augmentations whose
        probability is non-zero."""
        bs = self.batch_size
        nbat = (n + bs - 1) // bs
        sizes = np.full(nbat, bs, dtype=np.int64)
        sizes[-1] = n - bs * (nbat - 1)
        batch = np.repeat(np.arange(nbat), sizes)  # batch of each clip
        pos = np.arange(n) - batch * bs            # position within its batch
        if coins is None:
            coins = np.random.rand(nbat, 2)
        coins = np.asarray(coins, dtype=np.float64).reshape(nbat, 2)
        # gain (torch_audiomentations Gain, per_batch): one value per batch
        gain_db = np.zeros(n, dtype=np.float32)
        if self.p_gain > 0:
            g_on = _u(nbat) < self.p_gain
            g_db = _u(nbat, self.gain_min_db, self.gain_max_db)
            gain_db = np.where(g_on, g_db, 0.0).astype(np.float32)[batch]
        # colored noise (AddColoredNoise, per_batch): one (snr, f_decay) per batch; NaN snr = off
        colored_snr = np.full(n, np.nan, dtype=np.float32)
        colored_fd = np.zeros(n, dtype=np.float32)
        if self.p_colored > 0:
            c_on = _u(nbat) < self.p_colored
            c_snr = _u(nbat, *self.colored_snr)
            c_fd = _u(nbat, *self.colored_decay)
            colored_snr = np.where(c_on, c_snr, np.nan).astype(np.float32)[batch]
            colored_fd = c_fd.astype(np.float32)[batch]
        # background noise: consecutive T-sample segments of the noise stream
        noise_off = np.full(n, -1, dtype=np.int64)
        n_on = (coins[:, 0] < self.p_noise) if self.ring is not None else np.zeros(nbat, bool)
        if n_on.any():
            start = np.full(nbat, -1, dtype=np.int64)
            for b in np.flatnonzero(n_on):
                start[b] = self.starts[self.noise_idx]
                self.noise_idx = self._noise_advance(self.noise_idx, int(sizes[b]))
            sel = start[batch] >= 0
            noise_off[sel] = start[batch][sel] + pos[sel] * T
        # reverb: one IR per batch, taken in order (augmented.py:188-192)
        spec_idx = np.full(n, -1, dtype=np.int32)
        r_on = (coins[:, 1] < self.p_reverb) if self.spectra is not None else np.zeros(nbat, bool)
        if r_on.any():
            n_spec = self.spectra.shape[0]
            ir = (self.ir_idx + np.cumsum(r_on) - 1) % n_spec
            self.ir_idx = int((self.ir_idx + r_on.sum()) % n_spec)
            per_clip = np.where(r_on, ir, -1).astype(np.int32)[batch]
            spec_idx[:] = per_clip
        self._colored = (colored_snr, colored_fd)
        # band-stop (BandStopFilter, per_batch): one (center, bandwidth) per batch
        # whose coin came up; the filtered clips and their cutoffs
        p_bs = getattr(self, "p_bandstop", 0.0)
        b_on = (_u(nbat) < p_bs) if p_bs > 0 else np.zeros(nbat, bool)
        lo, hi = bandstop_cutoffs(int(b_on.sum()), getattr(self, "sample_rate", 16000))
        sel = b_on[batch]
        per = np.full(nbat, -1, dtype=np.int64)
        per[b_on] = np.arange(int(b_on.sum()))
        self._bandstop = (np.flatnonzero(sel).astype(np.int32), lo[per[batch][sel]], hi[per[batch][sel]])
        # pitch shift (PitchShift, per_batch): one fast shift per batch whose coin
        # came up (random.choices over the shifts); the clips of each shift
        self._pitch = []
        if getattr(self, "p_pitch", 0.0) > 0:
            p_on = _u(nbat) < self.p_pitch
            p_pick = torch.randint(0, len(self.pitch_shifts), (nbat,)).numpy()
            for j, f in enumerate(self.pitch_shifts):
                clips = np.flatnonzero((p_on & (p_pick == j))[batch]).astype(np.int32)
                if clips.size:
                    self._pitch.append((f.numerator, f.denominator, clips))
        # seven-band EQ (audiomentations, per clip): the clips whose coin came up
        # and their filters (parameters drawn for those clips only)
        p_eq = getattr(self, "p_eq", 0.0)
        e_on = (_u(n) < p_eq) if p_eq > 0 else np.zeros(n, bool)
        sr = getattr(self, "sample_rate", 16000)
        eq_idx = np.nonzero(e_on)[0].astype(np.int32)
        self._eq = (eq_idx, eq_coefficients(eq_parameters(eq_idx.size, getattr(self, "eq_gain_db", 0.0), sr), sr))
        # tanh distortion (audiomentations, per clip): NaN amount = off
        p_tanh = getattr(self, "p_tanh", 0.0)
        self._tanh = np.full(n, np.nan, dtype=np.float32)
        if p_tanh > 0:
            t_on = _u(n) < p_tanh
            t_amt = _u(n, *getattr(self, "tanh_range", (0.0, 0.0)))
            self._tanh = np.where(t_on, t_amt, np.nan).astype(np.float32)
        return noise_off, spec_idx, gain_db

    def prepare(self, n: int, coins: Optional[np.ndarray] = None) -> Dict[str, Any]:
        """Every host-side draw of one call over n clips (plan_batches, the
        background SNRs, the colored-noise seed) in the order __call__ makes
        them, with the EQ filters already in pinned memory: a pipelined caller
        prepares chunk s + 1 while the device works, then launches."""
        noise_off, spec_idx, gain_db = self.plan_batches(n, coins)
        ring_len = 0 if self.ring is None else self.ring.numel()
        if ring_len:
            noise_off = np.where(noise_off >= 0, noise_off % ring_len, -1)
        snr = torch.zeros(n, dtype=torch.float32)
        if (noise_off >= 0).any():  # torchaudio add_noise's snr: torch.rand in the reference (:271-272)
            snr = torch.from_numpy(_u(n, self.snr_min, self.snr_max).astype(np.float32))
        gain = None
        if self.p_gain > 0:  # torch_audiomentations convert_decibels_to_amplitude_ratio
            gain = torch.pow(10.0, torch.from_numpy(gain_db) / 20.0)
        eq_idx, eq_coef = self._eq
        eq = None
        if eq_idx.size:
            eq = (_pinned(torch.from_numpy(eq_coef)), _pinned(torch.from_numpy(eq_idx)))
        tanh = None if np.isnan(self._tanh).all() else torch.from_numpy(self._tanh)
        bs_idx, bs_lo, bs_hi = self._bandstop
        bandstop = None
        if bs_idx.size:
            bandstop = (torch.from_numpy(bs_idx), torch.from_numpy(bs_lo), torch.from_numpy(bs_hi))
        colored_snr, colored_fd = self._colored
        colored = None
        if not np.isnan(colored_snr).all():
            colored = (torch.from_numpy(colored_fd), torch.from_numpy(colored_snr),
                       int(torch.randint(0, 2 ** 62, (1,)).item()))
        return {"n": n, "noise_off": torch.from_numpy(noise_off), "spec_idx": torch.from_numpy(spec_idx),
                "snr": snr, "gain": gain, "eq": eq, "tanh": tanh, "bandstop": bandstop, "colored": colored,
                "pitch": [(a, b, _pinned(torch.from_numpy(c))) for a, b, c in getattr(self, "_pitch", [])]}

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                 prepared: Optional[Dict[str, Any]] = None) -> torch.Tensor:
        """x [n, >= 23040] f32 on the device -> augmented [n, 23040]."""
        n = x.shape[0]
        pr = self.prepare(n) if prepared is None else prepared
        if pr["n"] != n:
            raise ValueError(f"prepared for {pr['n']} clips, called with {n}")
        ev = self._tick("", None)
        if pr["eq"] is not None:  # per-clip Compose: EQ, then tanh (augmented.py:79-90), in place on out
            if out is None:
                out = torch.empty((n, T), dtype=torch.float32, device=x.device)
            if out.data_ptr() != x.data_ptr():
                out.copy_(x[:, :T])
            x = seven_band_eq(out, pr["eq"][0], idx=pr["eq"][1])
            ev = self._tick("eq", ev)
        if pr["tanh"] is not None:  # per-clip Compose, before the batch chain (augmented.py:325-328)
            x = tanh_distortion(x, pr["tanh"], out=out)
            out = x
            ev = self._tick("tanh", ev)
        for num, den, clips in pr.get("pitch") or []:  # batch chain: pitch shift first (augmented.py:93-100)
            if out is None:
                out = torch.empty((n, T), dtype=torch.float32, device=x.device)
            x = pitch_shift(x, clips, num, den, out=out, sample_rate=self.sample_rate)
            ev = self._tick("pitch", ev)
        if pr.get("bandstop") is not None:  # then band-stop, then colored noise (augmented.py:101-113)
            if out is None:
                out = x[:, :T].clone()
            elif out.data_ptr() != x.data_ptr():
                out.copy_(x[:, :T])
            x = self.plan.band_stop(out, *pr["bandstop"], out=out)
            ev = self._tick("bandstop", ev)
        colored = None
        if pr["colored"] is not None:  # colored noise precedes the gain (augmented.py:107-118)
            fd, csnr, seed = pr["colored"]
            if self.sample_rate == 16000 and os.environ.get("HBK_AUG_COLORED_FOLD", "1") != "0":
                colored = (fd, csnr, seed, self.batch_size)  # mixed in augment_kernel's pass
            else:
                x = self.plan.colored_noise(x, fd, csnr, seed=seed, out=out, sample_rate=self.sample_rate,
                                            clips_per_noise=self.batch_size)
                out = x
                ev = self._tick("colored", ev)
        y = self.plan.augment(x, self.ring, pr["noise_off"], pr["snr"], self.spectra, pr["spec_idx"],
                              out=out, gain=pr["gain"], colored=colored)
        self._tick("mix_reverb", ev)
        return y


# ---------------------------------------------------------------------------
# AugmentedAudioGenerator: the reference's class surface (augmented.py:16-427)
# over the device chain above.
# ---------------------------------------------------------------------------
def source_plan(source_lengths: Sequence[int], num_samples: int, batch_size: int, target_num_samples: int):
    """numpy's draws when an AugmentedAudioGenerator built over a source
    dataset of len(source_lengths) rows yields num_samples clips (the
    reference builds a new one per TrainingFeaturesGenerator.generate call,
    features.py:434-440): per batch of batch_size, the rows (a fresh
    SourceOrder: in order, re-shuffled when it runs out), each padded clip's
    leading silence (to_target_length), then the background-noise and reverb
    coins (augmented.py:396-427 -> :297-394). Returns (rows [num_samples],
    leading silence [num_samples], coins [nbat, 2])."""
    src = np.asarray(source_lengths, dtype=np.int64)
    order = SourceOrder(src.shape[0])
    rows, pres, coins = [], [], []
    for b0 in range(0, int(num_samples), int(batch_size)):
        r = order.take(min(int(batch_size), int(num_samples) - b0))
        rows.append(r)
        pres.append(target_length_offsets(src[r], target_num_samples))
        coins.append(np.random.rand(2))
    if not rows:
        return np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros((0, 2))
    return (np.concatenate(rows), np.concatenate(pres).astype(np.int32),
            np.array(coins, dtype=np.float64).reshape(-1, 2))


def target_length_offset(num_samples: int, target_num_samples: int) -> int:
    """Leading zeros to_target_length puts in front of a clip of num_samples
    (augmented.py:210-226): 0 when it is cropped or when exactly one sample is
    missing, else np.random.randint(int(S/4), int(3S/4)) from numpy's global
    RNG, S = target - num_samples (one draw per padded clip, in clip order)."""
    total = target_num_samples - num_samples
    if total <= 1:
        return 0
    return int(np.random.randint(int(total / 4), int(3 * total / 4)))


def target_length_offsets(lengths: Sequence[int], target_num_samples: int) -> np.ndarray:
    """target_length_offset for a whole batch in one vectorised draw: numpy's
    legacy randint with array bounds produces the same values, in clip order,
    and leaves the RNG in the same state as one scalar draw per padded clip."""
    lengths = np.asarray(lengths, dtype=np.int64)
    total = target_num_samples - lengths
    pre = np.zeros(lengths.shape[0], dtype=np.int32)
    pad = total > 1
    if pad.any():
        t = total[pad]
        pre[pad] = np.random.randint((t / 4).astype(np.int64), (3 * t / 4).astype(np.int64))
    return pre


def to_target_length(audio: np.ndarray, target_num_samples: int) -> np.ndarray:
    """Host form of AugmentedAudioGenerator.to_target_length
    (augmented.py:200-232): int16 -> /32768, crop to the target, or pad with
    random leading silence (float32 out)."""
    if audio.dtype == np.int16:
        audio = audio.astype(np.float32) / 32768.0
    n = audio.shape[0]
    if n >= target_num_samples:
        return audio[:target_num_samples]
    pre = target_length_offset(n, target_num_samples)
    out = np.zeros(target_num_samples, dtype=np.float32)
    out[pre:pre + n] = audio
    return out


def _audio_arrays(dataset: Any) -> List[Dict[str, Any]]:
    """Rows of an audio dataset as {"array", "sampling_rate"} dicts: an HF
    ``datasets.Dataset`` with an "audio" column, a list of such rows, a list of
    {"array", ...} dicts, or plain arrays / tensors (16 kHz)."""
    out = []
    for row in dataset:
        if isinstance(row, dict) and "audio" in row:
            row = row["audio"]
        if isinstance(row, dict):
            out.append({"array": row["array"], "sampling_rate": int(row.get("sampling_rate", 16000))})
        else:
            out.append({"array": row, "sampling_rate": 16000})
    return out


def _as_float_array(a: Any) -> np.ndarray:
    if torch.is_tensor(a):
        a = a.detach().cpu().numpy()
    a = np.asarray(a)
    if a.dtype == np.int16:
        return a.astype(np.float32) / 32768.0
    return a.astype(np.float32, copy=False)


class AugmentedAudioGenerator:
    """Drop-in for heybuddy.dataset.augmented.AugmentedAudioGenerator
    (augmented.py:16-427). Same constructor and methods; every batch runs on
    the MI355X: clip placement (hbk_place_clips), seven-band EQ, tanh
    distortion, colored noise, gain, background noise and reverb (hbk_*), in
    the reference's order (:297-394). The datasets are any iterable of audio
    rows (see _audio_arrays); clips at another rate are resampled (torchaudio's
    band-limited resampler, restated). The noise and IR sets are loaded into
    HBM once. Every augmentation of the reference's chain runs on the device."""

    def __init__(self, source_dataset: Any, device_id: Optional[int] = None,
                 augmentation_dataset: Any = None, impulse_response_dataset: Any = None,
                 target_length: float = 1.44, sample_rate: int = 16000, batch_size: int = 128,
                 seven_band_aug_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
                 seven_band_aug_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                 tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
                 tanh_min_distortion: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                 tanh_max_distortion: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                 pitch_shift_prob: float = 0.25, pitch_shift_semitones: int = 3,
                 band_stop_prob: float = 0.25,
                 colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                 colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
                 colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                 colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                 colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                 background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                 background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                 background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                 gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
                 reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB) -> None:
        if background_noise_prob > 0 and not augmentation_dataset:
            raise ValueError("Background noise is enabled but no augmentation dataset is provided")
        if reverb_prob > 0 and not impulse_response_dataset:
            raise ValueError("Reverb is enabled but no impulse response dataset is provided")
        self.device_id = device_id
        self.source_dataset = source_dataset
        self.augmentation_dataset = augmentation_dataset
        self.impulse_response_dataset = impulse_response_dataset
        self.target_length = target_length
        self.sample_rate = int(sample_rate)
        self.batch_size = int(batch_size)
        self.reverb_prob = reverb_prob
        self.background_noise_prob = background_noise_prob
        self.background_noise_min_snr_db = background_noise_min_snr_db
        self.background_noise_max_snr_db = background_noise_max_snr_db
        dev = None if device_id is None else torch.device("cuda", device_id)

        def bank(ds):
            if not ds:
                return None
            from heybuddy.util import resample
            rows = _audio_arrays(ds)
            return [resample(torch.from_numpy(_as_float_array(r["array"]).reshape(-1)), int(r["sampling_rate"]),
                             self.sample_rate) for r in rows]

        self.augmenter = BatchAugmenter(
            bank(augmentation_dataset), bank(impulse_response_dataset), device=dev,
            batch_size=self.batch_size, background_noise_prob=background_noise_prob,
            background_noise_min_snr_db=background_noise_min_snr_db,
            background_noise_max_snr_db=background_noise_max_snr_db, reverb_prob=reverb_prob,
            gain_prob=gain_prob, colored_noise_prob=colored_noise_prob,
            colored_noise_min_snr_db=colored_noise_min_snr_db, colored_noise_max_snr_db=colored_noise_max_snr_db,
            colored_noise_min_f_decay=colored_noise_min_f_decay, colored_noise_max_f_decay=colored_noise_max_f_decay,
            tanh_distortion_prob=tanh_distortion_prob, tanh_min_distortion=tanh_min_distortion,
            tanh_max_distortion=tanh_max_distortion, seven_band_prob=seven_band_aug_prob,
            seven_band_gain_db=seven_band_aug_gain_db, band_stop_prob=band_stop_prob, sample_rate=self.sample_rate,
            pitch_shift_prob=pitch_shift_prob, pitch_shift_semitones=pitch_shift_semitones)
        self.device = self.augmenter.device
        self._source: Optional[List[Dict[str, Any]]] = None
        self._order: Optional[SourceOrder] = None

    @property
    def target_num_samples(self) -> int:
        """augmented.py:123-128."""
        return int(self.target_length * self.sample_rate)

    def to_target_length(self, audio: np.ndarray) -> np.ndarray:
        return to_target_length(np.asarray(audio), self.target_num_samples)

    def to_audio_array(self, audio: Any) -> np.ndarray:
        """augmented.py:278-295: lists become float32 (float items) or int16."""
        if isinstance(audio, list):
            if not audio:
                raise ValueError("Audio list is empty")
            first = audio[0][0] if isinstance(audio[0], list) else audio[0]
            return np.array(audio, dtype=np.float32 if isinstance(first, float) else np.int16)
        return audio

    def get_next_audio_sample_dict(self) -> Dict[str, Any]:
        """The next source row: in order, then re-shuffled each time the
        dataset runs out (augmented.py:148-186; SourceOrder)."""
        if self._source is None:
            self._source = list(self.source_dataset)
            self._order = SourceOrder(len(self._source))
        row = self._source[int(self._order.take(1)[0])]
        return row if isinstance(row, dict) and "audio" in row else {"audio": _audio_arrays([row])[0]}

    def place_batch(self, batch: Sequence[Any]) -> torch.Tensor:
        """The per-clip placement of execute_augment_batch (:314-328) for a
        batch of audio rows: one device launch; the leading-silence draws come
        from numpy's global RNG in clip order, as to_target_length draws them.
        Clips at another rate are resampled first (util.resample; the reference
        resamples them in a second pass, :330-360, so in a mixed-rate batch its
        draws come in a different order)."""
        from heybuddy.util import resample
        T = self.target_num_samples
        arrays = []
        for audio in batch:
            a = audio["array"] if isinstance(audio, dict) else audio
            sr = audio.get("sampling_rate", self.sample_rate) if isinstance(audio, dict) else self.sample_rate
            a = _as_float_array(self.to_audio_array(a)).reshape(-1)
            if sr != self.sample_rate:
                a = resample(torch.from_numpy(a), int(sr), self.sample_rate).numpy()
            arrays.append(a)
        lens = np.array([a.shape[0] for a in arrays], dtype=np.int32)
        pre = target_length_offsets(lens, T)
        width = max(int(lens.max()), 1)
        host = torch.zeros((len(arrays), width), dtype=torch.float32).pin_memory()
        for i, a in enumerate(arrays):
            host[i, :a.shape[0]] = torch.from_numpy(a)
        return place_batch_device(host.to(self.device, non_blocking=True), lens, pre, T)

    def execute_augment_batch(self, batch: Sequence[Any]) -> torch.Tensor:
        """augmented.py:297-394 on the device: placement, then the batch chain
        (in place on the placed batch)."""
        placed = self.place_batch(batch)
        return self.augmenter(placed, out=placed)

    def plan_batches(self, lens: Sequence[int]):
        """numpy's draws for consecutive batches of batch_size clips of the
        given lengths, in the reference's order (augmented.py:396-427 ->
        :297-394): per batch, each padded clip's leading silence, then the
        background-noise and reverb coins. Returns (leading silence per clip,
        coins [nbat, 2])."""
        lens = np.asarray(lens, dtype=np.int64)
        pres, coins = [], []
        for b0 in range(0, lens.shape[0], self.batch_size):
            pres.append(target_length_offsets(lens[b0:b0 + self.batch_size], self.target_num_samples))
            coins.append(np.random.rand(2))
        pre = np.concatenate(pres).astype(np.int32) if pres else np.zeros(0, np.int32)
        return pre, np.array(coins, dtype=np.float64).reshape(-1, 2)

    def plan_source(self, source_lengths: Sequence[int], num_samples: int):
        """source_plan with this generator's batch size and target length."""
        return source_plan(source_lengths, num_samples, self.batch_size, self.target_num_samples)

    def prepare_device(self, clips: torch.Tensor, lengths: Optional[Sequence[int]] = None) -> Dict[str, Any]:
        """The host-side draws of one augment_device call (per batch: the
        placement offsets, then the two coins; then BatchAugmenter.prepare's
        torch draws), so that a pipelined caller can make them ahead of the
        launch."""
        n = clips.shape[0]
        lens = np.full(n, clips.shape[1], dtype=np.int32) if lengths is None else np.asarray(lengths, np.int32)
        pre, coins = self.plan_batches(lens)
        return {"lens": lens, "pre": pre, "chain": self.augmenter.prepare(n, coins)}

    def augment_device(self, clips: torch.Tensor, lengths: Optional[Sequence[int]] = None,
                       prepared: Optional[Dict[str, Any]] = None) -> torch.Tensor:
        """Device-resident form used by the feature generator: clips [n, S] f32
        on the device (clip i valid in [0, lengths[i])) -> augmented [n, T]."""
        pr = self.prepare_device(clips, lengths) if prepared is None else prepared
        placed = place_clips(clips, pr["lens"], pr["pre"], self.target_num_samples)  # the chain runs in place
        return self.augmenter(placed, out=placed, prepared=pr["chain"])

    def __call__(self, num_samples: int, **kwargs: Any) -> Iterator[Dict[str, Any]]:
        """augmented.py:396-427: yields {"audio": {"array", "sampling_rate"}, ...}."""
        total_batches = int(np.ceil(num_samples / self.batch_size))
        for i in range(total_batches):
            nb = min(self.batch_size, num_samples - i * self.batch_size)
            items = [self.get_next_audio_sample_dict() for _ in range(nb)]
            out = self.execute_augment_batch([it["audio"] for it in items]).cpu().numpy()
            for audio, item in zip(out, items):
                yield {"audio": {"array": audio, "sampling_rate": self.sample_rate},
                       **{k: v for k, v in item.items() if k != "audio"}}


def place_batch_device(src: torch.Tensor, lengths: np.ndarray, pre: np.ndarray, T: int) -> torch.Tensor:
    """[n, S] -> [n, T] placement (hbk_place_clips), or a no-op view when every
    clip is cropped at 0 and already long enough."""
    if not pre.any() and src.shape[1] >= T and (lengths >= T).all():
        return src[:, :T]
    return place_clips(src, lengths, pre, T)
