"""Batch augmentation on the device (replaces the noise-mix and reverb steps of
AugmentedAudioGenerator.execute_augment_batch, reference
src/python/heybuddy/dataset/augmented.py:297-394).

Semantics kept from the reference:
* one coin flip per BATCH for background noise (p 0.75, :383) and then one for
  reverb (p 0.75, :387), drawn with numpy's global RNG in that order;
* background noise: consecutive noise clips (cycling through the bank) are
  concatenated until they cover batch * T samples and cut into consecutive
  T-sample segments (:246-267); SNR ~ U[min, max] dB per clip (:269-270);
* reverb: ONE impulse response per batch, taken in order (:188-192);
* gain: torch_audiomentations Gain in per_batch mode (:116-120), one factor
  10^(g/20), g ~ U[-18, 6] dB, per batch with probability gain_prob (1.0),
  applied before the noise mix (it is the last transform of augment_batch).
Differences (by design): the IR spectra are computed once for the whole bank
instead of once per batch, every batch of a call is one kernel launch, and
clips never leave the device (the reference copies each clip back to host,
:419). The other augmentations (7-band EQ, tanh distortion, pitch shift,
band-stop, colored noise) are not on this path yet.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from heybuddy.constants import (DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB, DEFAULT_AUGMENT_GAIN_MAX_DB,
                                DEFAULT_AUGMENT_GAIN_MIN_DB, DEFAULT_AUGMENT_GAIN_PROB,
                                DEFAULT_AUGMENT_REVERB_PROB)
from heybuddy.kernels import ReverbPlan

__all__ = ["BatchAugmenter"]

T = 23040


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
                 max_gain_in_db: float = DEFAULT_AUGMENT_GAIN_MAX_DB) -> None:
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

    def plan_batches(self, n: int):
        """Per-clip noise offsets, spectrum indices and gains (dB) for n clips
        (host bookkeeping that mirrors the reference's dataset iteration)."""
        noise_off = np.full(n, -1, dtype=np.int64)
        spec_idx = np.full(n, -1, dtype=np.int32)
        gain_db = np.zeros(n, dtype=np.float32)
        for b0 in range(0, n, self.batch_size):
            nb = min(self.batch_size, n - b0)
            if np.random.rand() < self.p_gain:  # per_batch: one gain for the batch
                gain_db[b0:b0 + nb] = np.random.uniform(self.gain_min_db, self.gain_max_db)
            if np.random.rand() < self.p_noise and self.ring is not None:
                noise_off[b0:b0 + nb] = self.starts[self.noise_idx] + np.arange(nb) * T
                covered = 0
                while covered < nb * T:  # whole clips are consumed (augmented.py:249-254)
                    covered += self.lengths[self.noise_idx]
                    self.noise_idx = (self.noise_idx + 1) % len(self.lengths)
            if np.random.rand() < self.p_reverb and self.spectra is not None:
                spec_idx[b0:b0 + nb] = self.ir_idx
                self.ir_idx = (self.ir_idx + 1) % self.spectra.shape[0]
        return noise_off, spec_idx, gain_db

    def __call__(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [n, >= 23040] f32 on the device -> augmented [n, 23040]."""
        n = x.shape[0]
        noise_off, spec_idx, gain_db = self.plan_batches(n)
        ring_len = 0 if self.ring is None else self.ring.numel()
        if ring_len:
            noise_off = np.where(noise_off >= 0, noise_off % ring_len, -1)
        snr = torch.rand(n, device=self.device) * (self.snr_max - self.snr_min) + self.snr_min
        gain = None
        if self.p_gain > 0:  # torch_audiomentations convert_decibels_to_amplitude_ratio
            gain = torch.pow(10.0, torch.from_numpy(gain_db) / 20.0)
        return self.plan.augment(x, self.ring, torch.from_numpy(noise_off), snr, self.spectra,
                                 torch.from_numpy(spec_idx), out=out, gain=gain)
