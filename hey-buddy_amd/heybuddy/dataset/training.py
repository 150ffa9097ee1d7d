"""Training batch composition on the device (replaces the threaded batch
assembly of TrainingDatasetIterator, reference
src/python/heybuddy/dataset/training.py:29-277).

A batch is [positives | negatives...] in list order with labels 1 / 0
(_generate_batches, :245-277); the default mix is positives 50, adversarial
50 (label 0), large negatives int(1000 * 2/3), medium negatives the rest
(default(), :280-469). ``multiply_batch_size`` halves every share between
stages with max(1, int(n * r)) (:215-231). Each pool is an HBM-resident
embedding table ([N, 16, 96], f16 or f32) read in a per-pass random
permutation with wrap-around (PrecalculatedDatasetIterator.take,
precalculated.py:501-536) — sampled by index on the device, so there are no
host threads, no queue and no H2D copy per step.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

__all__ = ["DevicePool", "TrainingDatasetIterator", "WakeWordTrainingDatasetIterator"]


class DevicePool:
    def __init__(self, data: torch.Tensor, generator: Optional[torch.Generator] = None) -> None:
        self.data = data
        self.n = data.shape[0]
        self.gen = generator
        self.perm = self._perm()
        self.pos = 0
        self.total_taken = 0

    def _perm(self) -> torch.Tensor:
        return torch.randperm(self.n, device=self.data.device, generator=self.gen)

    def __len__(self) -> int:
        return self.n

    def take_indices(self, k: int) -> torch.Tensor:
        out = []
        while k > 0:
            m = min(k, self.n - self.pos)
            out.append(self.perm[self.pos:self.pos + m])
            self.pos += m
            k -= m
            self.total_taken += m
            if self.pos >= self.n:
                self.perm = self._perm()
                self.pos = 0
        return torch.cat(out)

    def take(self, k: int) -> torch.Tensor:
        return self.data.index_select(0, self.take_indices(k))


class TrainingDatasetIterator:
    def __init__(self, positive: Sequence[Tuple[DevicePool, int]], negative: Sequence[Tuple[DevicePool, int]],
                 **kwargs) -> None:
        self.positive: List[Tuple[DevicePool, int]] = list(positive)
        self.negative: List[Tuple[DevicePool, int]] = list(negative)
        self.started = False
        self.total_yielded_samples = 0

    def start(self) -> None:
        self.started = True

    def stop(self) -> None:
        self.started = False

    def multiply_batch_size(self, ratio: float) -> None:
        self.positive = [(d, max(1, int(n * ratio))) for d, n in self.positive]
        self.negative = [(d, max(1, int(n * ratio))) for d, n in self.negative]

    @property
    def batch_size(self) -> int:
        return sum(n for _, n in self.positive) + sum(n for _, n in self.negative)

    def next_batch(self) -> Tuple[torch.Tensor, torch.Tensor]:
        xs, ys = [], []
        for pool, n in self.positive:
            xs.append(pool.take(n))
            ys.append(torch.ones(n, dtype=torch.int64, device=pool.data.device))
        for pool, n in self.negative:
            xs.append(pool.take(n))
            ys.append(torch.zeros(n, dtype=torch.int64, device=pool.data.device))
        x = torch.cat([t.to(torch.float32) for t in xs])
        self.total_yielded_samples += x.shape[0]
        return x, torch.cat(ys)

    def __iter__(self):
        while True:
            yield self.next_batch()


class WakeWordTrainingDatasetIterator(TrainingDatasetIterator):
    @classmethod
    def default(cls, positive: torch.Tensor, adversarial: Optional[torch.Tensor] = None,
                large: Optional[torch.Tensor] = None, medium: Optional[torch.Tensor] = None,
                positive_per_batch: int = 50, adversarial_per_batch: int = 50,
                negative_per_batch: int = 1000, generator: Optional[torch.Generator] = None
                ) -> "WakeWordTrainingDatasetIterator":
        """training.py:280-469 with device tensors in place of the hosted datasets."""
        pos = [(DevicePool(positive, generator), positive_per_batch)]
        neg: List[Tuple[DevicePool, int]] = []
        if adversarial is not None:
            neg.append((DevicePool(adversarial, generator), adversarial_per_batch))
        if large is not None:
            n_large = negative_per_batch if medium is None else int(negative_per_batch * 2 / 3)
            neg.append((DevicePool(large, generator), n_large))
        if medium is not None:
            n_med = negative_per_batch if large is None else negative_per_batch - int(negative_per_batch * 2 / 3)
            neg.append((DevicePool(medium, generator), n_med))
        return cls(positive=pos, negative=neg)
