"""Precalculated feature sets (reference src/python/heybuddy/dataset/precalculated.py:376-570).

``PrecalculatedDatasetIterator`` keeps the reference's name-keyed ``.npy``
store (``{directory}/{name}.npy``, memory-mapped), ``from_array``, the
shuffled ``take(n)`` with wrap-around and reshuffle, ``iterate`` and the
labeled ``[N, 17, 96]`` layout (row 16 holds BERT token ids; ``take`` drops
it). The BERT-token exclusion filter needs a tokenizer download and is not on
this path. ``to_device`` moves the whole set into HBM for the on-device
sampler (heybuddy.dataset.training.DevicePool), which replaces the
reference's 12 host threads gathering memmap rows.

The hosted 72 GB negative sets (HostedPrecalculatedDatasetIterator,
:572-649) need a network download and are out of scope offline.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Iterator, Optional

import numpy as np

__all__ = ["LOCAL_DIR", "PrecalculatedDatasetIterator"]

LOCAL_DIR = os.path.abspath(os.environ.get("HEYBUDDY_PRECALCULATED_DIR",
                                           os.path.join(os.getcwd(), "precalculated")))


class PrecalculatedDatasetIterator:
    def __init__(self, name: str, directory: str = LOCAL_DIR, exclude_phrase: Optional[str] = None,
                 ordered: bool = False, labeled: bool = False, use_mem_map: bool = True,
                 shuffle: bool = True, data: Optional[np.ndarray] = None) -> None:
        if exclude_phrase is not None:
            raise NotImplementedError("token exclusion needs the BERT tokenizer download (out of scope)")
        self.directory = directory
        self.name = name
        self.exclude_phrase = exclude_phrase
        self.index = 0
        self.total_taken = 0
        self.ordered = ordered
        self.labeled = labeled
        self.use_mem_map = use_mem_map
        if data is not None:
            self._precalculated = data
        if not os.path.exists(self.precalculated_path):
            raise FileNotFoundError(f"Could not find precalculated features at {self.precalculated_path}.")
        if shuffle and not ordered:
            self.shuffle()

    @property
    def precalculated_path(self) -> str:
        return os.path.join(self.directory, f"{self.name}.npy")

    @property
    def precalculated(self) -> np.ndarray:
        if not hasattr(self, "_precalculated"):
            self._precalculated = np.load(self.precalculated_path, mmap_mode="r" if self.use_mem_map else None)
        return self._precalculated

    @property
    def indexes(self) -> np.ndarray:
        if not hasattr(self, "_indexes"):
            self._indexes = np.arange(len(self.precalculated))
        return self._indexes

    @classmethod
    def from_array(cls, array: np.ndarray, name: str, directory: str = LOCAL_DIR, ordered: bool = False,
                   keep_in_memory: bool = False) -> "PrecalculatedDatasetIterator":
        """Save ``array`` as ``{directory}/{name}.npy`` and open it (precalculated.py:471-491)."""
        os.makedirs(directory, exist_ok=True)
        np.save(os.path.join(directory, f"{name}.npy"), array)
        return cls(name, directory=directory, data=array if keep_in_memory else None, ordered=ordered)

    def shuffle(self) -> "PrecalculatedDatasetIterator":
        if not self.ordered:
            np.random.shuffle(self.indexes)
        return self

    def take(self, n: int) -> np.ndarray:
        """The next n rows of the (shuffled) order; at the end the order is
        reshuffled and the batch continues from its start (precalculated.py:501-536)."""
        batch = self.precalculated[self.indexes[self.index:self.index + n]]
        if batch.shape[0] < n:
            self.index = n - batch.shape[0]
            self.shuffle()
            batch = np.concatenate([batch, self.precalculated[self.indexes[:self.index]]])
        else:
            self.index += n
        if self.labeled:
            batch = batch[:, :-1]
        self.total_taken += n
        return batch

    def iterate(self) -> Iterator[np.ndarray]:
        while True:
            yield self.take(1)

    def to_device(self, device: Any, dtype: Any = None):
        """The whole set as one HBM tensor (labeled sets without the token row)."""
        import torch
        arr = np.asarray(self.precalculated)
        if self.labeled:
            arr = arr[:, :-1]
        t = torch.from_numpy(np.ascontiguousarray(arr)).to(device)
        return t if dtype is None else t.to(dtype)

    def metadata(self) -> Dict[str, Any]:
        return {"name": self.name, "path": self.precalculated_path, "shape": self.precalculated.shape,
                "ordered": self.ordered, "labeled": self.labeled, "use_mem_map": self.use_mem_map}

    def __len__(self) -> int:
        return self.precalculated.shape[0]

    def __iter__(self) -> Iterator[np.ndarray]:
        return self.iterate()

    def __repr__(self) -> str:
        return f"{type(self).__name__}(num_samples={len(self)})"
