"""Precalculated feature sets (reference src/python/heybuddy/dataset/precalculated.py:376-570).

``PrecalculatedDatasetIterator`` keeps the reference's name-keyed ``.npy``
store (``{directory}/{name}.npy``, memory-mapped), ``from_array``, the
shuffled ``take(n)`` with wrap-around and reshuffle, ``iterate`` and the
labeled ``[N, 17, 96]`` layout (row 16 holds BERT token ids; ``take`` drops
it). The BERT-token exclusion filter needs a tokenizer download and is not on
this path. ``to_device`` moves the whole set into HBM for the on-device
sampler (heybuddy.dataset.training.DevicePool), which replaces the
reference's 12 host threads gathering memmap rows.

``PrecalculatedTrainingDatasetGenerator`` / ``...LabeledTrainingDatasetGenerator``
(precalculated.py:40-374, the ``heybuddy extract`` command) cut every clip of
an audio dataset into 1.44-s windows (right-padded), featurize them on the
MI355X and write ``{output_dir}/{name}/{k}.npy`` files with the reference's
flush points (a file is written once the buffer reaches samples_per_file rows
after a batch; NaN rows are dropped). The windows of several process batches
are featurized in one device call; the per-batch bookkeeping is replayed in
order, so file boundaries match the reference's. The dataset is opened with
``datasets.load_dataset`` (local paths work offline; hub downloads do not).

The hosted 72 GB negative sets (HostedPrecalculatedDatasetIterator,
:572-649) need a network download and are out of scope offline.
"""
from __future__ import annotations

import math
import os
import re
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Tuple

import numpy as np

from heybuddy.util import logger

__all__ = ["LOCAL_DIR", "PrecalculatedDatasetIterator", "PrecalculatedTrainingDatasetGenerator",
           "PrecalculatedLabeledTrainingDatasetGenerator", "HostedPrecalculatedDatasetIterator",
           "PrecalculatedTrainingDatasetLarge", "PrecalculatedTrainingDatasetMedium", "PrecalculatedValidationDataset"]

LOCAL_DIR = os.path.abspath(os.environ.get("HEYBUDDY_PRECALCULATED_DIR",
                                           os.path.join(os.getcwd(), "precalculated")))


class PrecalculatedDatasetIterator:
    def __init__(self, name: str, directory: Optional[str] = None, exclude_phrase: Optional[str] = None,
                 ordered: bool = False, labeled: bool = False, use_mem_map: bool = True,
                 shuffle: bool = True, data: Optional[np.ndarray] = None,
                 exclude_tokens: Optional[Iterable[int]] = None) -> None:
        """exclude_phrase (labeled sets, precalculated.py:519-531): rows whose
        token row shares a token with the phrase are skipped. The reference
        tokenizes the phrase with bert-base-uncased (a download); here the token
        ids come from ``exclude_tokens`` (or HEYBUDDY_EXCLUDE_TOKENIZER, a local
        tokenizer directory); without either the phrase is not excluded (a
        warning is logged)."""
        self.directory = directory or LOCAL_DIR  # resolved per call: LOCAL_DIR may be re-pointed
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
        self.exclude_tokens = set(int(t) for t in exclude_tokens) if exclude_tokens is not None else None
        if exclude_phrase is not None and labeled and self.exclude_tokens is None:
            self.exclude_tokens = _phrase_tokens(exclude_phrase)
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
    def from_array(cls, array: np.ndarray, name: str, directory: Optional[str] = None, ordered: bool = False,
                   keep_in_memory: bool = False) -> "PrecalculatedDatasetIterator":
        """Save ``array`` as ``{directory}/{name}.npy`` and open it (precalculated.py:471-491)."""
        directory = directory or LOCAL_DIR
        os.makedirs(directory, exist_ok=True)
        np.save(os.path.join(directory, f"{name}.npy"), array)
        return cls(name, directory=directory, data=array if keep_in_memory else None, ordered=ordered)

    def shuffle(self) -> "PrecalculatedDatasetIterator":
        if not self.ordered:
            np.random.shuffle(self.indexes)
        return self

    def _next_rows(self, n: int) -> np.ndarray:
        """The next n rows of the (shuffled) order, reshuffling at the end and
        continuing from its start (precalculated.py:508-517)."""
        batch = self.precalculated[self.indexes[self.index:self.index + n]]
        if batch.shape[0] < n:
            self.index = n - batch.shape[0]
            self.shuffle()
            batch = np.concatenate([batch, self.precalculated[self.indexes[:self.index]]])
        else:
            self.index += n
        return batch

    def take(self, n: int) -> np.ndarray:
        """The next n rows of the (shuffled) order; at the end the order is
        reshuffled and the batch continues from its start (precalculated.py:501-536).
        Rows whose token row holds an excluded token are dropped and refilled
        from the following rows, as the reference does (:520-533) -- there by
        recursion, here by a loop (the same rows in the same order, and the
        same total_taken: every refill counts its own request), so a set that
        keeps only a few rows per lap fills any n without Python's recursion
        limit. A full lap of the set that adds no row raises ValueError."""
        parts = []
        want = n
        scanned_dry = 0  # rows read since a row was last kept
        while True:
            batch = self._next_rows(want)
            if self.labeled:
                if self.exclude_tokens:
                    keep = np.array([self.exclude_tokens.isdisjoint(set(np.asarray(r[-1]).astype(np.int64).ravel()))
                                     for r in batch], dtype=bool)
                    batch = batch[keep]
                batch = batch[:, :-1]
            self.total_taken += want
            parts.append(batch)
            got = batch.shape[0]
            if got >= want or not self.labeled:
                break
            scanned_dry = 0 if got else scanned_dry + want
            if scanned_dry >= max(len(self), 1):
                raise ValueError(f"{self.name}: every row contains an excluded token")
            want -= got
        return parts[0] if len(parts) == 1 else np.concatenate(parts)

    def iterate(self) -> Iterator[np.ndarray]:
        while True:
            yield self.take(1)

    def to_device(self, device: Any, dtype: Any = None):
        """The whole set as one HBM tensor (labeled sets without the token row)."""
        import torch
        arr = np.asarray(self.precalculated)
        if self.labeled:
            if self.exclude_tokens:
                tok = arr[:, -1].astype(np.int64)
                keep = ~np.isin(tok, np.fromiter(self.exclude_tokens, np.int64)).any(axis=1)
                arr = arr[keep]
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


def _phrase_tokens(phrase: str) -> Optional[set]:
    """The phrase's token ids (precalculated.py:398-434: special characters to
    spaces, BERT uncased), from a local tokenizer directory in
    HEYBUDDY_EXCLUDE_TOKENIZER; None (and a warning) when there is none."""
    text = re.sub(r"\s+", " ", re.sub(r"[^a-zA-Z0-9]", " ", phrase.replace("'", ""))).strip()
    path = os.environ.get("HEYBUDDY_EXCLUDE_TOKENIZER")
    if path:
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
        # the reference's BERTTokenizer drops [CLS] / [SEP] (tokens.py:57: ids[1:-1])
        return set(int(t) for t in tok(text, add_special_tokens=False)["input_ids"])
    logger.warning(f"no local tokenizer (HEYBUDDY_EXCLUDE_TOKENIZER): rows containing {phrase!r} are not excluded")
    return None


class HostedPrecalculatedDatasetIterator(PrecalculatedDatasetIterator):
    """A hosted feature set (precalculated.py:563-616): labeled, memory-mapped,
    named after its URL's file. The reference downloads it into the
    precalculated directory; offline the file must already be there
    (FileNotFoundError otherwise)."""
    precalculated_url: str = ""
    precalculated_ordered: bool = False
    precalculated_labeled: bool = True
    precalculated_use_mem_map: bool = True

    @classmethod
    def file_name(cls) -> str:
        return cls.precalculated_url.rsplit("/", 1)[-1]

    def __init__(self, directory: Optional[str] = None, exclude_phrase: Optional[str] = None,
                 exclude_tokens: Optional[Iterable[int]] = None) -> None:
        super().__init__(name=os.path.splitext(self.file_name())[0], directory=directory,
                         ordered=self.precalculated_ordered, labeled=self.precalculated_labeled,
                         exclude_phrase=exclude_phrase, use_mem_map=self.precalculated_use_mem_map,
                         exclude_tokens=exclude_tokens)


_HOSTED = "https://huggingface.co/datasets/benjamin-paine/hey-buddy/resolve/main/precalculated/common/"


class PrecalculatedTrainingDatasetLarge(HostedPrecalculatedDatasetIterator):
    """In-the-wild negatives for training (precalculated.py:618-626)."""
    precalculated_url = _HOSTED + "training-large.npy"


class PrecalculatedTrainingDatasetMedium(HostedPrecalculatedDatasetIterator):
    """In-the-wild negatives for training (precalculated.py:628-636)."""
    precalculated_url = _HOSTED + "training-medium.npy"


class PrecalculatedValidationDataset(HostedPrecalculatedDatasetIterator):
    """In-the-wild speech for the validation false-positive rate (precalculated.py:638-649)."""
    precalculated_url = _HOSTED + "validation.npy"


class PrecalculatedTrainingDatasetGenerator:
    """Audio dataset -> packed [N, 16, 96] embedding files (precalculated.py:40-278)."""

    # process batches featurized per device call (their windows share one launch)
    GROUP_WINDOWS = 8192

    def __init__(self, dataset_path: str, config_name: Optional[str] = None, split: str = "train",
                 audio_key: str = "audio", audio_array_key: Optional[str] = "array",
                 audio_sample_rate_key: Optional[str] = "sampling_rate", device_id: Optional[int] = None,
                 sample_rate: int = 16000, seconds_per_batch: float = 1.44, process_batch_size: int = 128,
                 embedding_batch_size: int = 32) -> None:
        self.dataset_path = dataset_path
        self.config_name = config_name
        self.split = split
        self.audio_key = audio_key
        self.audio_array_key = audio_array_key
        self.audio_sample_rate_key = audio_sample_rate_key
        self.device_id = device_id
        self.sample_rate = sample_rate
        self.seconds_per_batch = seconds_per_batch
        self.process_batch_size = process_batch_size
        self.embedding_batch_size = embedding_batch_size

    @property
    def samples_per_batch(self) -> int:
        return int(self.sample_rate * self.seconds_per_batch)

    @property
    def speech_embeddings(self):
        if not hasattr(self, "_speech_embeddings"):
            from heybuddy.embeddings import get_speech_embeddings
            self._speech_embeddings = get_speech_embeddings(device_id=self.device_id)
        return self._speech_embeddings

    def label_embeddings(self, embeddings: np.ndarray, batch: List[Tuple[np.ndarray, Dict[str, Any]]]) -> np.ndarray:
        return embeddings

    def open_dataset(self, streaming: bool, trust_remote_code: bool) -> Iterable[Dict[str, Any]]:
        from datasets import load_dataset
        return load_dataset(self.dataset_path, self.config_name, split=self.split, streaming=streaming,
                            trust_remote_code=trust_remote_code)

    def _sample_audio(self, sample: Dict[str, Any]) -> np.ndarray:
        """The reference's key lookups (:219-235) and resampling (:159-165)."""
        audio = sample.pop(self.audio_key)
        rate = None
        if self.audio_sample_rate_key is not None:
            if isinstance(audio, dict) and self.audio_sample_rate_key in audio:
                rate = audio[self.audio_sample_rate_key]
            elif self.audio_sample_rate_key in sample:
                rate = sample[self.audio_sample_rate_key]
        if self.audio_array_key is not None:
            audio = audio[self.audio_array_key]
        audio = np.asarray(audio)
        if rate is not None and rate != self.sample_rate:
            import torch
            from heybuddy.util import resample
            audio = resample(torch.from_numpy(audio.astype(np.float32)), int(rate), self.sample_rate).numpy()
        return audio.astype(np.float32)

    def _featurize(self, windows: List[np.ndarray]) -> np.ndarray:
        import torch
        se = self.speech_embeddings
        x = torch.from_numpy(np.stack(windows)).to(se.device)
        return se.featurize(x, remove_nan=False).cpu().numpy()

    def __call__(self, name: str, output_dir: str = LOCAL_DIR, max_hours: float = 1000.0,
                 dataset_streaming: bool = True, trust_remote_code: bool = False, samples_per_file: int = 10000,
                 dataset: Optional[Iterable[Dict[str, Any]]] = None) -> List[str]:
        """Write the files; returns their paths. ``dataset`` (an iterable of
        sample dicts) replaces ``load_dataset`` when given."""
        output_dir = os.path.join(output_dir, name)
        os.makedirs(output_dir, exist_ok=True)
        if dataset is None:
            dataset = self.open_dataset(dataset_streaming, trust_remote_code)
        spb, pbs = self.samples_per_batch, self.process_batch_size
        max_batches = int(max_hours * 3600 / self.seconds_per_batch / pbs)
        n_files = math.ceil(max_batches * pbs / samples_per_file)
        digits = int(math.log10(max(n_files, 1))) + 1
        files: List[str] = []
        state = {"buffer": None, "batches": 0}
        pending: List[List[Tuple[np.ndarray, Dict[str, Any]]]] = []

        def flush() -> None:
            path = os.path.join(output_dir, f"{len(files):0{digits}d}.npy")
            np.save(path, state["buffer"])
            files.append(path)
            state["buffer"] = None

        def drain() -> None:
            if not pending:
                return
            emb = self._featurize([a for b in pending for a, _ in b])
            off = 0
            for b in pending:
                e = self.label_embeddings(emb[off:off + len(b)], b)
                off += len(b)
                keep = ~np.isnan(e).any(axis=(1, 2))
                if not keep.all():
                    logger.warning(f"Removed {int((~keep).sum())} samples due to NaN values in embeddings.")
                e = e[keep]
                state["buffer"] = e if state["buffer"] is None else np.concatenate([state["buffer"], e])
                if state["buffer"].shape[0] >= samples_per_file:
                    flush()
            pending.clear()

        batch: List[Tuple[np.ndarray, Dict[str, Any]]] = []
        group = max(1, self.GROUP_WINDOWS // pbs)

        def close_batch() -> None:
            nonlocal batch
            pending.append(batch)
            batch = []
            state["batches"] += 1
            if len(pending) >= group:
                drain()

        for sample in dataset:
            sample = dict(sample)
            audio = self._sample_audio(sample)
            for i in range(0, len(audio), spb):
                w = audio[i:i + spb]
                if w.shape[0] < spb:
                    w = np.concatenate([w, np.zeros(spb - w.shape[0], np.float32)])
                batch.append((w, sample))
                if len(batch) >= pbs:
                    close_batch()
                if state["batches"] >= max_batches:
                    break
            if state["batches"] >= max_batches:
                break
        if batch and state["batches"] < max_batches:
            close_batch()
        drain()
        if state["buffer"] is not None:
            flush()
        return files


class PrecalculatedLabeledTrainingDatasetGenerator(PrecalculatedTrainingDatasetGenerator):
    """[N, 17, 96] files: row 16 holds the transcript's tokens
    (precalculated.py:280-374). The reference's BERTTokenizer downloads its
    vocabulary; here ``tokenizer`` is any callable text -> int array of
    ``tokenizer_max_length`` ids (e.g. a local transformers tokenizer)."""

    def __init__(self, dataset_path: str, config_name: Optional[str] = None, split: str = "train",
                 audio_key: str = "audio", audio_array_key: Optional[str] = "array",
                 audio_sample_rate_key: Optional[str] = "sampling_rate", transcript_key: str = "transcript",
                 device_id: Optional[int] = None, sample_rate: int = 16000, seconds_per_batch: float = 1.44,
                 process_batch_size: int = 128, embedding_batch_size: int = 32, tokenizer_max_length: int = 96,
                 tokenizer: Optional[Callable[[str], np.ndarray]] = None) -> None:
        super().__init__(dataset_path, config_name, split, audio_key, audio_array_key, audio_sample_rate_key,
                         device_id, sample_rate, seconds_per_batch, process_batch_size, embedding_batch_size)
        self.transcript_key = transcript_key
        self.tokenizer_max_length = tokenizer_max_length
        self._tokenizer = tokenizer
        self._cache: Dict[str, np.ndarray] = {}

    def tokenize(self, text: str) -> np.ndarray:
        if text not in self._cache:
            if self._tokenizer is None:
                raise NotImplementedError("labeled extraction needs a tokenizer (the reference's BERT vocabulary "
                                          "is a download); pass tokenizer=")
            ids = np.asarray(self._tokenizer(text), dtype=np.float32).reshape(-1)[:self.tokenizer_max_length]
            self._cache[text] = np.pad(ids, (0, self.tokenizer_max_length - ids.shape[0]))
        return self._cache[text]

    def label_embeddings(self, embeddings: np.ndarray, batch: List[Tuple[np.ndarray, Dict[str, Any]]]) -> np.ndarray:
        tokens = np.stack([self.tokenize(s[self.transcript_key]) for _, s in batch])[:, None, :]
        return np.concatenate([embeddings, tokens], axis=1).astype(np.float32)
