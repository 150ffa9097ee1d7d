"""Drop-in for heybuddy.dataset.training (reference
src/python/heybuddy/dataset/training.py): ``TrainingDatasetIterator`` and
``WakeWordTrainingDatasetIterator`` with the reference's constructors and
classmethods ``default`` (:280-469), ``testing`` (:471-630), ``validation``
(:632-703) and ``all`` (:705-905), same keyword names and defaults.

A batch is [positives | negatives...] in list order with labels 1 / 0
(_generate_batches, :245-277); the default mix is positives 50, adversarial
50 (label 0), large negatives int(1000 * 2/3), medium negatives the rest
(:436-451). ``multiply_batch_size`` scales every share with max(1, int(n * r))
between stages (:215-231); ``max_samples`` bounds the batches one iteration
yields (testing / validation, :88-118).

What differs (by design): each dataset is an HBM-resident embedding table
([N, 16, 96], f16 or f32) read in a per-pass random permutation with
wrap-around (PrecalculatedDatasetIterator.take, precalculated.py:501-536),
sampled by index on the device, so there are no host threads, no queue and no
host-to-device copy per step (``num_batch_threads`` / ``max_queued_batches``
are accepted and unused). Permutations come from a device generator seeded
by ``seed``, so data-parallel ranks draw identical global batches.

Offline (no network): the hosted negative sets (PrecalculatedTrainingDatasetLarge
/ Medium, PrecalculatedValidationDataset) are used when their files are in
the precalculated directory; otherwise synthetic negatives featurized on the
device stand in for them (``offline_negative_samples``, a warning is logged).
"""
from __future__ import annotations

import os
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from heybuddy.constants import (DEFAULT_ADVERSARIAL_BATCH_SIZE, DEFAULT_ADVERSARIAL_PHRASES,
                                DEFAULT_ADVERSARIAL_SAMPLES, DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB, DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                                DEFAULT_AUGMENT_BAND_STOP_PROB, DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB, DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB, DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                                DEFAULT_AUGMENT_GAIN_PROB, DEFAULT_AUGMENT_PHRASE_PROB, DEFAULT_AUGMENT_PHRASE_WORDS,
                                DEFAULT_AUGMENT_PITCH_SHIFT_PROB, DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
                                DEFAULT_AUGMENT_REVERB_PROB, DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                                DEFAULT_AUGMENT_SEVEN_BAND_PROB, DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
                                DEFAULT_AUGMENT_TANH_MAX_DISTORTION, DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                                DEFAULT_BATCH_THREADS, DEFAULT_NEGATIVE_BATCH_SIZE, DEFAULT_POSITIVE_BATCH_SIZE,
                                DEFAULT_POSITIVE_SAMPLES)
from heybuddy.util import logger

__all__ = ["DevicePool", "TrainingDatasetIterator", "WakeWordTrainingDatasetIterator",
           "OFFLINE_NEGATIVE_SAMPLES", "OFFLINE_VALIDATION_NEGATIVE_SAMPLES"]

SupplementalDatasetType = Optional[Union[str, List[str], Tuple[str, ...]]]
# synthetic stand-ins for the hosted sets when their files are absent (offline)
OFFLINE_NEGATIVE_SAMPLES = 200_000
OFFLINE_VALIDATION_NEGATIVE_SAMPLES = 25_000


class DevicePool:
    """An HBM-resident embedding table taken in per-pass random permutations
    with wrap-around (PrecalculatedDatasetIterator.take's order on the device)."""

    def __init__(self, data: torch.Tensor, generator: Optional[torch.Generator] = None) -> None:
        self.data = data
        self.n = data.shape[0]
        if self.n == 0:
            raise ValueError("empty dataset")
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


def _to_pool(ds: Any, device: torch.device, generator: Optional[torch.Generator]) -> DevicePool:
    if isinstance(ds, DevicePool):
        return ds
    if isinstance(ds, torch.Tensor):
        return DevicePool(ds.to(device), generator)
    if isinstance(ds, np.ndarray):
        return DevicePool(torch.from_numpy(np.ascontiguousarray(ds)).to(device), generator)
    if hasattr(ds, "to_device"):  # PrecalculatedDatasetIterator (labeled token row dropped, exclusion applied)
        return DevicePool(ds.to_device(device), generator)
    raise TypeError(f"unsupported dataset {type(ds).__name__}")


class TrainingDatasetIterator:
    """Batches of the positive and negative datasets (training.py:29-277)."""

    def __init__(self, max_samples: Optional[int] = None, num_batch_threads: int = 2,
                 max_queued_batches: int = 100, start: bool = True,
                 positive: Sequence[Tuple[Any, int]] = (), negative: Sequence[Tuple[Any, int]] = (),
                 device: Optional[Union[torch.device, int]] = None, seed: int = 0,
                 generator: Optional[torch.Generator] = None, **kwargs: Any) -> None:
        if not positive and not negative:
            raise ValueError("At least one positive or negative dataset is required")
        self.max_samples = max_samples
        self.num_batch_threads = num_batch_threads
        self.max_queued_batches = max_queued_batches
        self.total_yielded_samples = 0
        self.started = False
        self._device = device
        self._seed = seed
        self._gen = generator
        self.positive: List[Tuple[Any, int]] = list(positive)
        self.negative: List[Tuple[Any, int]] = list(negative)
        if start:
            self.start()

    @property
    def device(self) -> torch.device:
        for ds, _ in self.positive + self.negative:
            for t in (getattr(ds, "data", None), ds):
                if isinstance(t, torch.Tensor) and t.device.type == "cuda":
                    return t.device
        from heybuddy import _native
        return _native.require_device(self._device)

    def _pools(self) -> None:
        """Datasets -> device pools (once; PrecalculatedDatasetIterator files are read here)."""
        if all(isinstance(d, DevicePool) for d, _ in self.positive + self.negative):
            return
        dev = self.device
        if self._gen is None:
            self._gen = torch.Generator(device=dev).manual_seed(int(self._seed))
        self.positive = [(_to_pool(d, dev, self._gen), n) for d, n in self.positive]
        self.negative = [(_to_pool(d, dev, self._gen), n) for d, n in self.negative]

    def metadata(self) -> Dict[str, Any]:
        return {"max_samples": self.max_samples, "num_batch_threads": self.num_batch_threads,
                "positive": [{"length": len(d), "batch_size": n} for d, n in self.positive],
                "negative": [{"length": len(d), "batch_size": n} for d, n in self.negative]}

    def summary(self) -> str:
        lines = [f"Total batches yielded: {self.total_yielded_samples}"]
        for kind, lst in (("Positive", self.positive), ("Negative", self.negative)):
            for i, (d, n) in enumerate(lst):
                taken = getattr(d, "total_taken", 0)
                lines.append(f"{kind} dataset {i + 1}: {taken} samples taken out of {len(d)} unique samples "
                             f"({n} per batch, {taken / max(1, len(d)):.2%} seen)")
        return "\n".join(lines)

    def start(self) -> None:
        self.started = True

    def stop(self) -> None:
        self.started = False

    def check_restart(self) -> None:
        if not self.started:
            self.start()

    def multiply_batch_size(self, ratio: float) -> None:
        self.positive = [(d, max(1, int(n * ratio))) for d, n in self.positive]
        self.negative = [(d, max(1, int(n * ratio))) for d, n in self.negative]

    def half_batch_size(self) -> None:
        self.multiply_batch_size(0.5)

    def double_batch_size(self) -> None:
        self.multiply_batch_size(2)

    @property
    def batch_size(self) -> int:
        return sum(n for _, n in self.positive) + sum(n for _, n in self.negative)

    def next_batch(self) -> Tuple[torch.Tensor, torch.Tensor]:
        self._pools()
        xs, ys = [], []
        for pool, n in self.positive:
            xs.append(pool.take(n))
            ys.append(torch.ones(n, dtype=torch.int64, device=pool.data.device))
        for pool, n in self.negative:
            xs.append(pool.take(n))
            ys.append(torch.zeros(n, dtype=torch.int64, device=pool.data.device))
        return torch.cat([t.to(torch.float32) for t in xs]), torch.cat(ys)

    def iterate(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        yielded = 0
        while self.max_samples is None or yielded < self.max_samples:
            batch = self.next_batch()
            yielded += 1
            self.total_yielded_samples += 1
            yield batch

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        return self.iterate()


def _features_kwargs(loc: Dict[str, Any]) -> Dict[str, Any]:
    """The augment_* / phrase_* / streaming keywords get_training_features takes."""
    keys = [k for k in loc if k.startswith("augment_")] + ["phrase_augment_prob", "phrase_augment_words",
                                                            "dataset_streaming", "use_cache"]
    return {k: loc[k] for k in keys if k in loc}


class WakeWordTrainingDatasetIterator(TrainingDatasetIterator):
    """Training / testing / validation iterators of one wake phrase."""

    def __init__(self, max_samples: Optional[int] = None, num_batch_threads: int = 2, max_queued_batches: int = 100,
                 start: bool = True, positive: Sequence[Tuple[Any, int]] = (),
                 negative: Sequence[Tuple[Any, int]] = (), **kwargs: Any) -> None:
        super().__init__(max_samples=max_samples, num_batch_threads=num_batch_threads,
                         max_queued_batches=max_queued_batches, start=start, positive=positive, negative=negative,
                         **kwargs)

    @classmethod
    def from_tensors(cls, positive: torch.Tensor, adversarial: Optional[torch.Tensor] = None,
                     large: Optional[torch.Tensor] = None, medium: Optional[torch.Tensor] = None,
                     positive_per_batch: int = DEFAULT_POSITIVE_BATCH_SIZE,
                     adversarial_per_batch: int = DEFAULT_ADVERSARIAL_BATCH_SIZE,
                     negative_per_batch: int = DEFAULT_NEGATIVE_BATCH_SIZE,
                     generator: Optional[torch.Generator] = None, **kwargs: Any
                     ) -> "WakeWordTrainingDatasetIterator":
        """default()'s batch composition over device tensors."""
        pos = [(DevicePool(positive, generator), positive_per_batch)]
        neg: List[Tuple[Any, int]] = []
        if adversarial is not None:
            neg.append((DevicePool(adversarial, generator), adversarial_per_batch))
        if large is not None:
            n_large = negative_per_batch if medium is None else int(negative_per_batch * 2 / 3)
            neg.append((DevicePool(large, generator), n_large))
        if medium is not None:
            n_med = negative_per_batch if large is None else negative_per_batch - int(negative_per_batch * 2 / 3)
            neg.append((DevicePool(medium, generator), n_med))
        return cls(positive=pos, negative=neg, generator=generator, **kwargs)

    @staticmethod
    def _hosted(kind: str, wake_phrase: str, offline_samples: int, device_id: Optional[int], seed: int) -> Any:
        """A hosted negative set if its file is present, else the synthetic stand-in."""
        from heybuddy.dataset import precalculated as pc
        cls_ = {"large": pc.PrecalculatedTrainingDatasetLarge, "medium": pc.PrecalculatedTrainingDatasetMedium,
                "validation": pc.PrecalculatedValidationDataset}[kind]
        try:
            return cls_(exclude_phrase=wake_phrase)
        except FileNotFoundError:
            logger.warning(f"{cls_.__name__}: {cls_.file_name()} is not in {pc.LOCAL_DIR} (a download; no network): "
                           f"using {offline_samples} synthetic negatives featurized on the device instead")
            from heybuddy.dataset.features import synthetic_negative_features
            return synthetic_negative_features(f"synthetic-{kind}", offline_samples, device_id=device_id,
                                               seed=seed + {"large": 1, "medium": 2, "validation": 3}[kind])

    @classmethod
    def default(cls, wake_phrase: str, additional_wake_phrases: List[str] = [],
                num_positive_samples: int = DEFAULT_POSITIVE_SAMPLES,
                num_adversarial_phrases: int = DEFAULT_ADVERSARIAL_PHRASES,
                custom_adversarial_phrases: List[str] = [],
                num_adversarial_samples: int = DEFAULT_ADVERSARIAL_SAMPLES,
                positive_per_batch: int = DEFAULT_POSITIVE_BATCH_SIZE,
                negative_per_batch: int = DEFAULT_NEGATIVE_BATCH_SIZE,
                adversarial_per_batch: int = DEFAULT_ADVERSARIAL_BATCH_SIZE,
                use_cache: bool = True, dataset_streaming: bool = False,
                num_batch_threads: int = DEFAULT_BATCH_THREADS, start: bool = True,
                large_training: bool = True, medium_training: bool = True, custom_training: Optional[str] = None,
                phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
                phrase_augment_words: List[str] = DEFAULT_AUGMENT_PHRASE_WORDS,
                augment_dataset_streaming: bool = False,
                augment_background_dataset: SupplementalDatasetType = None,
                augment_impulse_dataset: SupplementalDatasetType = None,
                augment_seven_band_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
                augment_seven_band_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                augment_tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
                augment_tanh_min_distortion: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                augment_tanh_max_distortion: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                augment_pitch_shift_prob: float = DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
                augment_pitch_shift_semitones: int = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
                augment_band_stop_prob: float = DEFAULT_AUGMENT_BAND_STOP_PROB,
                augment_colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                augment_colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
                augment_colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                augment_colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                augment_colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                augment_background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                augment_background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                augment_background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                augment_gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
                augment_reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB,
                device_id: Optional[int] = None, seed: int = 0,
                offline_negative_samples: int = OFFLINE_NEGATIVE_SAMPLES) -> "WakeWordTrainingDatasetIterator":
        """training.py:280-469: the phrase's positive / adversarial features
        (TrainingFeaturesGenerator.get_training_features, augmented, cached by
        phrase name) plus the large / medium / custom negative sets."""
        from heybuddy.dataset.features import TrainingFeaturesGenerator
        from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
        fkw = _features_kwargs(locals())
        positive_list: List[Tuple[Any, int]] = []
        negative_list: List[Tuple[Any, int]] = []
        for i, phrase in enumerate([wake_phrase] + list(additional_wake_phrases)):
            pos, adv = TrainingFeaturesGenerator.get_training_features(
                wake_phrase=phrase, num_positive_samples=num_positive_samples,
                num_adversarial_samples=num_adversarial_samples, num_adversarial_phrases=num_adversarial_phrases,
                custom_adversarial_phrases=custom_adversarial_phrases if i == 0 else [],
                additional_wake_phrases=additional_wake_phrases if i == 0 else [], device_id=device_id, **fkw)
            positive_list.append((pos, positive_per_batch))
            negative_list.append((adv, adversarial_per_batch))
        if large_training:
            n = negative_per_batch if not medium_training else int(negative_per_batch * 2 / 3)
            negative_list.append((cls._hosted("large", wake_phrase, offline_negative_samples * 2 // 3, device_id,
                                              seed), n))
        if medium_training:
            n = negative_per_batch if not large_training else negative_per_batch - int(negative_per_batch * 2 / 3)
            negative_list.append((cls._hosted("medium", wake_phrase, offline_negative_samples
                                              - offline_negative_samples * 2 // 3, device_id, seed), n))
        if custom_training:
            negative_list.append((PrecalculatedDatasetIterator(
                name=os.path.splitext(os.path.basename(custom_training))[0],
                directory=os.path.dirname(custom_training), exclude_phrase=wake_phrase, labeled=True),
                negative_per_batch))
        return cls(positive=positive_list, negative=negative_list, num_batch_threads=num_batch_threads, start=start,
                   device=device_id, seed=seed)

    @classmethod
    def testing(cls, wake_phrase: str, additional_wake_phrases: List[str] = [], num_positive_samples: int = 1000,
                num_adversarial_samples: int = 1000, num_adversarial_phrases: int = 10,
                custom_adversarial_phrases: List[str] = [], positive_per_batch: int = 50,
                adversarial_per_batch: int = 50, use_cache: bool = True, dataset_streaming: bool = False,
                num_batch_threads: int = 1, start: bool = True,
                phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
                phrase_augment_words: List[str] = DEFAULT_AUGMENT_PHRASE_WORDS,
                augment_dataset_streaming: bool = False,
                augment_background_dataset: SupplementalDatasetType = None,
                augment_impulse_dataset: SupplementalDatasetType = None,
                augment_seven_band_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
                augment_seven_band_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
                augment_tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
                augment_tanh_min_distortion: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
                augment_tanh_max_distortion: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                augment_pitch_shift_prob: float = DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
                augment_pitch_shift_semitones: int = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
                augment_band_stop_prob: float = DEFAULT_AUGMENT_BAND_STOP_PROB,
                augment_colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                augment_colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
                augment_colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                augment_colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                augment_colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                augment_background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                augment_background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                augment_background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                augment_gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
                augment_reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB,
                device_id: Optional[int] = None, seed: int = 0) -> "WakeWordTrainingDatasetIterator":
        """training.py:471-630: augmented testing features (cached as ``{name}_tst``),
        max_samples = max(n_pos // pos_per_batch, n_adv // adv_per_batch) batches."""
        from heybuddy.dataset.features import TrainingFeaturesGenerator
        fkw = _features_kwargs(locals())
        positive_list: List[Tuple[Any, int]] = []
        negative_list: List[Tuple[Any, int]] = []
        for i, phrase in enumerate([wake_phrase] + list(additional_wake_phrases)):
            pos, adv = TrainingFeaturesGenerator.get_training_features(
                wake_phrase=phrase, num_positive_samples=num_positive_samples,
                num_adversarial_samples=num_adversarial_samples, num_adversarial_phrases=num_adversarial_phrases,
                custom_adversarial_phrases=custom_adversarial_phrases if i == 0 else [], testing=True,
                device_id=device_id, **fkw)
            positive_list.append((pos, positive_per_batch))
            negative_list.append((adv, adversarial_per_batch))
        return cls(positive=positive_list, negative=negative_list,
                   max_samples=max(num_positive_samples // positive_per_batch,
                                   num_adversarial_samples // adversarial_per_batch),
                   num_batch_threads=num_batch_threads, start=start, device=device_id, seed=seed + 17)

    @classmethod
    def validation(cls, wake_phrase: str, additional_wake_phrases: List[str] = [], positive_batch_size: int = 50,
                   negative_batch_size: int = 1000, num_samples: int = 1000, num_batch_threads: int = 1,
                   start: bool = True, precalculated_validation: bool = True, custom_validation: Optional[str] = None,
                   phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
                   phrase_augment_words: List[str] = DEFAULT_AUGMENT_PHRASE_WORDS,
                   device_id: Optional[int] = None, seed: int = 0,
                   offline_negative_samples: int = OFFLINE_VALIDATION_NEGATIVE_SAMPLES
                   ) -> "WakeWordTrainingDatasetIterator":
        """training.py:632-703: un-augmented, centre-padded positives
        (get_validation_features) against the validation negatives;
        max_samples = max(n_neg // negative_batch_size, n_pos // positive_batch_size)."""
        from heybuddy.dataset.features import TrainingFeaturesGenerator
        from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
        negative_list: List[Tuple[Any, int]] = []
        if precalculated_validation:
            negative_list.append((cls._hosted("validation", wake_phrase, offline_negative_samples, device_id, seed),
                                  negative_batch_size))
        if custom_validation:
            negative_list.append((PrecalculatedDatasetIterator(
                name=os.path.splitext(os.path.basename(custom_validation))[0],
                directory=os.path.dirname(custom_validation), exclude_phrase=wake_phrase, labeled=True),
                negative_batch_size))
        n_neg = sum(len(d) for d, _ in negative_list)
        pos = TrainingFeaturesGenerator.get_validation_features(wake_phrase=wake_phrase,
                                                                num_positive_samples=num_samples,
                                                                device_id=device_id)
        positive_list: List[Tuple[Any, int]] = [(pos, positive_batch_size)]
        for phrase in additional_wake_phrases:
            positive_list.append((TrainingFeaturesGenerator.get_validation_features(
                wake_phrase=phrase, num_positive_samples=num_samples, phrase_augment_prob=phrase_augment_prob,
                phrase_augment_words=phrase_augment_words, device_id=device_id), positive_batch_size))
        return cls(positive=positive_list, negative=negative_list, num_batch_threads=num_batch_threads,
                   max_samples=max(n_neg // negative_batch_size, len(pos) // positive_batch_size),
                   start=start, device=device_id, seed=seed + 29)

    @classmethod
    def all(cls, wake_phrase: str, additional_wake_phrases: List[str] = [], num_positive_samples: int = 100000,
            num_adversarial_samples: int = 50000, num_adversarial_phrases: int = 10,
            custom_adversarial_phrases: List[str] = [], positive_per_batch: int = 50, negative_per_batch: int = 1000,
            adversarial_per_batch: int = 50, num_batch_threads: int = 2, large_training: bool = True,
            medium_training: bool = True, custom_training: Optional[str] = None,
            validation_positive_batch_size: int = 50, validation_negative_batch_size: int = 1000,
            validation_num_positive_samples: int = 1000, validation_num_batch_threads: int = 1,
            validation_include_precalculated: bool = True, validation_custom: Optional[str] = None,
            testing_num_positive_samples: int = 1000, testing_num_adversarial_samples: int = 1000,
            testing_num_adversarial_phrases: int = 10, testing_custom_adversarial_phrases: List[str] = [],
            testing_positive_per_batch: Optional[int] = None, testing_adversarial_per_batch: Optional[int] = None,
            testing_num_batch_threads: int = 1, dataset_streaming: bool = False, start: bool = True,
            phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
            phrase_augment_words: List[str] = DEFAULT_AUGMENT_PHRASE_WORDS,
            augment_dataset_streaming: bool = False,
            augment_background_dataset: SupplementalDatasetType = None,
            augment_impulse_dataset: SupplementalDatasetType = None,
            augment_seven_band_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
            augment_seven_band_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
            augment_tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
            augment_tanh_min_distortion: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
            augment_tanh_max_distortion: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
            augment_pitch_shift_prob: float = DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
            augment_pitch_shift_semitones: int = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
            augment_band_stop_prob: float = DEFAULT_AUGMENT_BAND_STOP_PROB,
            augment_colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
            augment_colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
            augment_colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
            augment_colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
            augment_colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
            augment_background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
            augment_background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
            augment_background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
            augment_gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
            augment_reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB,
            device_id: Optional[int] = None, seed: int = 0,
            offline_negative_samples: int = OFFLINE_NEGATIVE_SAMPLES,
            offline_validation_negative_samples: int = OFFLINE_VALIDATION_NEGATIVE_SAMPLES
            ) -> Tuple["WakeWordTrainingDatasetIterator", "WakeWordTrainingDatasetIterator",
                       "WakeWordTrainingDatasetIterator"]:
        """training.py:705-905: (training, validation, testing)."""
        aug = {k: v for k, v in locals().items() if k.startswith("augment_")}
        common = dict(phrase_augment_prob=phrase_augment_prob, phrase_augment_words=phrase_augment_words,
                      dataset_streaming=dataset_streaming, start=False, device_id=device_id, seed=seed)
        training = cls.default(wake_phrase=wake_phrase, additional_wake_phrases=additional_wake_phrases,
                               num_positive_samples=num_positive_samples,
                               num_adversarial_samples=num_adversarial_samples,
                               num_adversarial_phrases=num_adversarial_phrases,
                               custom_adversarial_phrases=custom_adversarial_phrases,
                               positive_per_batch=positive_per_batch, negative_per_batch=negative_per_batch,
                               adversarial_per_batch=adversarial_per_batch, num_batch_threads=num_batch_threads,
                               large_training=large_training, medium_training=medium_training,
                               custom_training=custom_training, offline_negative_samples=offline_negative_samples,
                               **common, **aug)
        testing = cls.testing(wake_phrase=wake_phrase, additional_wake_phrases=additional_wake_phrases,
                              num_positive_samples=testing_num_positive_samples,
                              num_adversarial_samples=testing_num_adversarial_samples,
                              num_adversarial_phrases=testing_num_adversarial_phrases,
                              custom_adversarial_phrases=testing_custom_adversarial_phrases,
                              positive_per_batch=testing_positive_per_batch or positive_per_batch,
                              adversarial_per_batch=testing_adversarial_per_batch or adversarial_per_batch,
                              num_batch_threads=testing_num_batch_threads, **common, **aug)
        validation = cls.validation(wake_phrase=wake_phrase, additional_wake_phrases=additional_wake_phrases,
                                    positive_batch_size=validation_positive_batch_size,
                                    negative_batch_size=validation_negative_batch_size,
                                    num_batch_threads=validation_num_batch_threads,
                                    num_samples=validation_num_positive_samples, start=False,
                                    precalculated_validation=validation_include_precalculated,
                                    custom_validation=validation_custom, device_id=device_id, seed=seed,
                                    offline_negative_samples=offline_validation_negative_samples)
        if start:
            training.start()
            validation.start()
            testing.start()
        return training, validation, testing
