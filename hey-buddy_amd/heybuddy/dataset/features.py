"""Drop-in for heybuddy.dataset.features (reference src/python/heybuddy/dataset/features.py).

``TrainingFeaturesGenerator`` keeps the reference's constructor (every TTS /
augmentation / embedding parameter), ``autoconfigure``, ``generate``,
``__call__(num_samples) -> ndarray [n, 16, 96]``, ``default``,
``get_wake_phrase_file_name``, ``get_training_features`` and
``get_validation_features`` (:30-908). The pipeline per chunk is the
reference's (:360-490):

  TTS (n_tts = n // augment_sample_ratio utterances)
    -> AugmentedAudioGenerator (clip placement, tanh distortion, colored
       noise, gain, background noise, reverb; one device launch each)
    -> SpeechEmbeddings (STFT/mel + speech embedding + NaN replacement)

but the clips never leave HBM between the stages (``generate_device``), and
no child process is spawned per 25,000-clip chunk (the reference isolates a
host memory leak of its CPU/ORT path that this path does not have).

Offline stand-ins (outside the hot path, documented in DESIGN.md §7):
* TTS: Piper needs downloaded weights; ``heybuddy.synthetic.speech_clips``
  renders variable-length tone-syllable utterances per phrase instead.
* The default background / impulse-response datasets are Hugging Face repos
  (constants.py DEFAULT_BACKGROUND_DATASET / DEFAULT_IMPULSE_DATASET); when a
  dataset argument is such a name it is replaced by the synthetic noise / IR
  banks of ``heybuddy.synthetic`` (a warning is logged). Any in-memory audio
  dataset (HF ``Dataset``, list of arrays or {"array", "sampling_rate"} rows)
  is used as given.
"""
from __future__ import annotations

import math
import os
import random
import re
import zlib
from typing import Any, Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from heybuddy.constants import (DEFAULT_ADVERSARIAL_PHRASES, DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
                                DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
                                DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB, DEFAULT_AUGMENT_COLORED_NOISE_PROB,
                                DEFAULT_AUGMENT_GAIN_PROB, DEFAULT_AUGMENT_REVERB_PROB,
                                DEFAULT_AUGMENT_TANH_DISTORTION_PROB, DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
                                DEFAULT_AUGMENT_TANH_MIN_DISTORTION, DEFAULT_EMBEDDING_BATCH_SIZE,
                                DEFAULT_EMBEDDING_SPECTROGRAM_BATCH_SIZE, DEFAULT_FEATURE_BATCH_SIZE,
                                DEFAULT_AUGMENT_BATCH_SIZE, DEFAULT_AUGMENT_BAND_STOP_PROB,
                                DEFAULT_AUGMENT_PHRASE_PROB, DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
                                DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES, DEFAULT_AUGMENT_SAMPLE_RATIO,
                                DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB, DEFAULT_AUGMENT_SEVEN_BAND_PROB,
                                DEFAULT_BACKGROUND_DATASET, DEFAULT_IMPULSE_DATASET, DEFAULT_TTS_BATCH_SIZE)
from heybuddy.dataset.augmented import AugmentedAudioGenerator
from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
from heybuddy.util import logger

__all__ = ["TrainingFeaturesGenerator", "SyntheticSpeechGenerator", "safe_name", "synthetic_negative_features"]

SupplementalDatasetType = Any


def _gather_rows(local: torch.Tensor, n: int) -> torch.Tensor:
    """Every rank's contiguous share [clip_range(n, r, W)] of an [n, ...] device
    tensor, all-gathered (padded to equal sizes: uneven all_gather is not
    portable across backends) -> the whole [n, ...] on every rank."""
    import torch.distributed as dist
    from heybuddy import distributed as hd
    rank, world = hd.world()
    sizes = [b - a for a, b in (hd.clip_range(n, r, world) for r in range(world))]
    m = max(sizes)
    cpu = dist.get_backend() == "gloo"
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device="cpu" if cpu else local.device)
    pad[:local.shape[0]] = local.to(pad.device)
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:k] for b, k in zip(bufs, sizes)]).to(local.device)


def _sharded(fn, n: int) -> np.ndarray:
    """fn(m) -> [m, 16, 96] device features; under torch.distributed every
    rank featurizes its share (numpy's global RNG offset by the rank, so the
    shards differ) and the shares are all-gathered: the result is the same
    [n, 16, 96] array on every rank."""
    from heybuddy import distributed as hd
    rank, world = hd.world()
    if world == 1:
        return fn(n).cpu().numpy()
    lo, hi = hd.clip_range(n, rank, world)
    # every global stream the share draws from (numpy's for placement and the
    # coins, torch's CPU generator for the augmentation parameters, python's)
    # is offset by the rank for the share and restored afterwards: how many
    # draws a rank makes depends on its shard, and whatever runs next (the
    # trainer's parameter init) must see the same state on every rank
    state = np.random.get_state()
    t_state = torch.random.get_rng_state()
    p_state = random.getstate()
    salt = (int(state[1][0]) + 7919 * (rank + 1)) % (2 ** 32)
    np.random.seed(salt)
    torch.random.default_generator.manual_seed(salt)  # CPU only: device generators untouched
    random.seed(salt)
    try:
        local = fn(hi - lo)
    finally:
        np.random.set_state(state)
        torch.random.set_rng_state(t_state)
        random.setstate(p_state)
    return _gather_rows(local, n).cpu().numpy()


def _save_then_open(array: np.ndarray, name: str, directory: str, keep_in_memory: bool = False,
                    **kwargs: Any) -> PrecalculatedDatasetIterator:
    """PrecalculatedDatasetIterator.from_array, written by rank 0 only (every
    rank holds the same array), the other ranks open it after a barrier."""
    from heybuddy import distributed as hd
    rank, world = hd.world()
    if world == 1 or rank == 0:
        it = PrecalculatedDatasetIterator.from_array(array, name=name, directory=directory,
                                                     keep_in_memory=keep_in_memory, **kwargs)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        if rank != 0:
            it = PrecalculatedDatasetIterator(name, directory=directory, data=array if keep_in_memory else None,
                                              **kwargs)
    return it


def synthetic_negative_features(name: str, num_samples: int, device_id: Optional[int] = None, seed: int = 0,
                                directory: Optional[str] = None) -> PrecalculatedDatasetIterator:
    """Offline stand-in for a hosted negative set (precalculated.py:620-649,
    a download): ``num_samples`` synthetic tone-burst clips at 0.3 level
    featurized on the device, stored f16 as ``{directory}/{name}.npy`` (the
    combine --half layout) and reused while large enough."""
    from heybuddy import _native
    from heybuddy.dataset.precalculated import LOCAL_DIR
    from heybuddy.embeddings import SpeechEmbeddings
    from heybuddy.synthetic import synthetic_clips
    directory = directory or LOCAL_DIR
    try:
        it = PrecalculatedDatasetIterator(name, directory=directory)
        if len(it) >= num_samples:
            return it
    except FileNotFoundError:
        pass
    dev = _native.require_device(device_id)
    se = SpeechEmbeddings(device_id=dev.index)
    base = [0]

    def fn(m: int) -> torch.Tensor:
        parts = []
        off = int(np.random.randint(0, 2 ** 30))
        for s in range(0, m, 65536):
            k = min(65536, m - s)
            clips = synthetic_clips(k, seed=seed * 1_000_003 + off + s, device=dev).mul_(0.3)
            parts.append(se.featurize(clips))
        base[0] += m
        return torch.cat(parts) if parts else torch.empty((0, 16, 96), device=dev)

    feats = _sharded(fn, num_samples).astype(np.float16)
    return _save_then_open(feats, name, directory)


def safe_name(name: str) -> str:
    """util/string_util.py:145-151: lower-case, non-alphanumerics -> '_'."""
    return re.sub(r"[^a-z0-9]+", "_", name.lower()).strip("_")


class SyntheticSpeechGenerator:
    """Stands in for PiperSpeechGenerator (dataset/piper.py:16-191): ``(n)``
    yields {"audio": {"array", "sampling_rate"}} utterances of the phrase (or
    of adversarial phrases); ``device_batch(n)`` returns them as one HBM batch
    (clips [n, 24000], lengths)."""

    def __init__(self, phrase: str, adversarial: bool = False, num_adversarial_texts: int = 250,
                 device_id: Optional[int] = None, target_sample_rate: int = 16000, seed: Optional[int] = None,
                 **kwargs: Any) -> None:
        self.phrase = phrase
        self.adversarial = adversarial
        self.num_adversarial_texts = max(1, int(num_adversarial_texts))
        self.device = torch.device("cpu") if device_id is None else torch.device("cuda", device_id)
        self.sample_rate = target_sample_rate
        # not from numpy's global RNG: its stream carries exactly the reference's draws
        self.seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if seed is None else int(seed)

    def device_batch(self, n: int) -> Tuple[torch.Tensor, np.ndarray]:
        from heybuddy.synthetic import speech_clips
        return speech_clips(self.phrase, n, seed=self.seed, device=self.device, adversarial=self.adversarial,
                            num_phrases=self.num_adversarial_texts)

    def __call__(self, n: int):
        clips, lengths = self.device_batch(n)
        host = clips.cpu().numpy()
        for i in range(n):
            yield {"audio": {"array": host[i, :lengths[i]], "sampling_rate": self.sample_rate}}


def _is_hub_name(ds: Any) -> bool:
    if isinstance(ds, str):
        return bool(re.match(r"^[A-Za-z0-9\-_.]+/[A-Za-z0-9\-_.]+$", ds)) and not os.path.exists(ds)
    if isinstance(ds, (list, tuple)):
        return bool(ds) and all(isinstance(d, str) for d in ds)
    return False


class TrainingFeaturesGenerator:
    """Generate a dataset of features (features.py:30-908)."""

    def __init__(self, device_id: Optional[int] = None, use_tqdm: bool = True, use_autoconfigure: bool = True,
                 sample_rate: int = 16000, sample_batch_size: int = DEFAULT_FEATURE_BATCH_SIZE,
                 tts_text: str = "Hello, world!", tts_additional_texts: List[str] = [],
                 tts_adversarial: bool = False, tts_adversarial_num_phrases: int = DEFAULT_ADVERSARIAL_PHRASES,
                 tts_adversarial_custom_phrases: List[str] = [], tts_batch_size: int = DEFAULT_TTS_BATCH_SIZE,
                 tts_phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
                 tts_phrase_augment_words: Sequence[str] = (),
                 augment_target_length: float = 1.44, augment_batch_size: int = DEFAULT_AUGMENT_BATCH_SIZE,
                 augment_sample_ratio: float = DEFAULT_AUGMENT_SAMPLE_RATIO,
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
                 embedding_spectrogram_batch_size: int = DEFAULT_EMBEDDING_SPECTROGRAM_BATCH_SIZE,
                 embedding_batch_size: int = DEFAULT_EMBEDDING_BATCH_SIZE) -> None:
        self.device_id = device_id
        self.use_autoconfigure = use_autoconfigure
        self.use_tqdm = use_tqdm
        self.sample_rate = sample_rate
        self.sample_batch_size = sample_batch_size
        self.tts_text = tts_text
        self.tts_additional_texts = list(tts_additional_texts)
        self.tts_adversarial = tts_adversarial
        self.tts_adversarial_num_phrases = tts_adversarial_num_phrases
        self.tts_adversarial_custom_phrases = list(tts_adversarial_custom_phrases)
        self.tts_batch_size = tts_batch_size
        self.tts_phrase_augment_prob = tts_phrase_augment_prob
        self.tts_phrase_augment_words = list(tts_phrase_augment_words)
        self.augment_target_length = augment_target_length
        self.augment_sample_ratio = augment_sample_ratio
        self.augment_batch_size = augment_batch_size
        self.augment_dataset_streaming = augment_dataset_streaming
        self.augment_background_dataset = augment_background_dataset
        self.augment_impulse_dataset = augment_impulse_dataset
        self.augment_seven_band_prob = augment_seven_band_prob
        self.augment_seven_band_gain_db = augment_seven_band_gain_db
        self.augment_tanh_distortion_prob = augment_tanh_distortion_prob
        self.augment_tanh_min_distortion = augment_tanh_min_distortion
        self.augment_tanh_max_distortion = augment_tanh_max_distortion
        self.augment_pitch_shift_prob = augment_pitch_shift_prob
        self.augment_pitch_shift_semitones = augment_pitch_shift_semitones
        self.augment_band_stop_prob = augment_band_stop_prob
        self.augment_colored_noise_prob = augment_colored_noise_prob
        self.augment_colored_noise_min_snr_db = augment_colored_noise_min_snr_db
        self.augment_colored_noise_max_snr_db = augment_colored_noise_max_snr_db
        self.augment_colored_noise_min_f_decay = augment_colored_noise_min_f_decay
        self.augment_colored_noise_max_f_decay = augment_colored_noise_max_f_decay
        self.augment_background_noise_prob = augment_background_noise_prob
        self.augment_background_noise_min_snr_db = augment_background_noise_min_snr_db
        self.augment_background_noise_max_snr_db = augment_background_noise_max_snr_db
        self.augment_gain_prob = augment_gain_prob
        self.augment_reverb_prob = augment_reverb_prob
        self.embedding_spectrogram_batch_size = embedding_spectrogram_batch_size
        self.embedding_batch_size = embedding_batch_size
        self._augmenters: dict = {}

    @property
    def device(self) -> torch.device:
        from heybuddy import _native
        return _native.require_device(self.device_id)

    def autoconfigure(self) -> None:
        """features.py:171-218 for a GPU with >= 8 GiB: batch sizes 64 / 128 / 128 / 128.
        The MI355X path needs a HIP device (there is no CPU branch)."""
        from heybuddy import _native
        dev = _native.require_device(self.device_id)
        self.device_id = dev.index
        self.tts_batch_size = 64
        self.augment_batch_size = 128
        self.embedding_spectrogram_batch_size = 128
        self.embedding_batch_size = 128

    def get_speech_embeddings_model(self):
        from heybuddy.embeddings import get_speech_embeddings
        return get_speech_embeddings(device_id=self.device.index)

    def get_tts_generator(self) -> SyntheticSpeechGenerator:
        # the stand-in's seed counts the calls (distinct utterances per chunk, and no draw
        # from the RNG states __call__ restores per chunk)
        self._tts_calls = getattr(self, "_tts_calls", 0) + 1
        seed = (zlib.crc32(f"{self.tts_text}|{self.tts_adversarial}".encode()) + 7919 * self._tts_calls) % (2 ** 31 - 1)
        return SyntheticSpeechGenerator(self.tts_text, adversarial=self.tts_adversarial,
                                        num_adversarial_texts=self.tts_adversarial_num_phrases,
                                        device_id=self.device.index, target_sample_rate=self.sample_rate, seed=seed)

    def _bank(self, which: str, testing: bool) -> Any:
        ds = self.augment_background_dataset if which == "noise" else self.augment_impulse_dataset
        if ds is None or not _is_hub_name(ds):
            return ds
        from heybuddy.synthetic import impulse_responses, noise_bank
        logger.warning(f"{which} dataset {ds!r} is a Hugging Face repo (no network): using the synthetic "
                       f"{which} bank of heybuddy.synthetic")
        seed = 1000 + (7 if testing else 0)
        return noise_bank(64, seed=seed) if which == "noise" else impulse_responses(32, seed=seed + 1)

    def get_augmented_generator(self, dataset: Any = None, testing: bool = False) -> AugmentedAudioGenerator:
        key = (testing, self.augment_batch_size)
        if key not in self._augmenters:
            self._augmenters[key] = AugmentedAudioGenerator(
                dataset if dataset is not None else [], device_id=self.device.index,
                batch_size=self.augment_batch_size,
                target_length=self.augment_target_length, sample_rate=self.sample_rate,
                augmentation_dataset=self._bank("noise", testing),
                impulse_response_dataset=self._bank("ir", testing),
                seven_band_aug_prob=self.augment_seven_band_prob,
                seven_band_aug_gain_db=self.augment_seven_band_gain_db,
                tanh_distortion_prob=self.augment_tanh_distortion_prob,
                tanh_min_distortion=self.augment_tanh_min_distortion,
                tanh_max_distortion=self.augment_tanh_max_distortion,
                pitch_shift_prob=self.augment_pitch_shift_prob,
                pitch_shift_semitones=self.augment_pitch_shift_semitones,
                band_stop_prob=self.augment_band_stop_prob,
                colored_noise_prob=self.augment_colored_noise_prob,
                colored_noise_min_snr_db=self.augment_colored_noise_min_snr_db,
                colored_noise_max_snr_db=self.augment_colored_noise_max_snr_db,
                colored_noise_min_f_decay=self.augment_colored_noise_min_f_decay,
                colored_noise_max_f_decay=self.augment_colored_noise_max_f_decay,
                background_noise_prob=self.augment_background_noise_prob,
                background_noise_min_snr_db=self.augment_background_noise_min_snr_db,
                background_noise_max_snr_db=self.augment_background_noise_max_snr_db,
                gain_prob=self.augment_gain_prob, reverb_prob=self.augment_reverb_prob)
        return self._augmenters[key]

    def augment_device(self, clips: torch.Tensor, lengths: np.ndarray, num_samples: int,
                       testing: bool = False, validation: bool = False) -> torch.Tensor:
        """The middle stage of generate (features.py:412-458) on device data:
        n_tts utterances -> num_samples clips of T samples."""
        T = int(self.sample_rate * self.augment_target_length)
        n_tts = clips.shape[0]
        if validation:  # centred pad, no augmentation (:412-427)
            from heybuddy.kernels import place_clips
            lens = np.minimum(lengths, T).astype(np.int32)
            pre = ((T - lens) // 2).astype(np.int32)
            return place_clips(clips, lens, pre, T)
        # a fresh AugmentedAudioGenerator per call in the reference (:434-440): the source
        # rows in order, re-shuffled when they run out; the noise / IR iteration from the start
        aug = self.get_augmented_generator(testing=testing)
        aug.augmenter.noise_idx = aug.augmenter.ir_idx = 0
        rows, pre, coins = aug.plan_source(lengths, num_samples)
        lens = np.asarray(lengths)[rows].astype(np.int32)
        same = num_samples == n_tts and np.array_equal(rows, np.arange(n_tts))
        src = clips if same else clips.index_select(0, torch.from_numpy(rows).to(clips.device))
        prepared = {"lens": lens, "pre": pre, "chain": aug.augmenter.prepare(num_samples, coins)}
        return aug.augment_device(src, lens, prepared=prepared)

    def generate_device(self, num_samples: int, testing: bool = False, validation: bool = False) -> torch.Tensor:
        """features.py:360-490 with every stage in HBM: [num_samples, 16, 96] f32 on the device."""
        if self.use_autoconfigure:
            self.autoconfigure()
        if validation:
            tts_num_samples = num_samples
        else:
            tts_num_samples = max(1, min(num_samples, int(num_samples // self.augment_sample_ratio)))
        clips, lengths = self.get_tts_generator().device_batch(tts_num_samples)
        audio = self.augment_device(clips, lengths, num_samples, testing=testing, validation=validation)
        del clips
        return self.get_speech_embeddings_model().featurize(audio)

    def generate(self, num_samples: int, sample_save_path: Optional[str] = None,
                 augmented_sample_save_path: Optional[str] = None, testing: bool = False,
                 validation: bool = False) -> np.ndarray:
        """Samples -> embeddings [num_samples, 16, 96] (features.py:360-490)."""
        if sample_save_path or augmented_sample_save_path:
            logger.warning("sample wav export needs an audio writer; skipped")
        return self.generate_device(num_samples, testing=testing, validation=validation).cpu().numpy()

    def _chunks(self, num_samples: int, fn: Callable[[int], Any]) -> List[Any]:
        """fn over chunks of sample_batch_size (features.py:492-535). The
        reference runs each chunk in a forked ProcessPoolExecutor worker: every
        chunk starts from the caller's numpy / torch / random states and none
        of its draws reach the caller. The same here: the states are restored
        before each chunk and after the last."""
        sizes = [self.sample_batch_size] * math.ceil(num_samples / self.sample_batch_size)
        if num_samples % self.sample_batch_size:
            sizes[-1] = num_samples % self.sample_batch_size
        states = (np.random.get_state(), torch.random.get_rng_state(), random.getstate())
        parts = []
        try:
            for size in sizes:
                np.random.set_state(states[0])
                torch.random.set_rng_state(states[1])
                random.setstate(states[2])
                parts.append(fn(size))
        finally:
            np.random.set_state(states[0])
            torch.random.set_rng_state(states[1])
            random.setstate(states[2])
        return parts

    def __call__(self, num_samples: int, sample_save_path: Optional[str] = None,
                 augmented_sample_save_path: Optional[str] = None, testing: bool = False,
                 validation: bool = False) -> np.ndarray:
        """Chunks of sample_batch_size, concatenated (features.py:492-535)."""
        parts = self._chunks(num_samples, lambda s: self.generate(s, sample_save_path, augmented_sample_save_path,
                                                                 testing, validation))
        return parts[0] if len(parts) == 1 else np.concatenate(parts)

    def call_device(self, num_samples: int, testing: bool = False, validation: bool = False) -> torch.Tensor:
        """__call__ without the host copy: [num_samples, 16, 96] f32 in HBM."""
        parts = self._chunks(num_samples, lambda s: self.generate_device(s, testing=testing, validation=validation))
        if not parts:
            return torch.empty((0, 16, 96), dtype=torch.float32, device=self.device)
        return parts[0] if len(parts) == 1 else torch.cat(parts)

    @classmethod
    def default(cls, wake_phrase: str, adversarial: bool = False, num_adversarial_phrases: int = 10,
                additional_wake_phrases: List[str] = [], custom_adversarial_phrases: List[str] = [],
                dataset_streaming: bool = False, tts_batch_size: int = DEFAULT_TTS_BATCH_SIZE,
                phrase_augment_prob: float = DEFAULT_AUGMENT_PHRASE_PROB,
                phrase_augment_words: Sequence[str] = (), augment_target_length: float = 1.44,
                augment_background_dataset: SupplementalDatasetType = DEFAULT_BACKGROUND_DATASET,
                augment_impulse_dataset: SupplementalDatasetType = DEFAULT_IMPULSE_DATASET,
                **kwargs: Any) -> "TrainingFeaturesGenerator":
        """features.py:537-616 (augment_* / embedding_* keywords pass through)."""
        kwargs.pop("use_cache", None)
        if augment_background_dataset is None:
            augment_background_dataset = DEFAULT_BACKGROUND_DATASET
        if augment_impulse_dataset is None:
            augment_impulse_dataset = DEFAULT_IMPULSE_DATASET
        return cls(use_autoconfigure=True, tts_text=wake_phrase, tts_adversarial=adversarial,
                   tts_batch_size=tts_batch_size, tts_adversarial_num_phrases=num_adversarial_phrases,
                   tts_adversarial_custom_phrases=custom_adversarial_phrases,
                   tts_additional_texts=additional_wake_phrases, tts_phrase_augment_prob=phrase_augment_prob,
                   tts_phrase_augment_words=phrase_augment_words,
                   augment_background_dataset=augment_background_dataset,
                   augment_impulse_dataset=augment_impulse_dataset, augment_target_length=augment_target_length,
                   **kwargs)

    @classmethod
    def get_wake_phrase_file_name(cls, wake_phrase: str, testing: bool = False) -> str:
        return safe_name(wake_phrase).strip("_") + ("_tst" if testing else "")

    @classmethod
    def get_training_features(cls, wake_phrase: str, num_positive_samples: int, num_adversarial_samples: int,
                              num_adversarial_phrases: int = 10, additional_wake_phrases: List[str] = [],
                              custom_adversarial_phrases: List[str] = [], testing: bool = False,
                              use_cache: bool = True, save_samples: bool = True, keep_in_memory: bool = False,
                              directory: Optional[str] = None, device_id: Optional[int] = None, **kwargs: Any
                              ) -> Tuple[PrecalculatedDatasetIterator, PrecalculatedDatasetIterator]:
        """Positive and adversarial feature sets for a phrase, cached by name
        (``{name}.npy``, ``{name}_adv.npy``) and topped up when the cache is
        short (features.py:618-837). Under torch.distributed each rank
        featurizes its share of the missing rows; rank 0 writes the cache."""
        from heybuddy.dataset.precalculated import LOCAL_DIR
        directory = directory or LOCAL_DIR
        name = cls.get_wake_phrase_file_name(wake_phrase, testing=testing)
        out = []
        for suffix, adversarial, n in (("", False, num_positive_samples), ("_adv", True, num_adversarial_samples)):
            it_name = name + suffix
            existing = None
            if use_cache:
                try:
                    existing = PrecalculatedDatasetIterator(it_name, directory=directory)
                except FileNotFoundError:
                    existing = None
            have = len(existing) if existing is not None else 0
            if existing is not None and have >= n:
                out.append(existing)
                continue
            gen = cls.default(wake_phrase, adversarial=adversarial, num_adversarial_phrases=num_adversarial_phrases,
                              additional_wake_phrases=additional_wake_phrases,
                              custom_adversarial_phrases=custom_adversarial_phrases, device_id=device_id, **kwargs)
            feats = _sharded(lambda m: gen.call_device(m, testing=testing), n - have)
            if have:
                feats = np.concatenate([np.asarray(existing.precalculated), feats])
            out.append(_save_then_open(feats, it_name, directory, keep_in_memory=keep_in_memory))
        return out[0], out[1]

    @classmethod
    def get_validation_features(cls, wake_phrase: str, num_positive_samples: int, use_cache: bool = True,
                                keep_in_memory: bool = False, augment_target_length: float = 1.44,
                                directory: Optional[str] = None, device_id: Optional[int] = None,
                                **kwargs: Any) -> PrecalculatedDatasetIterator:
        """Un-augmented, centre-padded positive features (features.py:840-908)."""
        from heybuddy.dataset.precalculated import LOCAL_DIR
        directory = directory or LOCAL_DIR
        name = cls.get_wake_phrase_file_name(wake_phrase) + "_val"
        existing = None
        if use_cache:
            try:
                existing = PrecalculatedDatasetIterator(name, directory=directory)
            except FileNotFoundError:
                existing = None
        have = len(existing) if existing is not None else 0
        if existing is not None and have >= num_positive_samples:
            return existing
        gen = cls.default(wake_phrase, augment_target_length=augment_target_length, device_id=device_id)
        feats = _sharded(lambda m: gen.call_device(m, validation=True), num_positive_samples - have)
        if have:
            feats = np.concatenate([np.asarray(existing.precalculated), feats])
        return _save_then_open(feats, name, directory, keep_in_memory=keep_in_memory)
