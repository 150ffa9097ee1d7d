"""Reference runs of the two dataset drivers (TEST INFRASTRUCTURE ONLY; called
by oracle/make_golden.py --only drivers, where /root/reference exists).

extract_driver.npz  PrecalculatedTrainingDatasetGenerator.__call__ and the
                    labeled variant (ref dataset/precalculated.py:114-270,
                    :280-374) on synthetic datasets, with an index-encoding
                    featurizer (a window's samples ARE its embedding rows; a
                    window holding a NaN gives a NaN row). Pins file
                    boundaries, file names, row order, NaN drops, the
                    max_hours cut and the token rows. Small windows
                    (seconds_per_batch 0.05 = 800 samples) keep it tiny.
extract_numeric.npz the same driver at the reference's 1.44-s windows with the
                    oracle mel + SE20 stand-in embedding injected into its
                    SpeechEmbeddings (the HIP test featurizes the same
                    dataset on the device).
features_driver.npz TrainingFeaturesGenerator.__call__ (ref dataset/features.py
                    :360-535) with every augmentation probability 0, a
                    deterministic stand-in TTS, and the oracle featurizer:
                    chunks of sample_batch_size, the augment_sample_ratio
                    wrap (the source dataset re-shuffled by
                    datasets.Dataset.shuffle() when it runs out), the
                    to_target_length draws, the per-batch background / reverb
                    coins, validation's centre padding. The reference runs each
                    chunk in a forked ProcessPoolExecutor worker; the stand-in
                    executor runs it in process from the parent's numpy /
                    torch / random states and restores them afterwards (what
                    fork does). Records each chunk's source rows and leading
                    silences and the features.

The datasets and the stand-in TTS come from the generators below (seeded
numpy Generators), which the tests import to rebuild the same inputs.
"""
from __future__ import annotations

import os
import random
import shutil
import sys
import tempfile
import types
from concurrent.futures import Future

import numpy as np

SR = 16000
T = 23040


# ---------------------------------------------------------------- shared inputs
def extract_dataset(case: str):
    """Rows {"audio": {"array", "sampling_rate"}, "transcript"} of an extract
    case (fresh dicts on every call: the reference pops the audio key)."""
    rng = np.random.default_rng({"basic": 11, "cut": 12, "labeled": 13, "numeric": 14}[case])
    if case == "numeric":
        lens = [30000, 10000, 50000, 23040, 7000]
        win = None
    else:
        lens = [100, 799, 800, 801, 2500, 1600, 350, 4100, 60]
        win = 800
    words = ["hey", "buddy", "hello", "world", "okay"]
    rows = []
    for i, n in enumerate(lens):
        x = (0.3 * rng.standard_normal(n)).astype(np.float32)
        if case == "basic" and i == 4:
            x[win + 17] = np.nan          # the second window of clip 4 becomes a NaN row
        if case == "cut" and i == 7:
            x[3 * win + 5] = np.nan
        rows.append({"audio": {"array": x, "sampling_rate": SR},
                     "transcript": " ".join(words[(i + j) % 5] for j in range(1 + i % 3))})
    return rows


EXTRACT_CASES = {  # case -> (process_batch_size, samples_per_file, max_hours, seconds_per_batch, labeled)
    "basic": (4, 10, 1000.0, 0.05, False),
    "cut": (3, 4, 3.5 * 3 * 0.05 / 3600.0, 0.05, False),   # int(3.5) = 3 process batches
    "labeled": (4, 6, 1000.0, 0.05, True),
    "numeric": (2, 3, 1000.0, 1.44, False),
}


def index_embeddings(windows) -> np.ndarray:
    """The index-encoding featurizer: window w's samples, zero-padded to 1536,
    as its [16, 96] rows (a NaN sample stays a NaN)."""
    out = np.zeros((len(windows), 16 * 96), dtype=np.float32)
    for i, w in enumerate(windows):
        w = np.asarray(w, dtype=np.float32).reshape(-1)
        out[i, :w.shape[0]] = w
    return out.reshape(-1, 16, 96)


def token_ids(text: str, length: int = 96) -> np.ndarray:
    """Stand-in tokenizer: character codes, zero-padded to ``length``."""
    ids = np.zeros(length, dtype=np.float32)
    codes = [float(ord(c)) for c in text][:length]
    ids[:len(codes)] = codes
    return ids


def tts_clips(call: int, n: int):
    """The stand-in TTS's ``call``-th batch of n utterances (float32, 16 kHz):
    lengths 0.4-1.6 s (some longer than T: cropped, no draw), one of T - 1
    samples (total silence 1: no draw), every clip starting with a non-zero
    sample (so the leading silence is observable)."""
    rng = np.random.default_rng(1000 + call)
    lens = rng.integers(6400, 25600, n)
    if n > 1:
        lens[1] = T - 1
    clips = []
    for m in lens:
        t = np.arange(m) / SR
        f = rng.uniform(150, 600)
        x = 0.3 * np.sin(2 * np.pi * f * t) * np.hanning(m) + 0.02 * rng.standard_normal(m)
        x[0] = 0.05
        clips.append(x.astype(np.float32))
    return clips


FEATURES = dict(num_samples=21, sample_batch_size=8, augment_batch_size=3, augment_sample_ratio=2.0,
                validation_samples=6, seed=2024)
PROBS_OFF = dict(augment_seven_band_prob=0.0, augment_tanh_distortion_prob=0.0, augment_pitch_shift_prob=0.0,
                 augment_band_stop_prob=0.0, augment_colored_noise_prob=0.0, augment_background_noise_prob=0.0,
                 augment_gain_prob=0.0, augment_reverb_prob=0.0)


# ---------------------------------------------------------------- reference runs
class _ForkExecutor:
    """ProcessPoolExecutor stand-in with fork semantics for the RNG states."""

    def __init__(self, *a, **k):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def submit(self, fn, *args, **kwargs):
        import torch
        states = (np.random.get_state(), torch.random.get_rng_state(), random.getstate())
        fut = Future()
        try:
            fut.set_result(fn(*args, **kwargs))
        finally:
            np.random.set_state(states[0])
            torch.random.set_rng_state(states[1])
            random.setstate(states[2])
        return fut


def _oracle_speech_embeddings(hb):
    from heybuddy.embeddings import default_graph
    from oracle import embed as oemb
    from oracle import mel as omel
    se = hb.embeddings.SpeechEmbeddings()
    g = default_graph()
    se.spectrogram = lambda a: omel.mel_spectrogram_model(a)
    se.embeddings = lambda w: oemb.speech_embedding_model(g, w)
    return se


def make_extract(hb, golden: str) -> None:
    import datasets
    pc = hb.dataset.precalculated
    res = {}
    real_load = datasets.load_dataset
    try:
        for case, (pbs, spf, hours, spb, labeled) in EXTRACT_CASES.items():
            datasets.load_dataset = lambda *a, _c=case, **k: iter(extract_dataset(_c))
            cls = pc.PrecalculatedLabeledTrainingDatasetGenerator if labeled else pc.PrecalculatedTrainingDatasetGenerator
            gen = cls(dataset_path="synthetic/extract", process_batch_size=pbs, seconds_per_batch=spb,
                      sample_rate=SR)
            if case == "numeric":
                gen._speech_embeddings = _oracle_speech_embeddings(hb)
            else:
                gen._speech_embeddings = (lambda audio, spectrogram_batch_size=None, embedding_batch_size=None,
                                          remove_nan=True: index_embeddings(audio))
            if labeled:
                import torch

                class _Tok:
                    def __call__(self, text):
                        return torch.from_numpy(token_ids(text))
                gen._tokenizer = _Tok()
            out = tempfile.mkdtemp(prefix="hbx_")
            try:
                gen(case, output_dir=out, max_hours=hours, samples_per_file=spf)
                names = sorted(os.listdir(os.path.join(out, case)))
                arrays = [np.load(os.path.join(out, case, f)) for f in names]
            finally:
                shutil.rmtree(out, ignore_errors=True)
            res[f"{case}_names"] = np.array(names)
            res[f"{case}_rows"] = np.array([a.shape[0] for a in arrays])
            res[f"{case}_data"] = np.concatenate(arrays) if arrays else np.zeros((0, 16, 96), np.float32)
    finally:
        datasets.load_dataset = real_load
    numeric = {k: v for k, v in res.items() if k.startswith("numeric_")}
    driver = {k: v for k, v in res.items() if not k.startswith("numeric_")}
    np.savez_compressed(os.path.join(golden, "extract_driver.npz"), **driver)
    np.savez_compressed(os.path.join(golden, "extract_numeric.npz"), **numeric)
    print("extract fixtures written:", {k: v.shape for k, v in res.items() if k.endswith("_rows")})


def _stub_augmentation_libraries():
    """audiomentations / torch_audiomentations are not installed: at
    probability 0 their Compose returns the input unchanged (and draws from
    numpy nothing), which is all the reference run needs."""
    class _Compose:
        def __init__(self, transforms=None, **k):
            self.transforms = transforms

        def __call__(self, samples, sample_rate=None, **k):
            return samples

    class _T:
        def __init__(self, *a, p=0.0, **k):
            assert p == 0.0, "the reference run is made with every augmentation off"
    am = types.ModuleType("audiomentations")
    tam = types.ModuleType("torch_audiomentations")
    for m in (am, tam):
        m.Compose = _Compose
    for name in ("SevenBandParametricEQ", "TanhDistortion"):
        setattr(am, name, _T)
    for name in ("PitchShift", "BandStopFilter", "AddColoredNoise", "Gain"):
        setattr(tam, name, _T)
    sys.modules["audiomentations"] = am
    sys.modules["torch_audiomentations"] = tam


def make_features(hb, golden: str) -> None:
    import torch
    _stub_augmentation_libraries()
    fmod = hb.dataset.features
    amod = hb.dataset.augmented
    fmod.ProcessPoolExecutor = _ForkExecutor
    cfg = FEATURES
    rec = {"rows": [], "pre": [], "calls": 0}
    ids = {}

    class _TTS:
        def __call__(self, n):
            clips = tts_clips(rec["calls"], n)
            rec["calls"] += 1
            ids.clear()
            for j, c in enumerate(clips):
                ids[c[:8].tobytes() + np.int64(c.shape[0]).tobytes()] = j
            for c in clips:
                yield {"audio": {"array": c, "sampling_rate": SR}}

    real_next = amod.AugmentedAudioGenerator.get_next_audio_sample_dict
    real_place = amod.AugmentedAudioGenerator.to_target_length

    def next_dict(self):
        item = real_next(self)
        a = np.asarray(item["audio"]["array"], dtype=np.float32)
        rec["rows"].append(ids[a[:8].tobytes() + np.int64(a.shape[0]).tobytes()])
        return item

    def place(self, audio):
        out = real_place(self, audio)
        n = np.asarray(audio).shape[0]
        rec["pre"].append(int(np.argmax(out != 0)) if n < T else 0)
        return out
    amod.AugmentedAudioGenerator.get_next_audio_sample_dict = next_dict
    amod.AugmentedAudioGenerator.to_target_length = place
    se = _oracle_speech_embeddings(hb)
    res = {}
    try:
        for mode in ("train", "validation"):
            gen = fmod.TrainingFeaturesGenerator(
                use_tqdm=False, use_autoconfigure=False, sample_batch_size=cfg["sample_batch_size"],
                tts_text="hey buddy", augment_batch_size=cfg["augment_batch_size"],
                augment_sample_ratio=cfg["augment_sample_ratio"], augment_background_dataset=None,
                augment_impulse_dataset=None, **PROBS_OFF)
            gen.get_tts_generator = lambda: _TTS()
            gen.get_speech_embeddings_model = lambda: se
            rec.update(rows=[], pre=[], calls=0)
            np.random.seed(cfg["seed"])
            torch.manual_seed(cfg["seed"])
            n = cfg["num_samples"] if mode == "train" else cfg["validation_samples"]
            feats = gen(n, validation=(mode == "validation"))
            after = np.random.get_state()[1][:4].copy()
            res[f"{mode}_features"] = np.asarray(feats, dtype=np.float32)
            res[f"{mode}_rows"] = np.array(rec["rows"], dtype=np.int64)
            res[f"{mode}_pre"] = np.array(rec["pre"], dtype=np.int64)
            res[f"{mode}_rng_after"] = after
    finally:
        amod.AugmentedAudioGenerator.get_next_audio_sample_dict = real_next
        amod.AugmentedAudioGenerator.to_target_length = real_place
    res["seed"] = np.array(cfg["seed"])
    np.savez_compressed(os.path.join(golden, "features_driver.npz"), **res)
    print("features fixture written:", {k: v.shape for k, v in res.items()})
