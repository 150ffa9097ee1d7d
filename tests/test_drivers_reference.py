"""The two dataset drivers against runs of the REFERENCE itself
(tests/golden/{extract_driver,extract_numeric,features_driver}.npz, made by
oracle/make_golden.py --only drivers; see oracle/golden_drivers.py).

CPU (driver logic, bit-exact):
  * PrecalculatedTrainingDatasetGenerator.__call__ / the labeled variant (ref
    dataset/precalculated.py:114-270, :280-374) with the same index-encoding
    featurizer: file names, file boundaries, row order, NaN drops, the
    max_hours cut, token rows.
  * TrainingFeaturesGenerator.__call__'s numpy draws (ref dataset/features.py
    :360-535 -> augmented.py:148-162, :200-232, :370-392): per chunk (each
    from the caller's RNG state, as the reference's forked workers), the
    source rows (re-shuffled by datasets' shuffle() when they run out) and
    every clip's leading silence, in the reference's order; the caller's
    numpy state is left as it was.
GPU (numerics through the HIP featurizer, 1e-4 (1 + |ref|) as the
featurizer tests): the feature generator's training and validation features
and the extract driver's 1.44-s windows against the reference runs with the
oracle mel + SE20 stand-in injected.
"""
import os

import numpy as np
import pytest
import torch

from oracle import golden_drivers as gd

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _same(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    np.testing.assert_array_equal(np.nan_to_num(a), np.nan_to_num(b))


def _run_extract(tmp_path, case, device_id=None):
    from heybuddy.dataset.precalculated import (PrecalculatedLabeledTrainingDatasetGenerator,
                                                PrecalculatedTrainingDatasetGenerator)
    pbs, spf, hours, spb, labeled = gd.EXTRACT_CASES[case]
    if labeled:
        gen = PrecalculatedLabeledTrainingDatasetGenerator("synthetic/extract", process_batch_size=pbs,
                                                           seconds_per_batch=spb, sample_rate=gd.SR,
                                                           tokenizer=gd.token_ids, device_id=device_id)
    else:
        gen = PrecalculatedTrainingDatasetGenerator("synthetic/extract", process_batch_size=pbs,
                                                    seconds_per_batch=spb, sample_rate=gd.SR, device_id=device_id)
    if device_id is None:
        gen._featurize = gd.index_embeddings
    files = gen(case, output_dir=str(tmp_path), max_hours=hours, samples_per_file=spf,
                dataset=gd.extract_dataset(case))
    names = [os.path.basename(f) for f in files]
    assert names == sorted(os.listdir(os.path.join(tmp_path, case)))
    return names, [np.load(f) for f in files]


@pytest.mark.parametrize("case", ["basic", "cut", "labeled"])
def test_extract_driver_matches_reference(tmp_path, case):
    ref = np.load(os.path.join(GOLDEN, "extract_driver.npz"))
    names, arrays = _run_extract(tmp_path, case)
    assert names == list(ref[f"{case}_names"])
    assert [a.shape[0] for a in arrays] == list(ref[f"{case}_rows"])
    _same(np.concatenate(arrays), ref[f"{case}_data"])


def _tts_lengths(call, n):
    return [c.shape[0] for c in gd.tts_clips(call, n)]


def test_feature_generator_draws_match_reference():
    from heybuddy.dataset.augmented import source_plan
    from heybuddy.dataset.features import TrainingFeaturesGenerator
    ref = np.load(os.path.join(GOLDEN, "features_driver.npz"))
    cfg = gd.FEATURES
    gen = TrainingFeaturesGenerator(use_tqdm=False, use_autoconfigure=False,
                                    sample_batch_size=cfg["sample_batch_size"],
                                    augment_batch_size=cfg["augment_batch_size"],
                                    augment_sample_ratio=cfg["augment_sample_ratio"], **gd.PROBS_OFF)
    calls, rows, pres = [0], [], []

    def plan(n):  # generate()'s host draws (features.py:375-440), no device
        tts_n = max(1, min(n, int(n // gen.augment_sample_ratio)))
        lens = _tts_lengths(calls[0], tts_n)
        calls[0] += 1
        r, p, _ = source_plan(lens, n, gen.augment_batch_size, int(gen.augment_target_length * gd.SR))
        rows.append(r)
        pres.append(p)

    np.random.seed(cfg["seed"])
    gen._chunks(cfg["num_samples"], plan)
    np.testing.assert_array_equal(np.concatenate(rows), ref["train_rows"])
    np.testing.assert_array_equal(np.concatenate(pres), ref["train_pre"])
    np.testing.assert_array_equal(np.random.get_state()[1][:4], ref["train_rng_after"])


def test_source_order_reshuffles_like_datasets():
    """SourceOrder's re-shuffle = datasets.Dataset.shuffle() with numpy's
    global state (the installed datasets library itself as the check)."""
    import datasets
    from heybuddy.dataset.augmented import SourceOrder
    np.random.seed(5)
    ds = datasets.Dataset.from_dict({"i": list(range(7))})
    expect = list(range(7)) + [r["i"] for r in ds.shuffle()] + [r["i"] for r in ds.shuffle()]
    after = np.random.get_state()[1][:4].copy()
    np.random.seed(5)
    got = SourceOrder(7).take(21)
    assert got.tolist() == expect
    np.testing.assert_array_equal(np.random.get_state()[1][:4], after)


@pytest.fixture
def _device_tts(monkeypatch):
    from heybuddy.dataset import features as F
    calls = [0]

    def device_batch(self, n):
        clips = gd.tts_clips(calls[0], n)
        calls[0] += 1
        lens = np.array([c.shape[0] for c in clips])
        host = np.zeros((n, int(lens.max())), np.float32)
        for i, c in enumerate(clips):
            host[i, :c.shape[0]] = c
        return torch.from_numpy(host).to(self.device), lens

    monkeypatch.setattr(F.SyntheticSpeechGenerator, "device_batch", device_batch)
    return calls


def _close(got, ref):
    err = (np.abs(got - ref) / (1.0 + np.abs(ref))).max()
    assert err <= 1e-4, err


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["train", "validation"])
def test_feature_generator_matches_reference_run(_device_tts, mode):
    from heybuddy.dataset.features import TrainingFeaturesGenerator
    ref = np.load(os.path.join(GOLDEN, "features_driver.npz"))
    cfg = gd.FEATURES
    gen = TrainingFeaturesGenerator(device_id=0, use_tqdm=False, use_autoconfigure=False,
                                    sample_batch_size=cfg["sample_batch_size"], tts_text="hey buddy",
                                    augment_batch_size=cfg["augment_batch_size"],
                                    augment_sample_ratio=cfg["augment_sample_ratio"], **gd.PROBS_OFF)
    np.random.seed(cfg["seed"])
    torch.manual_seed(cfg["seed"])
    n = cfg["num_samples"] if mode == "train" else cfg["validation_samples"]
    got = gen(n, validation=(mode == "validation"))
    assert got.shape == ref[f"{mode}_features"].shape
    _close(got, ref[f"{mode}_features"])
    np.testing.assert_array_equal(np.random.get_state()[1][:4], ref[f"{mode}_rng_after"])


@pytest.mark.gpu
def test_extract_numeric_matches_reference_run(tmp_path):
    ref = np.load(os.path.join(GOLDEN, "extract_numeric.npz"))
    names, arrays = _run_extract(tmp_path, "numeric", device_id=0)
    assert names == list(ref["numeric_names"])
    assert [a.shape[0] for a in arrays] == list(ref["numeric_rows"])
    _close(np.concatenate(arrays), ref["numeric_data"])
