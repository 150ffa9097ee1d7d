"""TrainingFeaturesGenerator on the device (reference
dataset/features.py:360-535, :628-908) against the oracle composition.

The generator's inputs are recorded as it runs (the TTS stand-in's clips and
the source rows and placement offsets it draws from numpy's global RNG), and
the expected features are recomputed from them on the host: to_target_length
placement (augmented.py:200-232) of the recorded source row (in order, then
re-shuffled when the utterances run out: the augment_sample_ratio wrap of
features.py:430-446; the draws themselves are pinned against a reference run
in test_drivers_reference.py), then oracle.featurizer.featurize (the
reference's SpeechEmbeddings.__call__ orchestration with the oracle mel /
embedding; embeddings.py:153-234). Checked: chunking by sample_batch_size
(features.py:492-535), the wrap, placement, featurization and the row order
of the concatenated chunks; validation features are centre-padded and
un-augmented (features.py:840-908); the phrase cache is topped up, not
regenerated (features.py:686-760). Augmentations are switched off here (each
has its own parity test); tolerance 1e-4 (1 + |ref|), the featurizer's bound.
"""
import numpy as np
import pytest
import torch

from oracle import featurizer as ofeat

pytestmark = pytest.mark.gpu
T = 23040
OFF = dict(augment_seven_band_prob=0.0, augment_tanh_distortion_prob=0.0, augment_pitch_shift_prob=0.0,
           augment_band_stop_prob=0.0, augment_colored_noise_prob=0.0, augment_background_noise_prob=0.0,
           augment_gain_prob=0.0, augment_reverb_prob=0.0)


def _record(monkeypatch):
    from heybuddy.dataset import augmented as A
    from heybuddy.dataset import features as F
    rec = {"tts": [], "pre": [], "rows": []}
    real_batch = F.SyntheticSpeechGenerator.device_batch
    real_off = A.target_length_offsets
    real_plan = A.source_plan

    def plan(*a, **k):
        out = real_plan(*a, **k)
        rec["rows"].append(out[0].copy())
        return out

    def device_batch(self, n):
        clips, lens = real_batch(self, n)
        rec["tts"].append((clips.cpu().numpy(), np.asarray(lens).copy()))
        return clips, lens

    def offsets(lengths, target):
        pre = real_off(lengths, target)
        rec["pre"].append(pre.copy())
        return pre

    monkeypatch.setattr(F.SyntheticSpeechGenerator, "device_batch", device_batch)
    monkeypatch.setattr(A, "target_length_offsets", offsets)
    monkeypatch.setattr(A, "source_plan", plan)
    return rec


def _place(clip, length, pre):
    out = np.zeros(T, np.float32)
    L = min(int(length), T - int(pre))
    out[pre:pre + L] = clip[:L]
    return out


def _check(got, expected_audio, rows):
    from heybuddy.embeddings import default_graph
    ref = ofeat.featurize(expected_audio[rows], default_graph())
    err = (np.abs(got[rows] - ref) / (1.0 + np.abs(ref))).max()
    assert err <= 1e-4, err


def test_feature_generator_chunks_wrap_and_placement(monkeypatch):
    from heybuddy.dataset.features import TrainingFeaturesGenerator
    rec = _record(monkeypatch)
    gen = TrainingFeaturesGenerator(device_id=0, tts_text="hey buddy", sample_batch_size=48,
                                    augment_sample_ratio=2.0, **OFF)
    np.random.seed(11)
    got = gen(110)                                  # chunks 48, 48, 14 -> 24, 24, 7 utterances
    assert got.shape == (110, 16, 96) and got.dtype == np.float32
    assert [c.shape[0] for c, _ in rec["tts"]] == [24, 24, 7]
    audio = []
    for (clips, lens), pre, idx, m in zip(rec["tts"], rec["pre"], rec["rows"], (48, 48, 14)):
        assert pre.shape == (m,) and idx.shape == (m,)
        n_tts = clips.shape[0]
        assert (idx[:n_tts] == np.arange(n_tts)).all()        # the first pass in order
        if m >= 2 * n_tts:                                      # then a permutation of the utterances
            assert sorted(idx[n_tts:2 * n_tts].tolist()) == list(range(n_tts))
        audio += [_place(clips[j], lens[j], pre[i]) for i, j in enumerate(idx)]
    audio = np.stack(audio)
    _check(got, audio, [0, 5, 23, 24, 47, 48, 60, 95, 96, 101, 109])


def test_validation_features_centre_padded(monkeypatch):
    from heybuddy.dataset.features import TrainingFeaturesGenerator
    rec = _record(monkeypatch)
    gen = TrainingFeaturesGenerator(device_id=0, tts_text="hey buddy", sample_batch_size=64, **OFF)
    np.random.seed(12)
    got = gen(40, validation=True)
    clips, lens = rec["tts"][0]
    assert clips.shape[0] == 40 and not rec["pre"]  # no random placement draw
    lens = np.minimum(lens, T)
    audio = np.stack([_place(clips[i], lens[i], (T - lens[i]) // 2) for i in range(40)])
    _check(got, audio, [0, 13, 39])


def test_training_features_cache_top_up(tmp_path, monkeypatch):
    from heybuddy.dataset.features import TrainingFeaturesGenerator
    np.random.seed(13)
    kw = dict(directory=str(tmp_path), device_id=0, **OFF)
    pos, adv = TrainingFeaturesGenerator.get_training_features("hey buddy", 30, 20, **kw)
    assert (len(pos), len(adv)) == (30, 20)
    first = np.array(pos.precalculated)
    pos2, adv2 = TrainingFeaturesGenerator.get_training_features("hey buddy", 50, 20, **kw)
    assert len(pos2) == 50 and len(adv2) == 20
    np.testing.assert_array_equal(np.asarray(pos2.precalculated)[:30], first)   # topped up, not regenerated
    assert torch.isfinite(torch.from_numpy(np.asarray(pos2.precalculated))).all()
