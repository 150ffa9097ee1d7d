"""Clip placement: AugmentedAudioGenerator.to_target_length (reference
dataset/augmented.py:200-232) against the reference's own outputs with numpy's
global RNG seeded (tests/golden/to_target_length.npz, made by
oracle/golden_classifier.py:make_to_target_length). Bit-exact: it is a copy
with a random offset. The device path (hbk_place_clips) takes the offsets from
one vectorised draw (target_length_offsets) that must reproduce the
reference's per-clip draws and leave the RNG where the reference leaves it."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "to_target_length.npz")
T = 23040


def _inputs():
    g = np.load(GOLD)
    n = len([k for k in g.files if k.startswith("in")])
    return g, [g[f"in{i}"] for i in range(n)], [g[f"out{i}"] for i in range(n)]


def test_host_to_target_length_bit_exact():
    from heybuddy.dataset.augmented import to_target_length
    g, ins, outs = _inputs()
    np.random.seed(2024)
    for a, ref in zip(ins, outs):
        got = to_target_length(a.copy(), T)
        assert got.dtype == ref.dtype and got.shape == ref.shape
        np.testing.assert_array_equal(got, ref)
    assert np.random.rand() == float(g["rng_after"])


def test_vectorised_offsets_match_reference_draws():
    from heybuddy.dataset.augmented import target_length_offsets
    g, ins, outs = _inputs()
    np.random.seed(2024)
    pre = target_length_offsets([a.shape[0] for a in ins], T)
    assert np.random.rand() == float(g["rng_after"])
    for a, ref, p in zip(ins, outs, pre):
        n = min(a.shape[0], T)
        if a.dtype == np.int16:
            assert np.array_equal(ref[p:p + n], a[:n].astype(np.float32) / 32768.0)
        else:
            assert np.array_equal(ref[p:p + n], a[:n])
        assert not ref[:p].any() and not ref[p + n:].any()


@pytest.mark.gpu
def test_device_placement_bit_exact():
    from heybuddy.dataset.augmented import target_length_offsets
    from heybuddy.kernels import place_clips
    g, ins, outs = _inputs()
    width = max(a.shape[0] for a in ins)
    src = torch.zeros((len(ins), width), dtype=torch.float32)
    for i, a in enumerate(ins):
        v = a.astype(np.float32) / 32768.0 if a.dtype == np.int16 else a
        src[i, :a.shape[0]] = torch.from_numpy(v)
    lens = np.array([a.shape[0] for a in ins])
    np.random.seed(2024)
    pre = target_length_offsets(lens, T)
    out = place_clips(src.cuda(), lens, pre, T).cpu().numpy()
    for i, ref in enumerate(outs):
        np.testing.assert_array_equal(out[i], ref.astype(np.float32), err_msg=str(i))


@pytest.mark.gpu
def test_augmented_generator_batch_surface():
    """AugmentedAudioGenerator(...)(n) yields the reference's dicts of placed,
    augmented 23,040-sample clips (probabilities 0: exactly the placement)."""
    from heybuddy.dataset.augmented import AugmentedAudioGenerator
    g, ins, outs = _inputs()
    rows = [{"audio": {"array": a, "sampling_rate": 16000}, "id": i} for i, a in enumerate(ins)]
    gen = AugmentedAudioGenerator(rows, device_id=0, batch_size=16, background_noise_prob=0.0, reverb_prob=0.0,
                                  gain_prob=0.0, colored_noise_prob=0.0, tanh_distortion_prob=0.0,
                                  seven_band_aug_prob=0.0, pitch_shift_prob=0.0, band_stop_prob=0.0)
    np.random.seed(2024)
    items = list(gen(len(rows)))
    assert [it["id"] for it in items] == list(range(len(rows)))
    for it, ref in zip(items, outs):
        assert it["audio"]["sampling_rate"] == 16000
        np.testing.assert_array_equal(it["audio"]["array"], ref.astype(np.float32))
