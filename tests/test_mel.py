"""STFT + mel: oracle checks (CPU) and HIP kernel parity (GPU).

Tolerance (north star): mel features within 1e-4 fp32 of the oracle. That
bound holds for every bin of realistic clips (synthetic speech-like clips
with a noise floor). For DC / pure-tone / impulse edge clips, bins far below
the frame's energy sit under the fp32 FFT noise floor; those are checked
against ``oracle.mel.fp32_noise_tolerance`` (1e-4 + the achievable fp32
resolution), see DESIGN.md §Parity.
"""
import math

import numpy as np
import pytest
import torch

from oracle import mel as omel


def test_frame_count_matches_reference_formula():
    # embeddings.py:67 n_frames = ceil(t/160 - 3) for the 17,280-sample windows
    for t in (17280, 12640):
        assert omel.n_frames_for(t) == int(math.ceil(t / 160 - 3))
    assert omel.n_frames_for(17280) == 105        # test_embeddings.py: 105 -> truncated 100
    assert omel.n_frames_for(12640) == 76         # mel-spectrogram.js:37-49
    assert omel.n_frames_for(23040) == 141        # unique frames per 1.44 s clip
    assert omel.n_frames_for(24000) == 147


def test_fbank_shape_and_support():
    fb = omel.mel_fbank()
    assert fb.shape == (257, 32) and fb.dtype == np.float32
    nz = np.nonzero(fb.sum(axis=1))[0]
    assert nz.min() >= 1 and nz.max() <= 128
    # every filter is a single contiguous run (the kernel's sparse layout)
    for m in range(32):
        k = np.nonzero(fb[:, m])[0]
        assert k.size > 0 and k.max() - k.min() + 1 == k.size


def test_window_is_centered_periodic_hann():
    w = omel.hann_window()
    assert w.shape == (512,)
    assert np.all(w[:56] == 0) and np.all(w[456:] == 0)
    assert w[56] == 0.0 and abs(w[56 + 200] - 1.0) < 1e-7


def test_mel_model_graph_shapes():
    # MelSpectrogramModel shape KAT: 12,640 ones -> [1, 1, 76, 32] (mel-spectrogram.js:37-49)
    out = omel.mel_graph(np.ones((1, 12640), dtype=np.float32))
    assert out.shape == (1, 1, 76, 32)
    sq = omel.mel_spectrogram_model(np.ones((2, 17280), dtype=np.float32))
    assert sq.shape == (2, 105, 32)


def test_mel_frames_equal_reference_windowed_frames():
    """Computing each unique frame once equals the reference's per-audio-window
    frames: window w frame f == global frame 12 w + f (embeddings.py:190)."""
    rng = np.random.default_rng(1)
    pcm = rng.uniform(-0.5, 0.5, (2, 23040)).astype(np.float32)
    uniq, _, _ = omel.mel_frames(pcm)
    audio = pcm * np.float32(32767.0)
    for w, i in enumerate(range(0, 23040 - 17280 + 1, 1920)):
        ref = omel.mel_spectrogram_model(audio[:, i:i + 17280])
        np.testing.assert_allclose(uniq[:, 12 * w:12 * w + 105], ref, rtol=0, atol=2e-6)


# ----------------------------------------------------------------- GPU ----

def _clips(n=24, length=24000):
    from heybuddy.synthetic import edge_clips, synthetic_clips
    return synthetic_clips(n, length=length, seed=7), edge_clips(length)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])  # sparse VALU filterbank / split-f16 MFMA filterbank
def test_mel_kernel_parity_realistic_clips(variant):
    from heybuddy.kernels import MelPlan
    plan = MelPlan(omel.hann_window(), omel.mel_fbank()).set_variant(variant)
    clips, _ = _clips()
    out = plan(clips.cuda(), 141).cpu().numpy()
    ref, _, _ = omel.mel_frames(clips.numpy(), 141)
    err = np.abs(out - ref)
    assert out.shape == (24, 141, 32)
    assert err.max() <= 1e-4, f"max |diff| {err.max()}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_mel_kernel_parity_edge_clips(variant):
    from heybuddy.kernels import MelPlan
    plan = MelPlan(omel.hann_window(), omel.mel_fbank()).set_variant(variant)
    _, edges = _clips()
    out = plan(edges.cuda()).cpu().numpy()
    ref, mel_pow, energy = omel.mel_frames(edges.numpy())
    assert out.shape == ref.shape == (4, 147, 32)
    tol = omel.fp32_noise_tolerance(mel_pow, energy)
    bad = np.abs(out - ref) > tol
    assert not bad.any(), f"{bad.sum()} bins over tolerance; worst {np.abs(out - ref).max()}"
    # all-zero clip hits the log floor exactly: log10(1e-10)*10/10 + 2 = -8
    assert np.abs(out[0] + 8.0).max() <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_mel_kernel_ragged_and_strided(variant):
    """Odd clip counts (partial last block), a frame count below the maximum,
    and a strided (row-sliced) input."""
    from heybuddy.kernels import MelPlan
    plan = MelPlan(omel.hann_window(), omel.mel_fbank()).set_variant(variant)
    clips, _ = _clips(n=7, length=23040)
    big = torch.zeros((7, 24000))
    big[:, :23040] = clips
    dev = big.cuda()[:, :23040]
    out = plan(dev, 133).cpu().numpy()
    ref, _, _ = omel.mel_frames(clips.numpy(), 133)
    assert np.abs(out - ref).max() <= 1e-4
    one = plan(dev[:1], 1).cpu().numpy()
    assert np.abs(one - ref[:1, :1]).max() <= 1e-4
    empty = plan(dev[:0], 141)
    assert empty.shape == (0, 141, 32)
