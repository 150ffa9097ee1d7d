"""Featurizer drop-in (SpeechEmbeddings): orchestration pinned to the reference.

tests/golden/featurizer_index.npz and featurizer_oracle.npz were produced by
running the reference's own SpeechEmbeddings.__call__ (embeddings.py:153-234)
with index-encoding fakes and with the oracle mel / SE20 graphs injected
(oracle/make_golden.py). CPU tests pin the oracle orchestration and the host
window maps; GPU tests run the HIP drop-in through the C ABI.
"""
import os

import numpy as np
import pytest
import torch

from oracle import featurizer as ofeat

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name))


def test_window_plan_matches_reference_index_map():
    from heybuddy.embeddings import SpeechEmbeddings
    d = _load("featurizer_index.npz")
    for name, t in (("t24000", 24000), ("t23040", 23040), ("t17280", 17280)):
        starts, f_aw, f_total = SpeechEmbeddings.window_plan(t)
        codes = d[f"{name}_emb"][0, :, 0]
        assert list(codes.astype(int)) == starts, name
        # clip 1's codes carry +1000 (clip identity survives batching)
        assert list((d[f"{name}_emb"][1, :, 0] - 1000).astype(int)) == starts
        spec = d[f"{name}_spec"][0, :, 0].astype(int)
        n_aw = len(range(0, t - 17280 + 1, 1920))
        idx = np.concatenate([np.arange(f_aw) + 12 * w for w in range(n_aw)])
        tt = idx.size
        idx = idx[:tt - ((tt - 76) % 8)]
        np.testing.assert_array_equal(spec, idx)


def test_oracle_orchestration_matches_reference():
    from heybuddy.embedding_graph import se20_graph
    d = _load("featurizer_oracle.npz")
    g = se20_graph(int(d["graph_seed"]))
    emb, spec = ofeat.featurize(d["clips"], g, return_spectrograms=True)
    np.testing.assert_allclose(spec, d["spec_f32"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(emb, d["emb_f32"], rtol=1e-5, atol=1e-5)


def _close(out, ref, tol=1e-4):
    err = np.abs(out - ref)
    return (err <= tol * (1.0 + np.abs(ref))).all(), err.max()


@pytest.mark.gpu
def test_speech_embeddings_dropin_matches_reference_fixture():
    from heybuddy.embeddings import SpeechEmbeddings, set_default_graph
    from heybuddy.embedding_graph import se20_graph
    d = _load("featurizer_oracle.npz")
    set_default_graph(se20_graph(int(d["graph_seed"])))
    se = SpeechEmbeddings()
    emb, spec = se(list(d["clips"]), return_spectrograms=True)
    assert emb.shape == (3, 16, 96) and spec.shape == (3, 420, 32)
    ok, worst = _close(spec, d["spec_f32"])
    assert ok, f"spectrogram max |diff| {worst}"
    ok, worst = _close(emb, d["emb_f32"])
    assert ok, f"embedding max |diff| {worst}"
    e16 = se([d["int16"][0], d["int16"][1]], remove_nan=False)
    ok, worst = _close(e16, d["emb_i16"])
    assert ok, f"int16 path max |diff| {worst}"
    e2d = se(torch.from_numpy(d["clips"][:2].copy()))
    assert e2d.shape == (1, 16, 96)
    ok, worst = _close(e2d, d["emb_2d"])
    assert ok, f"2-D (channel-mean) path max |diff| {worst}"


@pytest.mark.gpu
def test_reference_shape_kats():
    """tests/test_embeddings.py of the reference."""
    from heybuddy.embeddings import get_speech_embeddings
    se = get_speech_embeddings()
    e, s = se(torch.randn((17280,)), return_spectrograms=True)
    assert s.shape == (1, 100, 32) and e.shape == (1, 4, 96)
    e, s = se(torch.randn((23040,)), return_spectrograms=True)
    assert s.shape == (1, 420, 32) and e.shape == (1, 16, 96)


@pytest.mark.gpu
def test_nan_replacement_and_building_blocks():
    from heybuddy.embeddings import SpeechEmbeddings
    se = SpeechEmbeddings()
    x = torch.from_numpy(_load("featurizer_oracle.npz")["clips"]).cuda()
    x[1, 5000] = float("nan")
    emb = se.featurize(x, remove_nan=False)
    assert torch.isnan(emb[1]).any() and not torch.isnan(emb[0]).any()
    fixed = se.featurize(x, remove_nan=True)
    assert not torch.isnan(fixed).any()
    assert torch.equal(fixed[1], fixed[0]) or torch.equal(fixed[1], fixed[2])
    # reference building blocks agree with the fused path
    a = x[:, :17280].double().mul(32767.0).float().cpu().numpy()
    spec = se.audio_to_spectrograms(torch.from_numpy(a[[0, 2]]))
    e = se.spectrograms_to_embeddings(spec)
    fused = se.featurize(x[[0, 2], :17280].contiguous())
    ok, worst = _close(e, fused.cpu().numpy())
    assert e.shape == (2, 4, 96) and ok, worst
