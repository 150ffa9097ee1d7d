"""Speech embedding: graph / window-map checks (CPU) and HIP parity (GPU).

The embedding graph is runtime data (heybuddy.embedding_graph); parity is
against oracle.embed.run_graph, which evaluates every 76-frame window on its
own exactly as SpeechEmbeddingModel.__call__ does (embeddings.py:32-42) — so
the GPU clip path's shared-prefix deduplication is checked too.
Both GEMM precisions of the plan are checked ('split': fp16 hi/lo pairs on
the f16 MFMA, ~2^-21 relative per operand; 'exact': f32 MFMA).
Tolerance: vs the fp64 oracle, |diff| <= 1e-4 * (1 + |ref|).
"""
import numpy as np
import pytest
import torch

from oracle import embed as oemb
from oracle import mel as omel


def test_se20_graph_signature():
    from heybuddy.embedding_graph import Conv, se20_graph
    g = se20_graph()
    convs = [op for op in g.ops if isinstance(op, Conv)]
    assert len(convs) == 20 and convs[-1].name == "conv2d_19" and convs[-1].act is None
    assert g.shapes()[-1] == (1, 1, 96)
    # reference KAT: SpeechEmbedding.test feeds [100, 32] zeros -> [4, 96]
    # (speech-embedding.js:50-68): windows of 76 at stride 8 over 100 frames
    assert (100 - 76) // 8 + 1 == 4


def test_window_starts_match_reference_slots():
    """slot 4w + q <- audio window w (1920 samples = 12 frames), embedding
    window q at stride 8 (embeddings.py:190, :136-143)."""
    from heybuddy.embedding_graph import WINDOW_STARTS
    assert WINDOW_STARTS == (0, 8, 16, 24, 12, 20, 28, 36, 24, 32, 40, 48, 36, 44, 52, 60)
    assert len(set(WINDOW_STARTS)) == 14 and max(WINDOW_STARTS) + 76 == 136


def test_oracle_graph_shapes_and_squeeze():
    from heybuddy.embedding_graph import se20_graph
    g = se20_graph()
    x = np.zeros((3, 76, 32, 1), dtype=np.float32)
    out = oemb.speech_embedding_model(g, x)
    assert out.shape == (3, 96)
    one = oemb.speech_embedding_model(g, x[:1])
    assert one.shape == (96,)  # the reference's .squeeze() drops n == 1


def _mel_clips(n, seed=3):
    from heybuddy.synthetic import synthetic_clips
    clips = synthetic_clips(n, seed=seed)
    mel, _, _ = omel.mel_frames(clips.numpy(), 141)
    return mel


def _oracle_clip_embeddings(graph, mel):
    from heybuddy.embedding_graph import WINDOW_STARTS
    wins = np.stack([mel[:, s:s + 76] for s in WINDOW_STARTS], axis=1)  # [B,16,76,32]
    ref = oemb.run_graph(graph, wins.reshape(-1, 76, 32))
    return ref.reshape(mel.shape[0], len(WINDOW_STARTS), -1)


def _close(out, ref, tol=1e-4):
    err = np.abs(out - ref)
    bound = tol * (1.0 + np.abs(ref))
    return (err <= bound).all(), err.max()


PRECISIONS = ["split", "exact"]


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PRECISIONS)
def test_embed_windows_parity(precision):
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    g = se20_graph()
    plan = EmbedPlan(g, precision=precision)
    rng = np.random.default_rng(5)
    wins = (rng.standard_normal((37, 76, 32)) * 2 + 6).astype(np.float32)
    out = plan.windows(torch.from_numpy(wins).cuda()).cpu().numpy()
    ref = oemb.run_graph(g, wins)
    ok, worst = _close(out, ref)
    assert out.shape == (37, 96) and ok, f"max |diff| {worst}"


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PRECISIONS)
def test_embed_clips_parity_shared_prefix(precision):
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    g = se20_graph()
    plan = EmbedPlan(g, precision=precision)
    assert plan.seq_frames == 136 and plan.n_prefix_ops == 13
    mel = _mel_clips(5)
    out = plan.clips(torch.from_numpy(mel).cuda()).cpu().numpy()
    ref = _oracle_clip_embeddings(g, mel)
    ok, worst = _close(out, ref)
    assert out.shape == (5, 16, 96) and ok, f"max |diff| {worst}"
    # duplicated windows (start 24 and 36 appear twice) give identical rows
    np.testing.assert_array_equal(out[:, 3], out[:, 8])
    np.testing.assert_array_equal(out[:, 7], out[:, 12])


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PRECISIONS)
def test_embed_clips_ragged_batches(precision):
    """Clip counts that leave partial task groups, and one clip."""
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    g = se20_graph()
    plan = EmbedPlan(g, precision=precision)
    mel = _mel_clips(3, seed=11)
    ref = _oracle_clip_embeddings(g, mel)
    for n in (1, 3):
        out = plan.clips(torch.from_numpy(mel[:n]).cuda()).cpu().numpy()
        ok, worst = _close(out, ref[:n])
        assert ok, f"n={n}: max |diff| {worst}"


@pytest.mark.gpu
def test_embed_pattern_kernels_match_generic_path(monkeypatch, capfd):
    """The plan picks the streaming p0s kernel (one wave per clip) for SE20's
    chain 0, the two-wave p1s pipeline for chain 1, the 16-clip p2s pipeline for
    chain 2 and the phase-deduplicated tail (2 phase images per clip instead of
    16 windows) on the 16-image t3s pipeline; HBK_EMBED_NO_T3S runs that tail on
    the generic split-f16 kernel, HBK_EMBED_NO_P0S /
    NO_P1S fall back to the banded p0 / p1 kernels, HBK_EMBED_NO_DEDUP to the
    per-window tail, and with every pattern disabled the generic split-f16
    kernel runs every chain. All paths match the oracle and each other."""
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    g = se20_graph()
    mel = _mel_clips(9, seed=21)  # 9 clips: waves with 3 and 2 clips, idle waves in the last block
    ref = _oracle_clip_embeddings(g, mel)
    monkeypatch.setenv("HBK_DEBUG_EMBED", "1")
    capfd.readouterr()
    outs = {}
    for name, env, want in (("p0s", {}, ("hbk p0s chain", "hbk p1s chain", "hbk p2s chain", "hbk tail dedup",
                                          "hbk t3s chain")),
                            ("not3s", {"HBK_EMBED_NO_T3S": "1"}, ("hbk p2s chain", "hbk tail dedup")),
                            ("p0", {"HBK_EMBED_NO_P0S": "1", "HBK_EMBED_NO_P1S": "1"},
                             ("hbk p0 chain", "hbk p1 chain", "hbk tail dedup")),
                            ("nodedup", {"HBK_EMBED_NO_DEDUP": "1"}, ("hbk p0s chain", "hbk p1s chain")),
                            ("generic", {"HBK_EMBED_NO_P0": "1", "HBK_EMBED_NO_P1": "1", "HBK_EMBED_NO_P2S": "1",
                                         "HBK_EMBED_NO_T3S": "1"}, ())):
        for k in ("HBK_EMBED_NO_P0S", "HBK_EMBED_NO_P1S", "HBK_EMBED_NO_P0", "HBK_EMBED_NO_P1", "HBK_EMBED_NO_P2S",
                  "HBK_EMBED_NO_DEDUP", "HBK_EMBED_NO_T3S"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        plan = EmbedPlan(g, precision="split")
        err = capfd.readouterr().err
        for w in want:
            assert w + ":" in err, (name, err)
        if not want:
            assert "hbk p0" not in err and "hbk p1" not in err and "hbk p2" not in err and "hbk t3" not in err, err
        if name in ("nodedup", "not3s"):
            assert "hbk t3s chain" not in err, err
        if name == "nodedup":
            assert "hbk tail dedup" not in err, err
        outs[name] = plan.clips(torch.from_numpy(mel).cuda()).cpu().numpy()
    for name, out in outs.items():
        ok, worst = _close(out, ref)
        assert ok, f"{name}: max |diff| {worst}"
    for name in ("p0", "not3s", "nodedup", "generic"):
        assert np.abs(outs["p0s"] - outs[name]).max() <= 1e-5 * (1.0 + np.abs(ref).max()), name


def _generic_graph(seed=9):
    """Shapes the SE20 stand-in does not have: cin 1 with a 2x3 kernel, channel
    counts that are not multiples of 8 / 32 (12, 40, 70, 33), a 1x1 conv, a
    (1, 2) pool and a kernel that spans the whole remaining image."""
    from heybuddy.embedding_graph import Conv, Graph, MaxPool
    rng = np.random.default_rng(seed)

    def conv(kh, kw, ci, co, act="leaky_relu"):
        w = rng.standard_normal((kh, kw, ci, co)) * np.sqrt(2.0 / (kh * kw * ci))
        return Conv(kh, kw, ci, co, w.astype(np.float32), (rng.standard_normal(co) * 0.1).astype(np.float32),
                    act=act)

    ops = [conv(2, 3, 1, 12), conv(1, 1, 12, 40), MaxPool(2, 2), conv(3, 2, 40, 70), MaxPool(1, 2),
           conv(7, 2, 70, 33, act=None)]
    return Graph(ops, (20, 12, 1), name="generic")


def test_generic_graph_shapes():
    g = _generic_graph()
    assert g.shapes()[-1] == (1, 1, 33)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PRECISIONS)
def test_embed_generic_graph_parity(precision):
    from heybuddy.kernels import EmbedPlan
    g = _generic_graph()
    plan = EmbedPlan(g, starts=(0,), device=0, precision=precision)
    rng = np.random.default_rng(2)
    wins = rng.standard_normal((23, 20, 12)).astype(np.float32)
    out = plan.windows(torch.from_numpy(wins).cuda()).cpu().numpy()
    ref = oemb.run_graph(g, wins)
    ok, worst = _close(out, ref)
    assert out.shape == (23, 33) and ok, f"max |diff| {worst}"


def _wide_graph(seed=13):
    """Convs wider than 96 output channels (130 inside a chain, 100 at a
    chain's end): the kernels run them in groups of output-channel blocks."""
    from heybuddy.embedding_graph import Conv, Graph, MaxPool
    rng = np.random.default_rng(seed)

    def conv(kh, kw, ci, co, act="leaky_relu"):
        w = rng.standard_normal((kh, kw, ci, co)) * np.sqrt(2.0 / (kh * kw * ci))
        return Conv(kh, kw, ci, co, w.astype(np.float32), (rng.standard_normal(co) * 0.1).astype(np.float32),
                    act=act)

    ops = [conv(3, 3, 1, 40), conv(1, 3, 40, 130), MaxPool(2, 2), conv(3, 3, 130, 100), MaxPool(1, 2),
           conv(7, 1, 100, 33, act=None)]
    return Graph(ops, (20, 12, 1), name="wide")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", PRECISIONS)
def test_embed_wide_channels_parity(precision):
    """More than 96 output channels (round 1 refused them), against the oracle."""
    from heybuddy.kernels import EmbedPlan
    g = _wide_graph()
    assert g.shapes()[-1] == (1, 1, 33)
    plan = EmbedPlan(g, starts=(0,), device=0, precision=precision)
    rng = np.random.default_rng(6)
    wins = rng.standard_normal((29, 20, 12)).astype(np.float32)
    out = plan.windows(torch.from_numpy(wins).cuda()).cpu().numpy()
    ref = oemb.run_graph(g, wins)
    ok, worst = _close(out, ref)
    assert out.shape == (29, 33) and ok, f"max |diff| {worst}"


@pytest.mark.gpu
def test_embed_split_precision_margin():
    """The split path sits orders of magnitude inside the tolerance: relative
    error vs the fp64 oracle below 1e-5 over SE20 windows."""
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    g = se20_graph()
    plan = EmbedPlan(g, precision="split")
    rng = np.random.default_rng(8)
    wins = (rng.standard_normal((64, 76, 32)) * 2 + 6).astype(np.float32)
    out = plan.windows(torch.from_numpy(wins).cuda()).cpu().numpy()
    ref = oemb.run_graph(g, wins)
    rel = np.abs(out - ref).max() / np.abs(ref).max()
    assert rel < 1e-5, rel


@pytest.mark.gpu
def test_featurize_across_the_16384_clip_chunk():
    """hbk_embed_clips works through the batch in 16,384-clip workspace chunks
    (hbk_embed.hip kChunkClips): 16,390 clips cross one boundary. The clips on
    both sides of it (and the first / last) against the oracle mel + graph."""
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.embeddings import SpeechEmbeddings
    from heybuddy.synthetic import synthetic_clips
    n = 16390
    clips = synthetic_clips(n, seed=21, device="cuda")
    se = SpeechEmbeddings(device_id=0)
    out, frames = se.featurize(clips, return_frames=True)
    pick = [0, 16381, 16382, 16383, 16384, 16385, 16386, n - 1]
    sub = clips[pick].cpu().numpy()
    mel_ref, _, _ = omel.mel_frames(sub, frames.shape[1])
    np.testing.assert_allclose(frames[pick].cpu().numpy(), mel_ref, rtol=1e-4, atol=1e-4)
    ref = _oracle_clip_embeddings(se20_graph(), mel_ref)
    ok, worst = _close(out[pick].cpu().numpy(), ref)
    assert out.shape == (n, 16, 96) and ok, f"max |diff| {worst}"


@pytest.mark.gpu
def test_embed_split_range_guard():
    """Split-f16 range guard (include/hbk.h, hbk_embed_range_status): every
    kernel that splits an activation into f16 hi / lo raises the plan's flag
    at |x| >= 65504; the host-returning entry points then recompute in exact
    f32. A plan whose weights leave the f16 range is refused."""
    from heybuddy.embedding_graph import Conv, Graph, se20_graph
    from heybuddy.embeddings import SpeechEmbeddingModel
    from heybuddy.kernels import EmbedPlan
    from heybuddy._native import HBKError
    g = se20_graph()
    split, exact = EmbedPlan(g, precision="split"), EmbedPlan(g, precision="exact")
    rng = np.random.default_rng(4)
    wins = (rng.standard_normal((9, 76, 32)) * 2 + 6).astype(np.float32)
    mel = _mel_clips(2, seed=5)
    split.windows(torch.from_numpy(wins).cuda())
    split.clips(torch.from_numpy(mel).cuda())
    assert not split.range_tripped()  # realistic inputs stay inside the range
    # per-window path (generic kernel) and clip path (p0 / p1 / x3) with inputs past 65504
    split.windows(torch.from_numpy(wins * 2e4).cuda())
    assert split.range_tripped()
    assert not split.range_tripped()  # the read cleared it
    split.clips(torch.from_numpy(mel * 1e5).cuda())
    assert split.range_tripped()
    assert not exact.range_tripped()
    # the reference-shaped entry point returns the exact-f32 result when tripped
    model = SpeechEmbeddingModel(device_id=0, graph=g)
    big = wins * 2e4
    out = model(big[:, :, :, None])
    ref = exact.windows(torch.from_numpy(big).cuda()).cpu().numpy()
    np.testing.assert_array_equal(out, ref)
    # weights outside the f16 range: refused in split, fine in exact
    ops = list(g.ops)
    c0 = ops[0]
    w = c0.weight.copy()
    w.flat[0] = 7e4
    ops[0] = Conv(c0.kh, c0.kw, c0.cin, c0.cout, w, c0.bias, act=c0.act, alpha=c0.alpha)
    g_big = Graph(ops, g.in_shape, name="se20-bigw")
    with pytest.raises(HBKError, match="65504"):
        EmbedPlan(g_big, precision="split")
    EmbedPlan(g_big, precision="exact")


@pytest.mark.gpu
@pytest.mark.parametrize("n_front", [1, 2, 3])
def test_embed_clips_front_back_split(n_front):
    """hbk_embed_clips_front + hbk_embed_clips_back (the scheduling split the
    pipelined bench uses: the last chains on the training stream) equal
    hbk_embed_clips bit for bit, at every split point of SE20's clip program,
    each half on its own stream and workspace."""
    from heybuddy.embedding_graph import se20_graph
    from heybuddy.kernels import EmbedPlan
    plan = EmbedPlan(se20_graph(), precision="split")
    assert 1 <= n_front < plan.n_chains
    mel = torch.from_numpy(_mel_clips(9, seed=5)).cuda()
    ref = plan.clips(mel)
    mid = torch.empty((9, plan.mid_floats(n_front)), device="cuda")
    out = torch.empty_like(ref)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        plan.clips_front(mel, n_front, mid)
    s2.wait_stream(s1)
    with torch.cuda.stream(s2):
        plan.clips_back(mid, 9, n_front, out)
    torch.cuda.current_stream().wait_stream(s2)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
