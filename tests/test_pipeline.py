"""heybuddy.pipeline: CU partitions for featurizing beside training.

CPU: the train CU set is spread evenly over the XCDs whether the mask's bit i
maps to XCD i // 32 or to XCD i % 8, and over the shader engines of the probed
mapping (XCD i % 8, SE (i // 8) % 4); the mask words hold exactly that set.
GPU: on a CU-masked stream (persistent grids sized to the mask) the embedding
chain gives the same bits as on the default stream, and the mel frames agree to
the last bit or two (the persistent mel kernel's frame-group-to-workgroup
assignment follows the grid size; measured max |d| 1.9e-6 on log-mel values);
the sync-free NaN-row replacement keeps clean rows and fills NaN rows from
NaN-free ones.
"""
import numpy as np
import pytest
import torch

from heybuddy.pipeline import cu_mask_words, train_cu_set


@pytest.mark.parametrize("n_train", [32, 64, 96, 128])
def test_train_cu_set_even_over_xcds(n_train):
    cus = train_cu_set(256, n_train)
    assert len(cus) == len(set(cus)) == n_train and all(0 <= c < 256 for c in cus)
    contiguous = np.bincount([c // 32 for c in cus], minlength=8)
    interleaved = np.bincount([c % 8 for c in cus], minlength=8)
    assert (contiguous == n_train // 8).all()
    assert (interleaved == n_train // 8).all()


@pytest.mark.parametrize("n_train", [32, 64, 96, 128])
@pytest.mark.parametrize("layout", ["spread", "se-whole"])
def test_train_cu_set_balanced_over_xcds_and_shader_engines(n_train, layout):
    """The probed MI355X mask mapping (profiles/r05h_cu_mask_layouts.log): bit i is XCD i % 8,
    shader engine (i // 8) % 4, CU i // 32 of that SE. The dispatcher balances workgroups over
    the XCDs and SEs, so both streams' CU sets must give every (XCD, SE) the same count (the
    train set; its complement then too) — unbalanced sets measured 30-45 % slower, and sets
    that leave an XCD empty are ignored by the runtime."""
    cus = train_cu_set(256, n_train, layout=layout)
    assert len(cus) == len(set(cus)) == n_train
    for part in (cus, sorted(set(range(256)) - set(cus))):
        per = np.zeros((8, 4), dtype=int)
        for c in part:
            per[c % 8, (c // 8) % 4] += 1
        if layout == "se-whole" and n_train % 64 == 0:  # whole SEs (else the spread fallback)
            assert (per.sum(1) == len(part) // 8).all()
            assert set(per.ravel()) <= {0, 8}
        else:
            assert (per == len(part) // 32).all()


def test_cu_mask_words():
    cus = train_cu_set(256, 64)
    words = cu_mask_words(cus, 256)
    assert len(words) == 8
    back = [32 * w + b for w, word in enumerate(words) for b in range(32) if word >> b & 1]
    assert back == sorted(cus)
    rest = sorted(set(range(256)) - set(cus))
    assert sum(bin(w).count("1") for w in cu_mask_words(rest, 256)) == 192


def test_replace_nan_rows_device_cpu_semantics():
    from heybuddy.embeddings import replace_nan_rows_device
    g = torch.Generator().manual_seed(0)
    e = torch.randn(12, 16, 96, generator=g)
    e[2, 5, 7] = float("nan")
    e[9] = float("nan")
    out = torch.empty_like(e)
    replace_nan_rows_device(e, out, generator=torch.Generator().manual_seed(1))
    clean = [i for i in range(12) if i not in (2, 9)]
    assert not torch.isnan(out).any()
    for i in clean:
        assert torch.equal(out[i], e[i])
    for i in (2, 9):
        assert any(torch.equal(out[i], e[j]) for j in clean)
    allnan = torch.full((3, 16, 96), float("nan"))
    assert (replace_nan_rows_device(allnan, torch.empty_like(allnan)) == 0).all()
    # with an extra zero row: the same result, the all-NaN case gathers the zero row
    ext = torch.cat([e, torch.zeros(1, 16, 96)])
    out2 = torch.empty_like(e)
    replace_nan_rows_device(ext, out2, generator=torch.Generator().manual_seed(1), zero_row=True)
    assert torch.equal(out2, out)
    allnan_ext = torch.cat([allnan, torch.zeros(1, 16, 96)])
    assert (replace_nan_rows_device(allnan_ext, torch.empty_like(allnan), zero_row=True) == 0).all()
    with pytest.raises(ValueError):  # an extra row is only taken when declared
        replace_nan_rows_device(ext, torch.empty_like(e))
    # +-inf without NaN is not a NaN row
    inf_row = e.clone()
    inf_row[4, 0, 0], inf_row[4, 0, 1] = float("inf"), -float("inf")
    out3 = torch.empty_like(e)
    replace_nan_rows_device(inf_row, out3, generator=torch.Generator().manual_seed(1))
    assert torch.equal(out3[4], inf_row[4])


@pytest.mark.gpu
def test_masked_stream_same_bits():
    from heybuddy.embedding_graph import WINDOW_STARTS
    from heybuddy.embeddings import embed_plan
    from heybuddy.kernels import embed_clips, mel_frames
    from heybuddy.pipeline import make_streams
    from heybuddy.spectrogram import default_mel_plan
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    clips = torch.randn((300, 24000), generator=g, device=dev) * 0.1
    mplan = default_mel_plan(dev, 32767.0)
    eplan = embed_plan(dev, WINDOW_STARTS)
    mel_ref = mel_frames(clips, mplan, 141).clone()
    ref = embed_clips(mel_ref, eplan).clone()
    fs, ts, keep = make_streams(dev, "split:64")
    for st in (fs, ts):
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            mel = mel_frames(clips, mplan, 141)
            out = embed_clips(mel_ref, eplan)
        torch.cuda.current_stream(dev).wait_stream(st)
        torch.cuda.synchronize()
        assert (mel - mel_ref).abs().max().item() <= 1e-5
        assert torch.equal(out, ref)
    del keep


@pytest.mark.gpu
def test_replace_nan_rows_device_gpu():
    from heybuddy.embeddings import replace_nan_rows_device
    dev = torch.device("cuda", 0)
    e = torch.randn(64, 16, 96, device=dev)
    e[5, 0, 0] = float("nan")
    e[40] = float("nan")
    out = torch.empty_like(e)
    replace_nan_rows_device(e, out)
    assert not torch.isnan(out).any()
    keep = [i for i in range(64) if i not in (5, 40)]
    assert torch.equal(out[keep], e[keep])


@pytest.mark.gpu
def test_nan_rows_fix_in_place():
    """hbk_nan_rows_fix (embeddings.py:209-234 in place, no host sync): NaN-free rows keep their
    bits, every NaN row becomes a copy of some NaN-free row, the draw depends on the seed and
    covers several sources, an all-NaN batch becomes zeros, a clean batch is untouched."""
    from heybuddy.kernels import nan_rows_fix
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    for n in (1, 7, 3000):
        e = torch.randn(n, 16, 96, device=dev, generator=g)
        ref = e.clone()
        bad = sorted({int(v) for v in torch.randint(0, n, (max(1, n // 5),), generator=g, device=dev).tolist()})
        if n > 1:
            bad = [b for b in bad if b != 0] or [n - 1]  # keep row 0 clean
        for i, b in enumerate(bad):
            e[b].view(-1)[(i * 37) % 1536] = float("nan")
        if n == 1:
            nan_rows_fix(e, seed=1)
            assert torch.equal(e, torch.zeros_like(e))  # every row NaN: zeros
            continue
        good = [i for i in range(n) if i not in bad]
        nan_rows_fix(e, seed=11)
        assert not torch.isnan(e).any()
        assert torch.equal(e[good], ref[good])
        src = []
        for b in bad:  # each patched row equals one NaN-free source row
            d = (ref[good] - e[b]).abs().flatten(1).amax(1)
            hit = torch.nonzero(d == 0).flatten()
            assert hit.numel() >= 1, f"row {b} is not a copy of a NaN-free row"
            src.append(good[int(hit[0])])
        if len(bad) >= 20:
            assert len(set(src)) > len(bad) // 4  # spread over many sources
    # a clean batch is left exactly as it is; an all-NaN batch becomes zeros
    e = torch.randn(257, 16, 96, device=dev, generator=g)
    ref = e.clone()
    nan_rows_fix(e, seed=2)
    assert torch.equal(e, ref)
    e.fill_(float("nan"))
    nan_rows_fix(e, seed=2)
    assert torch.equal(e, torch.zeros_like(e))
    # many blocks (2048 row ranges) and few NaN-free rows: the ordered list spans the blocks;
    # the same seed draws the same sources
    n = 100_003
    e = torch.full((n, 16, 96), float("nan"), device=dev)
    keep = torch.tensor([5, 40_000, 99_999, 100_002], device=dev)
    e[keep] = torch.randn(len(keep), 16, 96, device=dev, generator=g)
    ref = e[keep].clone()
    e2 = e.clone()
    nan_rows_fix(e, seed=9)
    nan_rows_fix(e2, seed=9)
    assert torch.equal(e, e2)
    assert torch.equal(e[keep], ref)
    flat = e.flatten(1)
    hits = torch.stack([(flat == ref[i].flatten()).all(1) for i in range(len(keep))])
    assert bool(hits.any(0).all())  # every row is one of the 4 NaN-free rows
    assert bool((hits.sum(1) > n // 8).all())  # each drawn about n / 4 times
