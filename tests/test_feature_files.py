"""Feature files: the appendable .npy writer against
numpy.load, its reference semantics (shape check, reopen-and-append, f16
pools), and the chunked loader (CPU device here; the same code feeds HBM)."""
import os

import numpy as np
import pytest
import torch

from heybuddy.util.numpy_util import AppendableNumpyArrayFile, load_to_device, read_npy_header


def test_append_roundtrip_and_reopen(tmp_path):
    p = str(tmp_path / "f.npy")
    rng = np.random.default_rng(0)
    chunks = [rng.standard_normal((n, 16, 96)).astype(np.float32) for n in (5, 0, 17, 1)]
    with AppendableNumpyArrayFile(p, delete_if_exists=True) as f:
        for c in chunks[:2]:
            f.append(c)
    # reopen (the reference's feature generator appends chunk by chunk across runs)
    with AppendableNumpyArrayFile(p) as f:
        for c in chunks[2:]:
            f.append(c)
    got = np.load(p)
    np.testing.assert_array_equal(got, np.concatenate(chunks))
    with open(p, "rb") as fp:
        shape, fortran, dtype, off = read_npy_header(fp)
    assert shape == (23, 16, 96) and not fortran and dtype == np.float32 and off % 64 == 0


def test_header_has_room_to_grow(tmp_path):
    p = str(tmp_path / "g.npy")
    with AppendableNumpyArrayFile(p) as f:
        f.append(np.zeros((1, 3), np.float32))
        off0 = f.header_length
        f.shape = (10 ** 18, 3)  # the growth axis at 19 digits still fits the reserved header
        f.update_header()
        assert f.header_length == off0
        f.shape = (1, 3)
        f.update_header()
    assert np.load(p).shape == (1, 3)


def test_shape_mismatch_and_half_pool(tmp_path):
    p = str(tmp_path / "h.npy")
    with AppendableNumpyArrayFile(p, dtype=np.float16) as f:  # combine --half
        f.append(np.ones((2, 16, 96), np.float32))
        with pytest.raises(ValueError):
            f.append(np.ones((2, 17, 96), np.float32))
    a = np.load(p)
    assert a.dtype == np.float16 and a.shape == (2, 16, 96)
    with pytest.raises(ValueError):
        AppendableNumpyArrayFile(p, dtype=np.float32)


def test_truncated_file_needs_recovery(tmp_path):
    p = str(tmp_path / "t.npy")
    with AppendableNumpyArrayFile(p) as f:
        f.append(np.ones((4, 8), np.float32))
    with open(p, "r+b") as fp:
        fp.truncate(os.path.getsize(p) - 4)
    with pytest.raises(ValueError, match="recovery"):
        AppendableNumpyArrayFile(p)


def test_load_to_device_chunks(tmp_path):
    p = str(tmp_path / "l.npy")
    x = np.random.default_rng(1).standard_normal((1000, 16, 96)).astype(np.float32)
    with AppendableNumpyArrayFile(p) as f:
        f.append(x[:600])
        f.append(x[600:])
    t = load_to_device(p, torch.device("cpu"), chunk_rows=128)
    np.testing.assert_array_equal(t.numpy(), x)
    h = load_to_device(p, torch.device("cpu"), dtype=torch.float16, chunk_rows=333, rows=slice(100, 900))
    np.testing.assert_array_equal(h.numpy(), x[100:900].astype(np.float16))


@pytest.mark.gpu
def test_load_to_device_hbm(tmp_path):
    p = str(tmp_path / "d.npy")
    x = np.random.default_rng(2).standard_normal((3000, 16, 96)).astype(np.float16)
    with AppendableNumpyArrayFile(p) as f:
        for i in range(0, 3000, 700):
            f.append(x[i:i + 700])
    t = load_to_device(p, torch.device("cuda", 0), dtype=torch.float32, chunk_rows=512)
    assert t.is_cuda and t.dtype == torch.float32
    np.testing.assert_array_equal(t.cpu().numpy(), x.astype(np.float32))


def test_labeled_take_excludes_phrase_tokens(tmp_path):
    """PrecalculatedDatasetIterator.take on a labeled [N, 17, 96] set (ref
    precalculated.py:520-533): rows whose token row holds an excluded id are
    dropped and refilled from the following rows; the token row is cut off;
    a set whose every row is excluded raises instead of recursing."""
    from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
    np.random.seed(0)
    n = 40
    arr = np.zeros((n, 17, 96), np.float32)
    arr[:, :16] = np.arange(n, dtype=np.float32)[:, None, None]  # row id in the features
    arr[:, 16, :3] = [[7592, 2088 if i % 3 == 0 else 3000, 0] for i in range(n)]
    np.save(tmp_path / "lab.npy", arr)
    it = PrecalculatedDatasetIterator("lab", directory=str(tmp_path), labeled=True, exclude_tokens=[2088])
    got = np.concatenate([it.take(8) for _ in range(10)])
    assert got.shape == (80, 16, 96)
    ids = got[:, 0, 0].astype(int)
    assert not np.any(ids % 3 == 0) and set(ids) == {i for i in range(n) if i % 3}
    it2 = PrecalculatedDatasetIterator("lab", directory=str(tmp_path), labeled=True, exclude_tokens=[7592])
    with pytest.raises(ValueError):
        it2.take(8)
    # the phrase tokens drop [CLS] / [SEP] (ref tokens.py:57), so a token row with them is not excluded
    dev = it.to_device("cpu")
    assert dev.shape == (n - len(range(0, n, 3)), 16, 96)


def test_labeled_take_mostly_excluded_fills_without_recursion(tmp_path):
    """a set that keeps one row in 50 fills take(n) far past
    Python's recursion limit (the refill is a loop), with the reference's row
    order: the kept rows of the shuffled order, lap after lap."""
    from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
    np.random.seed(1)
    n = 500
    arr = np.zeros((n, 17, 96), np.float16)
    arr[:, :16] = (np.arange(n) % 2048).astype(np.float16)[:, None, None]
    arr[:, 16, 0] = [5 if i % 50 else 6 for i in range(n)]  # rows 0, 50, ... kept
    np.save(tmp_path / "sparse.npy", arr)
    it = PrecalculatedDatasetIterator("sparse", directory=str(tmp_path), labeled=True, exclude_tokens=[5])
    got = it.take(3000)  # 300 laps of the set
    assert got.shape == (3000, 16, 96)
    assert set(got[:, 0, 0].astype(int)) == set(range(0, n, 50))
    assert it.total_taken >= 3000
