"""Feature files: appendable ``.npy`` and their path into HBM.

The reference writes every featurized chunk into one growing ``.npy`` file
(``AppendableNumpyArrayFile``, reference src/python/heybuddy/util/numpy_util.py:395-564,
header helpers :108-300) and trains from memory maps of such files
(``[N,16,96]`` f32 embeddings; ``combine --half`` stores f16, __main__.py:150-165).
This module keeps that file format and API:

* the header is a format-1.0 ``.npy`` header whose text is padded so that the
  row count (axis 0) can reach 21 digits without the header growing; appends
  are positional writes at the end of the data followed by an in-place rewrite
  of the row count, so the file is a valid ``.npy`` after every append;
* ``load_to_device`` streams a (memory-mapped) feature file into a device
  tensor through a pinned staging buffer in chunks, so a 72 GB negative pool
  never needs to fit in host RAM at once; the trainer then samples it on the
  device (``heybuddy.dataset.training``).
"""
from __future__ import annotations

import os
import struct
import threading
from typing import Any, Optional, Tuple

import numpy as np

__all__ = ["AppendableNumpyArrayFile", "read_npy_header", "load_to_device"]

_MAGIC = b"\x93NUMPY"
_RESERVE = 21  # growth-axis digits the header always has room for (any int64 row count)
_ALIGN = 64    # numpy pads the header so the data starts 64-B aligned


def _render_header(rows: int, tail: Tuple[int, ...], descr: str, size: Optional[int] = None) -> bytes:
    """Format-1.0 header for a C-order array of shape (rows, *tail).

    The dict text is followed by enough spaces that ``rows`` can grow to
    ``_RESERVE`` digits without the header (hence the data offset) moving.
    ``size`` pins the total header size of an existing file."""
    shape = (rows, *tail)
    body = "{'descr': %r, 'fortran_order': False, 'shape': %r, }" % (descr, shape)
    body += " " * (_RESERVE - len(str(rows)))
    fixed = len(_MAGIC) + 4  # magic, version (1, 0), uint16 header length
    need = fixed + len(body) + 1
    if size is None:
        size = (need + _ALIGN - 1) // _ALIGN * _ALIGN
    elif need > size:
        raise ValueError(f"shape {shape} no longer fits the file's {size}-byte header")
    body = body.ljust(size - fixed - 1) + "\n"
    if len(body) > 0xFFFF:
        raise ValueError("array header exceeds the .npy 1.0 limit")
    return _MAGIC + b"\x01\x00" + struct.pack("<H", len(body)) + body.encode("latin1")


def read_npy_header(fp) -> Tuple[Tuple[int, ...], bool, np.dtype, int]:
    """(shape, fortran_order, dtype, data offset) of an open ``.npy`` file."""
    fp.seek(0)
    major, _ = np.lib.format.read_magic(fp)
    reader = np.lib.format.read_array_header_1_0 if major == 1 else np.lib.format.read_array_header_2_0
    shape, fortran, dtype = reader(fp)
    return tuple(shape), bool(fortran), dtype, fp.tell()


def _pwrite_all(fd: int, buf, offset: int) -> None:
    view = memoryview(buf)
    while len(view):  # one pwrite moves at most ~2 GiB on Linux
        n = os.pwrite(fd, view, offset)
        view, offset = view[n:], offset + n


class AppendableNumpyArrayFile:
    """A ``.npy`` file that grows along axis 0 (the reference's feature-file
    writer, numpy_util.py:395-564; same constructor and ``append`` / ``close``
    surface, C order only).

    The file is a valid ``.npy`` after every append when
    ``rewrite_header_on_append`` is set (else after ``close``): data goes to the
    end with positional writes and only the row count in the fixed-size
    header changes.

    >>> import numpy, tempfile
    >>> tf = tempfile.NamedTemporaryFile(suffix=".npy")
    >>> with AppendableNumpyArrayFile(tf.name, delete_if_exists=True) as f:
    ...     f.append(numpy.array([1, 2, 3]))
    ...     f.append(numpy.array([4, 5, 6]))
    >>> numpy.load(tf.name)
    array([1, 2, 3, 4, 5, 6])
    """

    def __init__(self, filename: str, delete_if_exists: bool = False, rewrite_header_on_append: bool = True,
                 dtype: Optional[np.dtype] = None) -> None:
        self.filename = filename
        self.rewrite_header_on_append = rewrite_header_on_append
        self.lock = threading.Lock()
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.shape: Optional[Tuple[int, ...]] = None
        self.header_length = 0
        self._fd: Optional[int] = None
        self._end = 0  # byte offset of the end of the data
        if os.path.exists(filename) and (delete_if_exists or os.path.getsize(filename) == 0):
            os.unlink(filename)
        if os.path.exists(filename):
            self._open_existing()

    @property
    def initialized(self) -> bool:
        return self._fd is not None

    def _open_existing(self) -> None:
        with open(self.filename, "rb") as fp:
            shape, fortran, dtype, offset = read_npy_header(fp)
        if fortran:
            raise ValueError(f"{self.filename}: Fortran-order feature files are not appendable here")
        if dtype.hasobject:
            raise ValueError(f"{self.filename}: object dtype cannot be appended to")
        if self.dtype is not None and self.dtype != dtype:
            raise ValueError(f"{self.filename} stores {dtype}; {self.dtype} was requested")
        if not shape:
            raise ValueError(f"{self.filename}: a 0-d array has no axis to grow")
        _render_header(shape[0], shape[1:], np.lib.format.dtype_to_descr(dtype), offset)  # room to grow?
        size = os.path.getsize(self.filename)
        expect = offset + int(np.prod(shape)) * dtype.itemsize
        if size != expect:
            raise ValueError(f"{self.filename} holds {size - offset} data bytes but its header says "
                             f"{expect - offset}: the file needs recovery before appending")
        self.dtype, self.shape, self.header_length, self._end = dtype, shape, offset, size
        self._fd = os.open(self.filename, os.O_RDWR)

    def _header(self) -> bytes:
        return _render_header(self.shape[0], self.shape[1:], np.lib.format.dtype_to_descr(self.dtype),
                              self.header_length)

    def update_header(self) -> None:
        with self.lock:
            if self._fd is not None:
                os.pwrite(self._fd, self._header(), 0)

    def append(self, arr: np.ndarray) -> None:
        arr = np.asarray(arr)
        if arr.ndim == 0:
            raise ValueError("cannot append a 0-d array")
        with self.lock:
            if self._fd is None:  # first append creates the file
                self.dtype = self.dtype or arr.dtype
                self.shape = (0, *arr.shape[1:])
                self._fd = os.open(self.filename, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
                self.header_length = len(_render_header(0, self.shape[1:], np.lib.format.dtype_to_descr(self.dtype)))
                self._end = self.header_length
                os.pwrite(self._fd, self._header(), 0)
            if tuple(arr.shape[1:]) != tuple(self.shape[1:]):
                raise ValueError(f"cannot append rows of shape {arr.shape[1:]} to {self.filename}, "
                                 f"whose rows are {self.shape[1:]}")
            data = np.ascontiguousarray(arr, dtype=self.dtype)
            if data.nbytes:
                _pwrite_all(self._fd, data.reshape(-1).view(np.uint8), self._end)
            self._end += data.nbytes
            self.shape = (self.shape[0] + arr.shape[0], *self.shape[1:])
            if self.rewrite_header_on_append:
                os.pwrite(self._fd, self._header(), 0)

    def close(self) -> None:
        with self.lock:
            if self._fd is None:
                return
            os.pwrite(self._fd, self._header(), 0)
            os.close(self._fd)
            self._fd = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self) -> "AppendableNumpyArrayFile":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def load_to_device(path: str, device, dtype=None, chunk_rows: int = 65536, rows: Optional[slice] = None):
    """Memory-map a feature file and copy it into one device tensor, ``chunk_rows``
    rows at a time through a pinned staging buffer (host RAM stays bounded).
    ``dtype`` (e.g. torch.float16 for ``combine --half`` pools) converts on the
    device after each chunk lands."""
    import torch

    mm = np.load(path, mmap_mode="r")  # allow_pickle stays False
    if rows is not None:
        mm = mm[rows]
    src_dtype = torch.from_numpy(np.empty(0, dtype=mm.dtype)).dtype
    out = torch.empty(mm.shape, dtype=dtype or src_dtype, device=device)
    if mm.shape[0] == 0:
        return out
    n = min(chunk_rows, mm.shape[0])
    pinned = torch.empty((n, *mm.shape[1:]), dtype=src_dtype).pin_memory() if torch.cuda.is_available() \
        else torch.empty((n, *mm.shape[1:]), dtype=src_dtype)
    stage = torch.empty((n, *mm.shape[1:]), dtype=src_dtype, device=device)
    for r0 in range(0, mm.shape[0], n):
        k = min(n, mm.shape[0] - r0)
        if torch.cuda.is_available():
            torch.cuda.current_stream(out.device).synchronize()  # the previous chunk left the pinned buffer
        pinned[:k].numpy()[...] = mm[r0:r0 + k]
        stage[:k].copy_(pinned[:k], non_blocking=True)
        out[r0:r0 + k].copy_(stage[:k])
    return out
