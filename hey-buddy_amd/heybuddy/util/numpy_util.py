"""Feature files: appendable ``.npy`` and their path into HBM.

The reference writes every featurized chunk into one growing ``.npy`` file
(``AppendableNumpyArrayFile``, reference src/python/heybuddy/util/numpy_util.py:395-564,
header helpers :108-300) and trains from memory maps of such files
(``[N,16,96]`` f32 embeddings; ``combine --half`` stores f16, __main__.py:150-165).
This module keeps that file format and API:

* the header is a format-1.0 ``.npy`` header whose text is padded so that the
  growth axis (axis 0, or the last axis for Fortran order) can reach 21 digits
  without the header growing; appending rewrites the shape in place, so the
  file is a valid ``.npy`` after every append (``numpy.load`` reads it);
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
_GROWTH_DIGITS = 21  # room for the growth axis (fits any int64 length)


def _header_bytes(shape: Tuple[int, ...], fortran_order: bool, descr: Any, header_len: Optional[int] = None) -> bytes:
    text = "{'descr': %r, 'fortran_order': %r, 'shape': %r, }" % (descr, fortran_order, tuple(shape))
    if shape:
        grow = shape[-1] if fortran_order else shape[0]
        text += " " * max(0, _GROWTH_DIGITS - len(repr(grow)))
    # magic (6) + version (2) + length (2) + text + "\n", padded to a multiple of 64
    base = len(_MAGIC) + 2 + 2
    if header_len is None:
        total = -(-(base + len(text) + 1) // 64) * 64
    else:
        total = header_len
        if base + len(text) + 1 > total:
            raise ValueError("header does not fit in the reserved length")
    text = text + " " * (total - base - len(text) - 1) + "\n"
    if len(text) > 0xFFFF:
        raise ValueError("header too long for format 1.0")
    return _MAGIC + bytes([1, 0]) + struct.pack("<H", len(text)) + text.encode("latin1")


def read_npy_header(fp) -> Tuple[Tuple[int, ...], bool, np.dtype, int]:
    """(shape, fortran_order, dtype, data offset) of an open ``.npy`` file."""
    fp.seek(0)
    version = np.lib.format.read_magic(fp)
    if version == (1, 0):
        shape, fortran, dtype = np.lib.format.read_array_header_1_0(fp)
    else:
        shape, fortran, dtype = np.lib.format.read_array_header_2_0(fp)
    return tuple(shape), bool(fortran), dtype, fp.tell()


class AppendableNumpyArrayFile:
    """Append arrays to one ``.npy`` file (reference numpy_util.py:395-564).

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
        self.initialized = False
        self.fp = None
        self.dtype = None if dtype is None else np.dtype(dtype)
        if os.path.exists(filename):
            if os.path.getsize(filename) == 0 or delete_if_exists:
                os.unlink(filename)
            else:
                self.initialize_file()

    def initialize_file(self) -> None:
        self.fp = open(self.filename, "rb+")
        self.shape, self.fortran_order, dtype, self.header_length = read_npy_header(self.fp)
        if dtype.hasobject:
            raise ValueError("Object arrays cannot be appended to")
        if self.dtype is not None and dtype != self.dtype:
            raise ValueError(f"{self.filename} holds {dtype}, not {self.dtype}")
        self.dtype = dtype
        if len(_header_bytes(self.shape, self.fortran_order, np.lib.format.dtype_to_descr(dtype))) > self.header_length:
            raise ValueError(f"Header of {self.filename} not appendable")
        self.fp.seek(0, os.SEEK_END)
        if self.fp.tell() - self.header_length != int(np.prod(self.shape)) * dtype.itemsize:
            raise ValueError(f"Cannot append to {self.filename}, needs recovery (data length != header shape)")
        self.initialized = True

    def _write_array_header(self) -> None:
        if self.fp is None:
            return
        self.fp.seek(0, os.SEEK_SET)
        self.fp.write(_header_bytes(self.shape, self.fortran_order, np.lib.format.dtype_to_descr(self.dtype),
                                    self.header_length))

    def update_header(self) -> None:
        with self.lock:
            self._write_array_header()

    def append(self, arr: np.ndarray) -> None:
        arr = np.asarray(arr)
        with self.lock:
            if not self.initialized:
                dtype = self.dtype if self.dtype is not None else arr.dtype
                data = np.ascontiguousarray(arr, dtype=dtype)
                with open(self.filename, "wb") as fp:
                    fp.write(_header_bytes(data.shape, False, np.lib.format.dtype_to_descr(data.dtype)))
                    data.tofile(fp)
                self.initialize_file()
                return
            c = -1 if self.fortran_order else 1
            if self.shape[::c][1:] != arr.shape[::c][1:]:
                raise ValueError(f"Shapes {self.shape[::c][1:][::c]} and {arr.shape[::c][1:][::c]} do not match")
            self.fp.seek(0, os.SEEK_END)
            arr.astype(self.dtype, copy=False).flatten(order="F" if self.fortran_order else "C").tofile(self.fp)
            if self.fortran_order:
                self.shape = (*self.shape[:-1], self.shape[-1] + arr.shape[-1])
            else:
                self.shape = (self.shape[0] + arr.shape[0], *self.shape[1:])
            if self.rewrite_header_on_append:
                self._write_array_header()

    def close(self) -> None:
        with self.lock:
            if self.initialized:
                if not self.rewrite_header_on_append:
                    self._write_array_header()
                self.fp.close()
                self.fp = None
                self.initialized = False

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
