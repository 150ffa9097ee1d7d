"""The C ABI (include/hbk.h) without a GPU: libhbk.so loads, exports every
declared entry point, the Python prototypes cover them, and the product path
refuses to run without a HIP device instead of falling back to the CPU."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hbk.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbk_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from heybuddy import _native
    if not os.path.exists(_native.LIB_PATH):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "hey-buddy_amd"))
        import build
        build.build()
    return _native.lib()


def test_every_declared_symbol_is_exported(lib):
    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n


def test_python_prototypes_match_header():
    from heybuddy import _native
    assert sorted(_native.exported_symbols()) == _declared()


def test_status_and_errors_without_gpu(lib):
    assert lib.hbk_version().decode().startswith("hbk")
    n = ctypes.c_int(-1)
    assert lib.hbk_device_count(ctypes.byref(n)) == 0 and n.value >= 0
    # argument errors come back as a status + thread-local message, no exception
    assert lib.hbk_mel_plan_create(None, None, 512, 160, 32, 1.0, 1e-10, 10.0, 2.0, None) != 0
    assert b"plan is NULL" in lib.hbk_last_error()
    assert lib.hbk_reverb_plan_create(24000, ctypes.byref(ctypes.c_void_p())) != 0
    assert b"23040" in lib.hbk_last_error()


def test_mlp_layout_is_host_only_and_matches_state_dict(lib):
    """Plan creation and the parameter layout need no device."""
    h = ctypes.c_void_p()
    assert lib.hbk_mlp_plan_create(1536, 96, 64, 2, ctypes.byref(h)) == 0
    n = ctypes.c_int64()
    offs = (ctypes.c_int64 * 24)()
    assert lib.hbk_mlp_layout(h, ctypes.byref(n), offs, 24) == 0
    assert n.value == 256417
    assert offs[0] == 0 and offs[1] == 1536 and offs[2] == 3072
    lib.hbk_mlp_plan_destroy(h)


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the GPU-less refusal")
def test_product_path_refuses_without_gpu():
    from heybuddy._native import HBKUnavailable
    from heybuddy.embeddings import SpeechEmbeddings
    with pytest.raises(HBKUnavailable):
        SpeechEmbeddings()(np.zeros(23040, dtype=np.float32))
