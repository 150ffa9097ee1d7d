"""Test configuration: the ``gpu`` marker and import paths.

``-m "not gpu"`` runs here (no GPU): oracle vs golden vectors, host logic, the
C ABI's exported symbols, gloo DP tests. ``-m gpu`` runs on an MI355X box:
the HIP kernels vs the oracle through the C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hey-buddy_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libhbk.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
