import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "audio-analyzer-omega_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libomega.so on the device)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def normwise(a, b):
    """|a-b|_inf / max|b| (SURVEY.md §7 'Parity tolerances': normwise, not per-bin relative)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / den) if den > 0 else float(np.max(np.abs(a)))


@pytest.fixture(scope="session")
def golden():
    return load_golden
