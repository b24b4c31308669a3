import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session")
def gray():
    return np.load(os.path.join(GOLDEN, "middlebury_gray.npz"))


@pytest.fixture(scope="session")
def bm_expected():
    return np.load(os.path.join(GOLDEN, "bm_expected.npz"))


@pytest.fixture(scope="session")
def synth_expected():
    return np.load(os.path.join(GOLDEN, "synth_expected.npz"))


@pytest.fixture(scope="session")
def guided_expected():
    return np.load(os.path.join(GOLDEN, "guided_expected.npz"))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O
