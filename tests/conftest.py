import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpvae-1_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libmpvae_hip.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN

