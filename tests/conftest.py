import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Build the native tree once per session if the in-tree artefacts are missing."""
    from devspace_amd import buildtools

    buildtools.ensure_built()
    return ROOT


@pytest.fixture
def devspace_bin():
    return os.path.join(ROOT, "bin", "devspace")
