import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: E402  (tests only)
    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def cvr():
    import cudavolumerenderer_amd as m
    m.load()
    return m
