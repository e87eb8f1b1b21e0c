import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session", autouse=True)
def _built_oracle():
    """The C oracle is test infrastructure; build it on first use."""
    from oracle import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()
