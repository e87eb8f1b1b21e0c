import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--odesat-lib", default="", help="A/B tooling: run the tests against this libodesat_hip "
                                                      "build (scripts/build_variant.sh) instead of the in-tree one")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu")
    if config.getoption("--odesat-lib"):
        from odesat_amd import _lib
        _lib.use_library(config.getoption("--odesat-lib"))


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session", autouse=True)
def _built_oracle():
    """The C oracle is test infrastructure; build it on first use."""
    from oracle import oracle
    if not os.path.exists(oracle.LIB_PATH):
        oracle.build()


class Experiments:
    """The library's experiment knobs (odesat_set_experiment) for one test, restored at teardown:
    xp.set("WAVE", 1), xp.delete("GROUP_WIDTH").  Values may be given as strings ("1", "640"); the term
    layout of PART_TERMS by name (region / ell / slot)."""

    TERMS = {"region": 0, "ell": 1, "slot": 2}

    def __init__(self):
        from odesat_amd import _lib
        self._lib = _lib
        self.saved = {}

    def _remember(self, key):
        if key not in self.saved:
            self.saved[key] = self._lib.get_experiment(key)

    def set(self, key, value):
        self._remember(key)
        if key == "PART_TERMS" and isinstance(value, str) and value in self.TERMS:
            value = self.TERMS[value]
        self._lib.set_experiment(key, None if value is None else int(value))

    def delete(self, key):
        self._remember(key)
        self._lib.set_experiment(key, None)

    def restore(self):
        for k, v in self.saved.items():
            self._lib.set_experiment(k, v)
        self.saved.clear()


@pytest.fixture
def xp():
    e = Experiments()
    yield e
    e.restore()
