"""Test configuration.

`-m "not gpu"` (CPU, this container): oracle vs the reference's fixtures, host logic,
C-ABI symbol export, gloo multi-process sharding.  `-m gpu` (MI355X): the HIP path
through the C ABI against the oracle (tests/test_gpu_*.py).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "fhe-fed_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
PALISADE_DIR = os.path.join(GOLDEN, "palisade") + os.sep
PALISADE_PYBIND_DIR = os.path.join(GOLDEN, "palisade_pybind") + os.sep


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: large-size property tests")


def set_switch(monkeypatch, var, val):
    """An A/B probe switch for the rest of the test: the environment variable, then the library's
    re-read (switches are never read on a launch path).  val None removes it."""
    if val is None:
        monkeypatch.delenv(var, raising=False)
    else:
        monkeypatch.setenv(var, val)
    import SHELFI_FHE

    SHELFI_FHE.reload_switches()


@pytest.fixture(autouse=True)
def _switches_restored():
    """After each test (and after monkeypatch has restored the environment): the library's switches
    re-read, so a test's probe switch never leaks into the next one."""
    yield
    if "SHELFI_FHE" in sys.modules:
        try:
            sys.modules["SHELFI_FHE"].reload_switches()
        except (OSError, AttributeError):
            pass


@pytest.fixture(scope="session")
def palisade_keys():
    import palisade_fixture as P

    return P.read_keys(PALISADE_DIR)
