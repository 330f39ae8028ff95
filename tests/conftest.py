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


@pytest.fixture(scope="session")
def palisade_keys():
    import palisade_fixture as P

    return P.read_keys(PALISADE_DIR)
