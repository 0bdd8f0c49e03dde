"""Shared test setup.

`-m "not gpu"`: oracle vs the reference's own known answers, host logic, the
C-ABI library's exports and error paths (no device calls).
`-m gpu`: parity of the HIP path against the oracle and the golden fixtures,
through the C ABI, on a real MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device; runs through the C ABI")


@pytest.fixture(scope="session")
def rt():
    import raytracinginoneweekendinrust_amd as rt
    return rt


@pytest.fixture(scope="session")
def orc():
    import oracle_ffi
    return oracle_ffi
