"""Shared test setup.

`-m "not gpu"` runs here (no GPU): oracle vs the reference's golden vector, independent KKT
certificates for the oracle, host logic, and the C-ABI library's load/export surface.
`-m gpu` runs on an MI355X: HIP kernels vs the oracle, bit for bit, through the C-ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def _have_gpu():
    try:
        import qpgpu

        return qpgpu.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _have_gpu():
        pytest.fail("no GPU visible: -m gpu tests must run on an MI355X box")
    import qpgpu

    return qpgpu
