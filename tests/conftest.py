"""Test configuration: import paths, the `gpu` marker, shared tolerances.

-m "not gpu": oracle vs reference goldens, host logic, C-ABI exports (no GPU).
-m gpu      : the HIP engine (through the C-ABI) vs goldens and the oracle.
"""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "yuma-simulation_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Tolerance stated by BASELINE.json north_star: <= 1e-5 relative on fp32
# dividends and bonds; identical discrete decisions (consensus, clipping).
RTOL = 1e-5
ATOL_FRAC = 1e-6  # absolute floor, as a fraction of max|expected|


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libyuma_hip.so")


def assert_close(actual, expected, rtol=RTOL, atol_frac=ATOL_FRAC, what=""):
    a = np.asarray(actual, dtype=np.float64)
    e = np.asarray(expected, dtype=np.float64)
    assert a.shape == e.shape, f"{what}: shape {a.shape} != {e.shape}"
    finite = np.isfinite(e)
    scale = np.max(np.abs(e[finite])) if finite.any() else 0.0
    atol = atol_frac * scale
    nan_ok = np.array_equal(np.isnan(a), np.isnan(e))
    inf_ok = np.array_equal(np.isinf(a) & (a > 0), np.isinf(e) & (e > 0)) and np.array_equal(
        np.isinf(a) & (a < 0), np.isinf(e) & (e < 0))
    assert nan_ok and inf_ok, f"{what}: NaN/inf pattern differs"
    m = finite & np.isfinite(a)
    err = np.abs(a[m] - e[m])
    tol = atol + rtol * np.abs(e[m])
    bad = err > tol
    if bad.any():
        i = np.argmax(err - tol)
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} elements out of tolerance; worst |{a[m][i]} - {e[m][i]}| = {err[i]:.3e} > {tol[i]:.3e}")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load
