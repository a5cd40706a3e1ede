import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def assert_posterior_close(a, b, rel=1e-6, floor=1e-12, abs_small=1e-18, what=""):
    """SURVEY.md §8(d) tolerance: |a-b| <= rel*max(|a|,|b|) for entries >= floor*rowmax,
    absolute abs_small below that (underflow tails).  Rows are the first axis."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.size == 0:
        return
    a2 = a.reshape(a.shape[0], -1)
    b2 = b.reshape(b.shape[0], -1)
    rowmax = np.maximum(np.abs(a2).max(1), np.abs(b2).max(1))[:, None]
    big = np.maximum(np.abs(a2), np.abs(b2)) >= floor * rowmax
    err = np.abs(a2 - b2)
    tol = np.where(big, rel * np.maximum(np.abs(a2), np.abs(b2)), abs_small)
    bad = ~(err <= tol) & ~(np.isnan(a2) & np.isnan(b2)) & ~(a2 == b2)
    if bad.any():
        i, j = np.argwhere(bad)[0]
        raise AssertionError(f"{what}: {bad.sum()} entries out of tolerance; first at {i},{j}: "
                             f"{a2[i, j]!r} vs {b2[i, j]!r}")


def assert_z_close(a, b, rel=1e-6, what="Z"):
    """Z / cZ parity: 1e-6 relative, except where Z is ill-conditioned.
    Z = qnorm(gs, lower=F) is computed from gs, a double near 1 at the -7.16 cap (and
    near 0 at the other end).  Near 1, gs has an absolute resolution of 2^-53, so
    one-ulp differences in gs -- the floor of reproducibility; R itself rounds its long
    double sum to double -- move Z by far more than 1e-6.  Accept pairs whose upper-tail
    masses pnorm(-|Z|) agree to 4 ulps of 1 (8.9e-16 absolute).  cZ (BH over n genes,
    R/functions.R:3527-3531) multiplies a gene's tail mass by up to n / rank <= n before
    qnorm, so for cZ (`what` naming it) the tail bound is n times that."""
    from scipy.stats import norm
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape
    same_nan = np.isnan(a) & np.isnan(b)
    ok_rel = np.abs(a - b) <= rel * np.maximum(np.abs(a), np.abs(b)) + 1e-12
    ta, tb = norm.sf(np.abs(a)), norm.sf(np.abs(b))
    scale = a.size if "cZ" in what else 1
    ok_tail = (np.sign(a) == np.sign(b)) & (np.abs(ta - tb) <= 4 * 2.0 ** -53 * scale)
    bad = ~(same_nan | ok_rel | ok_tail)
    if bad.any():
        i = np.nonzero(bad)[0][0]
        raise AssertionError(f"{what}: {bad.sum()} values out of tolerance; first at {i}: {a[i]!r} vs {b[i]!r}")


def gpu_available():
    try:
        import ctypes
        from scde_amd import _lib
        L = _lib.lib()
        h = ctypes.c_void_p()
        rc = L.scde_ctx_create(0, ctypes.byref(h))
        if rc == 0:
            L.scde_ctx_destroy(h)
            return True
    except Exception:
        return False
    return False


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
