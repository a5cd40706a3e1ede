"""The Z / cZ parity checker itself (conftest.assert_z_close / assert_cz_close, SURVEY.md
§8(d)), on the CPU: the BH propagation bound against brute force, and the checker's verdicts
on the committed 20,000-gene config-3 oracle table with controlled perturbations — it must
accept the reference formula's own 1 - gs rounding (one ulp of gs on the Z < 0 branch, pushed
through the oracle's BH) and reject a 1e-5 relative change of a well-conditioned Z or cZ."""
import numpy as np
import pytest

from conftest import assert_cz_close, assert_z_close, bh_propagated_bound, golden


def _bh(p):
    # R's p.adjust(p, "BH") (R/functions.R:3529)
    n = p.size
    o = np.argsort(-p, kind="stable")
    q = np.minimum.accumulate(n / np.arange(n, 0, -1) * p[o])
    out = np.empty(n)
    out[o] = np.minimum(1.0, q)
    return out


def test_bh_bound_brute_force():
    rng = np.random.default_rng(7)
    for _ in range(200):
        n = int(rng.integers(1, 40))
        p = rng.random(n) ** 4
        e = rng.random(n) * 1e-3 * p
        bound = bh_propagated_bound(p, e)
        for _ in range(5):
            dp = p + rng.uniform(-1, 1, n) * e
            assert np.all(np.abs(_bh(dp) - _bh(p)) <= bound * (1 + 1e-12) + 1e-300)


def _table():
    g = golden("config3_full.npz")
    return g["results"][:, 4].copy(), g["results"][:, 5].copy()


def _cz(z, oracle):
    import ctypes
    z = np.ascontiguousarray(z, np.float64)
    cz = np.zeros(z.size)
    oracle.lib().o_bh_cz(z.ctypes.data_as(ctypes.c_void_p), z.size, cz.ctypes.data_as(ctypes.c_void_p))
    return cz


def test_checker_on_config3_table(oracle):
    from scipy.stats import norm
    z, cz = _table()
    assert np.array_equal(_cz(z, oracle), cz)  # the fixture's cZ is the oracle's BH of its Z
    assert_z_close(z, z)
    assert_cz_close(cz, cz, z, z)
    # the reference formula's floor: the capped Z < 0 genes are qnorm(gs, lower=F) of gs one
    # ulp away -- accepted, and their BH effect on every other gene too
    neg = np.nonzero((z < 0) & (norm.sf(-z) < 1e-10))[0]
    assert neg.size > 0
    gs = norm.cdf(-z[neg])          # 1 - tail, rounded as R holds it (a double near 1)
    z2 = z.copy()
    z2[neg] = norm.isf(np.nextafter(gs, 2.0))  # gs one ulp up: tail one ulp smaller
    z2[neg] = np.where(np.isfinite(z2[neg]), z2[neg], z[neg])
    assert_z_close(z2, z)
    assert_cz_close(_cz(z2, oracle), cz, z2, z)
    # a 1e-5 relative change of a well-conditioned Z is rejected ...
    well = np.nonzero((norm.sf(np.abs(z)) > 1e-6) & (np.abs(z) > 1))[0]
    z3 = z.copy()
    z3[well[0]] *= 1 + 1e-5
    with pytest.raises(AssertionError):
        assert_z_close(z3, z)
    # ... and so is a cZ off by 1e-5 relative where nothing upstream excuses it
    top = np.argsort(-np.abs(cz))
    pos = [i for i in np.nonzero((cz != 0) & (norm.sf(np.abs(cz)) > 1e-6))[0]][0]
    cz3 = cz.copy()
    cz3[pos] *= 1 + 1e-5
    with pytest.raises(AssertionError):
        assert_cz_close(cz3, cz, z, z)
    assert top.size == z.size
