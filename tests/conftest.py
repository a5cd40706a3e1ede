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


#: margins of every Z / cZ comparison in this session, printed in the terminal summary
Z_MARGINS = []

#: SURVEY.md §8(d): Z and cZ are compared as values (1e-6 relative) where the tail mass is
#: at least this, and as tail probabilities below it
TAIL_WELL = 1e-10
#: the reference's own rounding floor on the 1 - gs branch: Z < 0 is qnorm(gs, lower=F) of a
#: double gs >= 0.5 (R/functions.R:3524-3526), so its tail 1 - gs is resolved only to
#: ulp(gs) = 2^-53; two computations whose posteriors differ in the last bits give gs an
#: ulp or two apart.  Z > 0 is qnorm(gs + zv, lower=F) of a small sum: no such floor.
GS_ULPS = 4 * 2.0 ** -53


def _tails(z):
    from scipy.stats import norm
    return norm.sf(np.abs(z))


def _z_floor(z):
    """Per-gene tail floor of the reference formula (0 on the Z >= 0 branch)."""
    return np.where(z < 0, GS_ULPS, 0.0)


def assert_z_close(a, b, rel=1e-6, what="Z"):
    """Z parity on SURVEY.md §8(d)'s contract (R/functions.R:3514-3531), per gene:

    * tail mass t = pnorm(|Z|, lower=F) of the reference value >= 1e-10: |dZ| <= 1e-6 |Z|
      (plus 1e-12 absolute for Z within rounding of 0, where gs ~ 0.5 and zl/zg switch);
    * t < 1e-10 (|Z| > 6.36, up to the 7.16 cap of the 1e-15 pseudo-count): the tail
      probabilities agree to 1e-6 relative, beyond the reference formula's own floor on the
      Z < 0 branch (GS_ULPS: that tail is 1 - gs of a double gs near 1);
    * signs agree, NaN only against NaN.

    Records the margins (max relative dZ where well conditioned, max tail ratio elsewhere)
    in Z_MARGINS for the terminal summary."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    same_nan = np.isnan(a) & np.isnan(b)
    ta, tb = _tails(a), _tails(b)
    well = tb >= TAIL_WELL
    dz = np.abs(a - b)
    ok_rel = dz <= rel * np.maximum(np.abs(a), np.abs(b)) + 1e-12
    dt = np.abs(ta - tb)
    ok_tail = (np.sign(a) == np.sign(b)) & (dt <= rel * np.maximum(ta, tb) + _z_floor(b))
    ok = same_nan | np.where(well, ok_rel, ok_tail)
    with np.errstate(invalid="ignore", divide="ignore"):
        rz = np.where(well & ~same_nan, dz / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300), 0.0)
        rt = np.where(~well & ~same_nan, dt / np.maximum(np.maximum(ta, tb), 1e-300), 0.0)
    Z_MARGINS.append(dict(what=what, n=int(a.size), n_well=int((well & ~same_nan).sum()),
                          n_tail=int((~well & ~same_nan).sum()), max_rel_dZ=float(rz.max(initial=0.0)),
                          max_rel_dtail=float(rt.max(initial=0.0)),
                          n_floor=int((~well & ~same_nan & (dt > rel * np.maximum(ta, tb))).sum())))
    if not ok.all():
        i = np.nonzero(~ok)[0][0]
        raise AssertionError(f"{what}: {(~ok).sum()} values out of tolerance; first at {i}: {a[i]!r} vs {b[i]!r} "
                             f"(tails {ta[i]!r} vs {tb[i]!r})")


def bh_propagated_bound(p_ref, e):
    """Per-gene bound on |d p.adjust(p, 'BH')| from per-gene input errors e (R's form,
    pmin(1, cummin(n/i * p[o]))[ro] with o = order(p, decreasing=TRUE), R/functions.R:3529):
    the cummin is 1-Lipschitz in the max norm, so gene i's adjusted value moves by at most
    max over the genes ranked at or above it (p_j >= p_i) of n/rank_j * e_j."""
    p_ref = np.asarray(p_ref, np.float64)
    n = p_ref.size
    o = np.argsort(-p_ref, kind="stable")
    rank = np.arange(n, 0, -1, dtype=np.float64)
    q = np.maximum.accumulate((n / rank) * np.asarray(e, np.float64)[o])
    out = np.empty(n)
    out[o] = q
    return out


def assert_cz_close(cza, czb, za, zb, rel=1e-6, what="cZ"):
    """cZ parity (R/functions.R:3527-3531: cZ = sign(Z) qnorm(BH(pnorm(|Z|, lower=F)), lower=F)).
    cZ is a function of the whole Z vector, so each gene is bounded by its own propagated
    error: the observed Z tail differences of the genes at or above it in the BH order,
    times n/rank, through the cummin (bh_propagated_bound), plus 1e-6 of its own adjusted
    tail.  Where the adjusted tail is >= 1e-10 and nothing ill-conditioned feeds its cummin
    this is 1e-6 relative on cZ; the summary counts the genes whose bound came from the
    reference formula's 1 - gs floor upstream (`n_prop`)."""
    cza, czb, za, zb = (np.asarray(v, np.float64) for v in (cza, czb, za, zb))
    assert cza.shape == czb.shape == za.shape == zb.shape, what
    same_nan = np.isnan(cza) & np.isnan(czb)
    fin = ~(np.isnan(za) | np.isnan(zb))
    pa, pb = _tails(za), _tails(zb)
    e = np.where(fin, np.abs(pa - pb), 0.0)
    prop = np.zeros_like(pb)
    if fin.any():
        prop[fin] = bh_propagated_bound(pb[fin], e[fin])
    qa, qb = _tails(cza), _tails(czb)
    dq = np.abs(qa - qb)
    own = rel * np.maximum(qa, qb)
    dcz = np.abs(cza - czb)
    ok_rel = dcz <= rel * np.maximum(np.abs(cza), np.abs(czb)) + 1e-12
    ok_prop = ((np.sign(cza) == np.sign(czb)) | (cza == 0) | (czb == 0)) & (dq <= own + prop * (1 + 1e-9))
    ok = same_nan | ok_rel | ok_prop
    well = (qb >= TAIL_WELL) & ~same_nan
    with np.errstate(invalid="ignore", divide="ignore"):
        rz = np.where(well, dcz / np.maximum(np.maximum(np.abs(cza), np.abs(czb)), 1e-300), 0.0)
        rt = np.where(~same_nan, dq / np.maximum(np.maximum(qa, qb), 1e-300), 0.0)
    Z_MARGINS.append(dict(what=what, n=int(cza.size), n_well=int(well.sum()), n_tail=int((~well & ~same_nan).sum()),
                          max_rel_dZ=float(rz.max(initial=0.0)), max_rel_dtail=float(rt.max(initial=0.0)),
                          n_prop=int((~same_nan & ~ok_rel & ok_prop).sum()),
                          max_prop_over_tail=float(np.where(~same_nan, prop / np.maximum(qb, 1e-300), 0.0)
                                                   .max(initial=0.0))))
    if not ok.all():
        i = np.nonzero(~ok)[0][0]
        raise AssertionError(f"{what}: {(~ok).sum()} values out of tolerance; first at {i}: {cza[i]!r} vs {czb[i]!r} "
                             f"(adjusted tails {qa[i]!r} vs {qb[i]!r}, propagated bound {prop[i]!r})")


def pytest_terminal_summary(terminalreporter):
    if not Z_MARGINS:
        return
    terminalreporter.section("Z / cZ parity margins (SURVEY.md §8(d))")
    for m in Z_MARGINS:
        terminalreporter.write_line(" ".join(f"{k}={v:.3g}" if isinstance(v, float) else f"{k}={v}"
                                             for k, v in m.items()))


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
