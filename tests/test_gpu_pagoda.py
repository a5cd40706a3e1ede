"""PAGODA helper .Call symbols (src/pagoda.cpp) on the GPU vs the CPU oracle
(oracle/pagoda_oracle.c; parity unpinned in the SURVEY.md section 8(c) sense -- no R here,
the oracle is cross-checked against numpy below).

Bar: winsorizeMatrix bit-exact (it only moves values); matCorr / matWCorr /
plSemicompleteCor2 1e-12 relative (rounding order only), union counts exact.
"""
import numpy as np
import pytest

from oracle import pagoda as OP


# ------------------------------------------------------------------ oracle vs numpy (CPU)
def test_oracle_winsorize_is_clamp_to_order_statistics():
    rng = np.random.default_rng(0)
    m = rng.normal(size=(30, 57))
    for trim in (0.0, 0.05, 0.2):
        ntr = int(np.floor(57 * trim + 0.5))
        w = OP.winsorizeMatrix(m, trim)
        s = np.sort(m, axis=1)
        if ntr == 0:
            np.testing.assert_array_equal(w, m)
        else:
            np.testing.assert_array_equal(w, np.clip(m, s[:, [ntr]], s[:, [57 - ntr - 1]]))


def test_oracle_correlations_against_numpy():
    rng = np.random.default_rng(1)
    x = rng.normal(size=(80, 7))
    y = rng.normal(size=(80, 3))
    np.testing.assert_allclose(OP.matCorr(x, y), np.corrcoef(x.T, y.T)[:7, 7:], rtol=1e-12, atol=1e-14)
    w = rng.uniform(0.1, 1.0, size=x.shape)
    c = OP.matWCorr(x, w)
    for i in range(7):
        for j in range(i + 1, 7):
            jw = np.sqrt(w[:, i] * w[:, j])
            jw /= jw.sum()
            a = x[:, i] - x[:, i] @ jw
            b = x[:, j] - x[:, j] @ jw
            assert c[j, i] == pytest.approx((a * b) @ jw / np.sqrt((a * a @ jw) * (b * b @ jw)), rel=1e-12)
            assert c[i, j] == 0.0
    assert np.all(np.diag(c) == 1.0)


def _pl(rng, np_=40, genes=300):
    pl = []
    for _ in range(np_):
        k = int(rng.integers(0, 60))
        i = np.sort(rng.choice(genes, size=k, replace=False))
        pl.append((i, rng.normal(size=k)))
    return pl


def test_oracle_plcor_against_set_intersection():
    rng = np.random.default_rng(2)
    pl = _pl(rng)
    res = OP.plSemicompleteCor2(pl)
    for a in range(len(pl)):
        for b in range(a + 1, len(pl)):
            ia, va = pl[a]
            ib, vb = pl[b]
            common, xa, xb = np.intersect1d(ia, ib, return_indices=True)
            assert res["n"][a, b] == len(ia) + len(ib) - len(common)
            l12 = (va[xa] * vb[xb]).sum()
            l11, l22 = (vb[xb] ** 2).sum(), (va[xa] ** 2).sum()
            want = l12 / np.sqrt(l11 * l22) if l11 * l22 > 0 else 0.0
            assert res["r"][a, b] == pytest.approx(want, rel=1e-12, abs=1e-15)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("k,n,trim", [(40, 57, 0.05), (300, 1000, 3 / 1000), (7, 10, 0.5), (25, 3000, 0.01),
                                      (3, 9000, 10 / 9000), (5, 16, 0.0)])
def test_winsorize_matches_oracle(k, n, trim):
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(k + n)
    m = rng.normal(size=(k, n))
    m[0, 0] = 1000.0
    m[1 % k, :5] = 0.25  # ties
    np.testing.assert_array_equal(PG.winsorizeMatrix(m, trim), OP.winsorizeMatrix(m, trim))


@pytest.mark.gpu
def test_winsorize_matrix_count_trim():
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(3)
    m = rng.normal(size=(12, 64))
    np.testing.assert_array_equal(PG.winsorize_matrix(m, 3), OP.winsorize_matrix(m, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(50, 9), (400, 130), (2000, 64)])
def test_matwcorr_matches_oracle(k, n):
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(k)
    f = rng.normal(size=(k, 3))
    m = f @ rng.normal(size=(3, n)) + rng.normal(size=(k, n))
    w = rng.uniform(0.0, 1.0, size=(k, n))
    got, want = PG.matWCorr(m, w), OP.matWCorr(m, w)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-14)
    assert np.all(np.triu(got, 1) == 0) and np.all(np.diag(got) == 1)


@pytest.mark.gpu
@pytest.mark.parametrize("k,nx,ny", [(300, 500, 1), (64, 33, 17)])
def test_matcorr_matches_oracle(k, nx, ny):
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(nx)
    x = rng.normal(size=(k, nx))
    y = x[:, :ny] * 0.5 + rng.normal(size=(k, ny))
    np.testing.assert_allclose(PG.matCorr(x, y), OP.matCorr(x, y), rtol=1e-11, atol=1e-14)


@pytest.mark.gpu
def test_plsemicompletecor2_matches_oracle():
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(4)
    pl = _pl(rng, np_=150, genes=500)
    got, want = PG.plSemicompleteCor2(pl), OP.plSemicompleteCor2(pl)
    np.testing.assert_array_equal(got["n"], want["n"])
    np.testing.assert_allclose(got["r"], want["r"], rtol=1e-12, atol=1e-15)


# ---- pagoda.varnorm's posterior-mode consumer (R/functions.R:1414-1507)
def _varnorm_inputs(ngenes=70):
    from conftest import golden
    from oracle import oracle as O
    g = golden("esmef500.npz")
    models = {c: g["models"][:, j] for j, c in enumerate(O.MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}
    return models, np.ascontiguousarray(g["counts"][:ngenes]), {"x": g["prior_x"], "y": g["prior_y"]}


def test_oracle_varnorm_poisson_tail():
    """sfp's upper tail P(X >= c) at the boundary cases R's ppois(c - 1, lambda, FALSE) has."""
    from scipy.stats import poisson
    lam = 0.1
    assert poisson.sf(-1, lam) == 1.0  # count 0
    assert poisson.sf(0, lam) == pytest.approx(1 - np.exp(-lam), rel=1e-14)
    assert poisson.sf(2, lam) == pytest.approx(1 - np.exp(-lam) * (1 + lam + lam * lam / 2), rel=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("expected,batched", [(True, False), (False, False), (True, True)])
def test_varnorm_weights_match_oracle(expected, batched):
    from oracle import pagoda as OP
    from scde_amd import api
    from scde_amd import pagoda as PG
    models, counts, prior = _varnorm_inputs()
    C = counts.shape[1]
    batch = np.array(["b%d" % (i % 3) for i in range(C)]) if batched else None
    api.set_rand("glibc")
    got = PG.pagoda_varnorm_weights(models, counts, prior, batch=batch, n_cores=2, n_randomizations=20,
                                    use_expected_value=expected)
    codes = np.array([i % 3 for i in range(C)]) if batched else None
    want = OP.varnorm_weights(models, counts, prior["x"], batch_codes=codes, n_randomizations=20, n_cores=2,
                              use_expected_value=expected)
    # the joint posteriors' SURVEY 8(d) bar (1e-6 relative) carries into their expected values
    # and through log(mode) into matw; the row-maximum modes are grid values, exact
    rt = 1e-6 if expected else 0.0
    np.testing.assert_allclose(got["avmodes"], want["modes"][0], rtol=rt)
    np.testing.assert_allclose(got["matw"], want["matw"], rtol=1e-6 if expected else 1e-12, atol=1e-15)
    if batched:
        np.testing.assert_allclose(got["modes"], want["modes"][1:], rtol=rt)
        np.testing.assert_allclose(got["bmatw"], want["bmatw"], rtol=1e-6, atol=1e-15)
