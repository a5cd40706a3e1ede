"""CPU tests: the oracle (oracle/) against the reference's own known answers and
against independent references for the third-party arithmetic it restates."""
import ctypes
import os

import mpmath
import numpy as np
import pytest

from conftest import golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# vignettes/diffexp.md:113-119 (scde.expression.difference, n.randomizations=100, n.cores=1)
VIGNETTE_TOP6 = {
    "Dppa5a": (8.075220, 9.984631, 11.575807, 8.075220, 7.160813, 5.989598),
    "Pou5f1": (5.370220, 7.200073, 9.189043, 5.370220, 7.160328, 5.989598),
    "Gm13242": (5.688455, 7.677425, 9.785734, 5.688455, 7.159979, 5.989598),
    "Tdh": (5.807793, 8.075220, 10.302866, 5.807793, 7.159589, 5.989598),
    "Ift46": (5.449779, 7.359190, 9.228822, 5.449779, 7.150242, 5.989598),
    "4930509G22Rik": (5.409999, 7.478528, 9.785734, 5.409999, 7.115605, 5.978296),
}
# vignettes/diffexp.md:138-139 (scde.test.gene.expression.difference("Tdh"), 1e3 randomizations)
VIGNETTE_TDH_SINGLE = (5.728235, 8.03544, 10.30287, 5.728235, 7.151425, 7.151425)


def test_rand_matches_libc(oracle):
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 2, 1379, 2001, 12345, 4294967295):
        libc.srand(ctypes.c_uint(seed))
        ref = [libc.rand() for _ in range(3000)]
        assert list(oracle.rand_stream(seed, 3000)) == ref


def test_draw_sequence(oracle):
    # first draws for seed 1, n = 20
    assert list(oracle.draw_stream(1, 20, 10)) == [16, 7, 15, 15, 18, 3, 6, 15, 5, 11]


def test_darwin_rand_is_park_miller(oracle):
    oracle.set_rng(2)
    try:
        s = oracle.rand_stream(1, 4)
    finally:
        oracle.set_rng(0)
    # the "minimal standard" sequence from seed 1 (Park & Miller 1988)
    assert list(s) == [16807, 282475249, 1622650073, 984943658]


def test_stirlerr_halves(oracle):
    mpmath.mp.dps = 40
    L = oracle.lib()
    for i in range(1, 31):
        n = mpmath.mpf(i) / 2
        ref = mpmath.loggamma(n + 1) - (n + mpmath.mpf(1) / 2) * mpmath.log(n) + n - mpmath.log(mpmath.sqrt(2 * mpmath.pi))
        assert abs(L.o_stirlerr(i / 2) - float(ref)) <= 1e-16 * max(1e-3, abs(float(ref)))


def test_dnbinom_dpois_vs_mpmath(oracle):
    mpmath.mp.dps = 50
    rng = np.random.default_rng(7)
    for _ in range(400):
        x = int(rng.integers(0, 3000)) if rng.random() < 0.7 else int(rng.integers(0, 20))
        size = float(np.exp(rng.uniform(np.log(0.01), np.log(1000))))
        prob = float(size / (size + np.exp(rng.uniform(-20, 16))))
        X, S, Pm = mpmath.mpf(x), mpmath.mpf(size), mpmath.mpf(prob)
        ref = (mpmath.loggamma(X + S) - mpmath.loggamma(S) - mpmath.loggamma(X + 1) + S * mpmath.log(Pm)
               + X * mpmath.log(1 - Pm))
        got = oracle.dnbinom_log(x, size, prob)
        assert abs(got - float(ref)) <= 1e-11 * max(1.0, abs(float(ref))), (x, size, prob)
        lam = float(np.exp(rng.uniform(-5, 9)))
        refp = float(-lam + X * mpmath.log(lam) - mpmath.loggamma(X + 1))
        assert abs(oracle.dpois_log(x, lam) - refp) <= 1e-12 * max(1.0, abs(refp))


def test_qnorm_pnorm_vs_mpmath(oracle):
    mpmath.mp.dps = 40
    for p in list(np.exp(-np.linspace(0.01, 40, 200))) + list(np.linspace(0.01, 0.99, 50)):
        ref = float(mpmath.sqrt(2) * mpmath.erfinv(2 * mpmath.mpf(p) - 1))
        assert abs(oracle.qnorm(p, True) - ref) <= 5e-15 * max(1.0, abs(ref))
        assert abs(oracle.qnorm(p, False) + ref) <= 5e-15 * max(1.0, abs(ref))
    for x in np.linspace(-37, 37, 501):
        ref = float(mpmath.ncdf(x))
        assert abs(oracle.pnorm(x, True) - ref) <= 1e-14 * ref
        ref = float(mpmath.ncdf(-x))
        assert abs(oracle.pnorm(x, False) - ref) <= 1e-14 * ref


def test_r_chunks(oracle):
    # N=13788, n=10 -> seeds 1, 1379, 2758, ..., 12411
    ch = oracle.r_chunks(13788, 10)
    seeds = [int(c[0]) + 1 for c in ch]
    assert seeds[:3] == [1, 1379, 2758] and seeds[-1] == 12411
    assert sum(len(c) for c in ch) == 13788
    assert [int(c[0]) + 1 for c in oracle.r_chunks(20000, 10)] == list(range(1, 20000, 2000))


def _vignette_inputs():
    v = golden("esmef_vignette_inputs.npz")
    from oracle.oracle import MODEL_COLUMNS
    models = {c: v["models"][:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(v["models"][:, j]))}
    return v, models


def test_vignette_table_golden():
    """The committed oracle run over all 12,142 genes reproduces the vignette's printed table."""
    g = golden("esmef_vignette_darwin.npz")
    genes = list(g["genes"])
    order = np.argsort(-g["Z"], kind="stable")[:6]
    assert [genes[i] for i in order] == ["Dppa5a", "Pou5f1", "Gm13242", "Tdh", "Ift46", "4930509G22Rik"]
    for name, ref in VIGNETTE_TOP6.items():
        i = genes.index(name)
        got = [g[k][i] for k in ("lb", "mle", "ub", "ce", "Z", "cZ")]
        np.testing.assert_allclose(got, ref, atol=5e-7, rtol=0)


def test_vignette_live_oracle(oracle):
    """Live oracle on the six vignette genes (Darwin rand) and the single-gene Tdh test."""
    v, models = _vignette_inputs()
    genes = list(v["genes"])
    idx = [genes.index(n) for n in VIGNETTE_TOP6]
    oracle.set_rng(2)
    try:
        r = oracle.scde_expression_difference(models, v["counts"][idx], v["prior_x"], v["prior_y"], v["groups"],
                                              n_randomizations=100, n_cores=1)
        for j, (name, ref) in enumerate(VIGNETTE_TOP6.items()):
            got = [r[k][j] for k in ("lb", "mle", "ub", "ce", "Z")]
            np.testing.assert_allclose(got, ref[:5], atol=5e-7, rtol=0, err_msg=name)
        t = genes.index("Tdh")
        r = oracle.scde_expression_difference(models, v["counts"][[t]], v["prior_x"], v["prior_y"], v["groups"],
                                              n_randomizations=1000, n_cores=1)
        got = [r[k][0] for k in ("lb", "mle", "ub", "ce", "Z", "cZ")]
        np.testing.assert_allclose(got, VIGNETTE_TDH_SINGLE, atol=6e-6, rtol=0)
    finally:
        oracle.set_rng(0)


def test_oracle_reproduces_golden_small(oracle):
    """The oracle is deterministic against its committed golden vectors (es.mef 500 genes, B=50)."""
    g = golden("esmef500.npz")
    from oracle.oracle import MODEL_COLUMNS
    models = {c: g["models"][:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}
    r = oracle.scde_expression_difference(models, g["counts"][:60], g["prior_x"], g["prior_y"], g["groups"],
                                          n_randomizations=int(g["nboot"]), n_cores=1, return_posteriors=True)
    np.testing.assert_array_equal(r["joint.posteriors"][0], g["jp1"][:60])
    np.testing.assert_array_equal(r["joint.posteriors"][1], g["jp2"][:60])
    for k in ("lb", "mle", "ub", "ce", "Z"):
        np.testing.assert_array_equal(r["results"][k], g[k][:60])


def test_config3_fixture_matches_live_oracle(oracle):
    """tests/golden/config3_full.npz (tools/make_config3_fixture.py: the oracle over all 20,000
    genes of the bench's config-3 set in 16 n.cores chunks, cZ by BH over every gene) holds what
    the oracle computes: its prior is the numpy restatement's for these counts, and a window
    across the first chunk boundary (genes 1,240-1,259: two draw lists) recomputed live gives
    the stored lb/mle/ub/ce/Z bit for bit; cZ is the BH of the stored Z column."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from oracle.prior import expression_prior
    g = np.load(os.path.join(ROOT, "tests", "golden", "config3_full.npz"), allow_pickle=False)
    seed, ngenes, ncells, nboot, ncores = (int(v) for v in g["meta"])
    models, counts, groups = bench.synthetic(seed, ngenes, ncells, two_groups=True)
    prior = expression_prior(models, counts, bench.LENGTH_OUT)
    np.testing.assert_array_equal(prior["x"], g["prior_x"])
    np.testing.assert_array_equal(prior["y"], g["prior_y"])
    lo, hi = 1240, 1260
    oracle.set_rng(0)
    r = oracle.scde_expression_difference(models, np.ascontiguousarray(counts[lo:hi]), g["prior_x"], g["prior_y"],
                                          groups, n_randomizations=nboot, n_cores=ncores, gene_offset=lo,
                                          ngenes_total=ngenes)
    want = g["results"][lo:hi]
    for j, k in enumerate(("lb", "mle", "ub", "ce", "Z")):
        np.testing.assert_array_equal(r[k], want[:, j], err_msg=k)
    z = np.ascontiguousarray(g["results"][:, 4])
    cz = np.zeros(ngenes)
    oracle.lib().o_bh_cz(oracle._p(z), ngenes, oracle._p(cz))
    np.testing.assert_array_equal(cz, g["results"][:, 5])
