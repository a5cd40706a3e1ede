"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's published known answers.  Tolerance: posteriors
|a-b| <= 1e-6 max(|a|,|b|) above 1e-12 of the row max, 1e-18 absolute below;
grid-valued outputs (lb/mle/ub/ce, modes) exact; matSlideMult bit-exact."""
import numpy as np
import pytest

from conftest import assert_cz_close, assert_posterior_close, assert_z_close, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


def _models(g, key="models"):
    from oracle.oracle import MODEL_COLUMNS
    m = g[key]
    return {c: m[:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(m[:, j]))}


def _group_inputs(oracle, g, genes, cells):
    models = _models(g)
    sub = {k: v[cells] for k, v in models.items()}
    mm, lt, sq = oracle.model_matrix(sub)
    ucl, uci = oracle.ucl_uci(g["counts"][genes][:, cells])
    mag = oracle.marginals_from_prior_x(g["prior_x"])
    return mm, lt, sq, ucl, uci, mag


# ------------------------------------------------------------------ .Call layer
@pytest.mark.parametrize("nboot,seed,postflag,ensemble", [
    (50, 1, 0, 0), (17, 1379, 1, 0), (0, 1, 2, 0), (20, 5, 3, 0), (10, 1, 0, 1), (1, 7, 0, 0), (100, 2, 0, 0)])
def test_logBootPosterior_esmef(api, oracle, nboot, seed, postflag, ensemble):
    g = golden("esmef500.npz")
    genes = np.arange(0, 500, 3)
    cells = np.nonzero(g["groups"] == 0)[0]
    mm, lt, sq, ucl, uci, mag = _group_inputs(oracle, g, genes, cells)
    ref = oracle.logBootPosterior(mm, ucl, uci, mag, nboot, seed, postflag, lt, sq, ensemble)
    got = api.logBootPosterior(mm, ucl, uci, mag, nboot, seed, postflag, lt, sq, ensemble)
    if postflag == 0:
        assert_posterior_close(got, ref, what="jp")
        return
    assert_posterior_close(got["jp"], ref["jp"], what="jp")
    if "modes" in ref:
        np.testing.assert_array_equal(got["modes"], ref["modes"])
    if "post" in ref:
        for i, (a, b) in enumerate(zip(got["post"], ref["post"])):
            np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-13, err_msg=f"post cell {i}")


def test_logBootPosterior_knn_localtheta(api, oracle):
    """12-column models: local theta fit + squared-logit concomitant."""
    g = golden("knn300.npz")
    models = _models(g)
    mm, lt, sq = oracle.model_matrix(models)
    assert lt == 1 and sq == 1
    ucl, uci = oracle.ucl_uci(g["counts"])
    mag = oracle.marginals_from_prior_x(g["prior_x"])
    got = api.logBootPosterior(mm, ucl, uci, mag, int(g["nboot"]), 1, 1, lt, sq, 0)
    assert_posterior_close(got["jp"], g["jp"], what="knn jp vs golden")
    np.testing.assert_array_equal(got["modes"], g["modes"])
    ref = oracle.logBootPosterior(mm, ucl, uci, mag, 7, 11, 3, lt, sq, 0)
    got = api.logBootPosterior(mm, ucl, uci, mag, 7, 11, 3, lt, sq, 0)
    assert_posterior_close(got["jp"], ref["jp"], what="knn jp")
    for a, b in zip(got["post"][:8], ref["post"][:8]):
        np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("postflag", [0, 1, 2, 3])
def test_logBootBatchPosterior(api, oracle, postflag):
    g = golden("esmef500.npz")
    genes = np.arange(0, 500, 4)
    cells = np.arange(40)
    mm, lt, sq, ucl, uci, mag = _group_inputs(oracle, g, genes, cells)
    batch = (np.arange(40) * 7) % 3
    batchil = [np.nonzero(batch == b)[0].astype(np.int32) for b in range(3)]
    comp = [5, 0, 9]
    ref = oracle.logBootBatchPosterior(mm, ucl, uci, mag, batchil, comp, 12, 3, postflag, lt, sq)
    got = api.logBootBatchPosterior(mm, ucl, uci, mag, batchil, comp, 12, 3, postflag, lt, sq)
    if isinstance(ref, dict):
        assert_posterior_close(got["jp"], ref["jp"], what="batch jp")
        if "modes" in ref:
            np.testing.assert_array_equal(got["modes"], ref["modes"])
        if "post" in ref:
            for a, b in zip(got["post"], ref["post"]):
                np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-13)
    else:
        assert_posterior_close(got, ref, what="batch jp")


def test_jpmat(api, oracle):
    rng = np.random.default_rng(5)
    mats = [np.asfortranarray(-rng.gamma(2.0, 30.0, (37, 53))) for _ in range(9)]
    ref = oracle.jpmatLogBoot(mats, 13, 4)
    got = api.jpmatLogBoot(mats, 13, 4)
    assert_posterior_close(got, ref, what="jpmatLogBoot")
    matll = [mats[:4], mats[4:]]
    ref = oracle.jpmatLogBatchBoot(matll, [3, 2], 6, 9)
    got = api.jpmatLogBatchBoot(matll, [3, 2], 6, 9)
    assert_posterior_close(got, ref, what="jpmatLogBatchBoot")


def test_jpmat_degenerate_rows_exact(api, oracle):
    """Rows whose sums are dominated by huge magnitudes go through the reference-order
    fallback and must match the oracle bit for bit."""
    n, G = 6, 40
    mats = []
    for m in range(5):
        a = np.full((n, G), -3.0)
        a[:, m % 2::2] = -1e300 * (1 + 0.01 * m)
        a[:, 7] = -1.5
        mats.append(np.asfortranarray(a + np.arange(G)[None, :] * 1e-3))
    ref = oracle.jpmatLogBoot(mats, 8, 2)
    got = api.jpmatLogBoot(mats, 8, 2)
    np.testing.assert_array_equal(got, ref)


def test_logboot_degenerate_exact(api, oracle):
    """Every grid point clamped in some drawn cell: the fallback reproduces the reference's
    rounding-determined result exactly."""
    g = golden("esmef500.npz")
    mag = oracle.marginals_from_prior_x(g["prior_x"])
    mm = np.full((2, 12), np.nan, order="F")
    mm[0, :6] = [-10.0, 500.0, np.log(0.1), 0.7, 2.0, 1000.0]
    mm[1, :6] = [-1.4, 0.56, np.log(0.1), 0.7, 0.65, 0.77]
    counts = np.array([[0, 100000], [0, 0], [3, 5]], np.int32)
    ucl, uci = oracle.ucl_uci(counts)
    for nboot, seed in ((10, 1), (33, 2)):
        ref = oracle.logBootPosterior(mm, ucl, uci, mag, nboot, seed, 0)
        got = api.logBootPosterior(mm, ucl, uci, mag, nboot, seed, 0)
        np.testing.assert_allclose(got[0], ref[0], rtol=1e-13, atol=0)
        assert_posterior_close(got, ref, what="degenerate jp")


def test_matSlideMult_bit_exact(api, oracle):
    rng = np.random.default_rng(11)
    # n - 1 not a multiple of the slide's 4-lag groups (10, 403, 7, 3, 2) exercises the group
    # that straddles lag 0; n = 3 has no group entirely on the negative side
    for nr, n in ((17, 401), (5, 801), (3, 1), (1, 2), (64, 33), (9, 10), (6, 403), (4, 7), (5, 3)):
        a = np.asfortranarray(rng.random((nr, n)))
        b = np.asfortranarray(rng.random((nr, n)) ** 3)
        np.testing.assert_array_equal(api.matSlideMult(a, b), oracle.matSlideMult(a, b))


def test_ratio_and_summary(api, oracle):
    g = golden("esmef500.npz")
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    rp = api.calculate_ratio_posterior(g["jp1"], g["jp2"], prior)
    ref = oracle.calculate_ratio_posterior(g["jp1"], g["jp2"], g["prior_y"])
    assert_posterior_close(rp.values, ref, rel=1e-12, what="ratio")
    np.testing.assert_allclose(rp.values, g["ratio"], rtol=1e-12, atol=1e-300)
    s = api.quick_distribution_summary(rp)
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(s[k].to_numpy(), g[k], err_msg=k)
    np.testing.assert_allclose(s["Z"].to_numpy(), g["Z"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(s["cZ"].to_numpy(), g["cZ"], rtol=1e-9, atol=1e-9)


# ------------------------------------------------------------------ R-level API
def _frame_inputs(g):
    import pandas as pd
    models = pd.DataFrame(_models(g), index=list(g["cells"]))
    counts = pd.DataFrame(g["counts"], index=list(g["genes"]), columns=list(g["cells"]))
    groups = pd.Series(pd.Categorical(np.where(g["groups"] == 0, "ESC", "MEF"), categories=["ESC", "MEF"]),
                       index=list(g["cells"]))
    return models, counts, groups


def test_expression_difference_golden(api):
    g = golden("esmef500.npz")
    models, counts, groups = _frame_inputs(g)
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    out = api.scde_expression_difference(models, counts, prior, groups=groups, n_randomizations=int(g["nboot"]),
                                         n_cores=1, return_posteriors=True)
    assert_posterior_close(out["joint.posteriors"][0], g["jp1"], what="jp1")
    assert_posterior_close(out["joint.posteriors"][1], g["jp2"], what="jp2")
    assert_posterior_close(out["difference.posterior"].values, g["ratio"], what="ratio")
    res = out["results"]
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), g[k], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), g["Z"])
    assert_cz_close(res["cZ"].to_numpy(), g["cZ"], res["Z"].to_numpy(), g["Z"])


def test_vignette_table_on_gpu(api):
    """The published table (vignettes/diffexp.md:113-119) reproduced on the GPU, all 12,142 genes."""
    from test_oracle import VIGNETTE_TOP6
    v = golden("esmef_vignette_inputs.npz")
    models, counts, groups = _frame_inputs(v)
    prior = {"x": v["prior_x"], "y": v["prior_y"]}
    api.set_rand("darwin")
    try:
        res = api.scde_expression_difference(models, counts, prior, groups=groups, n_randomizations=100, n_cores=1)
    finally:
        api.set_rand("glibc")
    top = res.sort_values("Z", ascending=False, kind="stable").head(6)
    assert list(top.index) == list(VIGNETTE_TOP6)
    for name, ref in VIGNETTE_TOP6.items():
        got = res.loc[name, ["lb", "mle", "ub", "ce", "Z", "cZ"]].to_numpy(dtype=float)
        np.testing.assert_allclose(got, ref, atol=5e-7, rtol=0, err_msg=name)
    gd = golden("esmef_vignette_darwin.npz")
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), gd[k], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), gd["Z"])


def test_vignette_glibc_all_genes(api):
    v = golden("esmef_vignette_inputs.npz")
    gd = golden("esmef_vignette_glibc.npz")
    models, counts, groups = _frame_inputs(v)
    res = api.scde_expression_difference(models, counts, {"x": v["prior_x"], "y": v["prior_y"]}, groups=groups,
                                         n_randomizations=100, n_cores=1)
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), gd[k], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), gd["Z"])


def test_n_cores_chunk_seeds(api, oracle):
    """n.cores > 1 changes the per-chunk seeds (R/functions.R:606-617) exactly as in R."""
    g = golden("esmef500.npz")
    models = _models(g)
    cells = np.nonzero(g["groups"] == 1)[0]
    sub = {k: v[cells] for k, v in models.items()}
    counts = g["counts"][:300][:, cells]
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    for nc in (1, 10, 7):
        ref = oracle.scde_posteriors(sub, counts, g["prior_x"], n_randomizations=15, n_cores=nc)
        got = api.scde_posteriors(sub, counts, prior, n_randomizations=15, n_cores=nc)
        assert_posterior_close(got, ref, what=f"n_cores={nc}")


def test_posteriors_modes_and_post(api, oracle):
    g = golden("knn300.npz")
    models = _models(g)
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    counts = g["counts"][:80]
    ref = oracle.scde_posteriors(models, counts, g["prior_x"], n_randomizations=9, return_individual_posteriors=True,
                                 return_individual_posterior_modes=True, n_cores=1)
    got = api.scde_posteriors(models, counts, prior, n_randomizations=9, return_individual_posteriors=True,
                              return_individual_posterior_modes=True, n_cores=1)
    assert_posterior_close(got["jp"], ref["jp"], what="jp")
    np.testing.assert_array_equal(got["modes"], ref["modes"])
    for a, b in zip(got["post"], ref["post"]):
        np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12)


def test_edge_cases(api, oracle):
    g = golden("esmef500.npz")
    models = _models(g)
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    cells = np.arange(6)
    sub = {k: v[cells] for k, v in models.items()}
    cases = {
        "single gene": g["counts"][[17]][:, cells],
        "all zero": np.zeros((3, 6), np.int32),
        "no zeros anywhere": g["counts"][:20][:, cells] + 1,
        "huge counts": np.array([[0, 1, 2, 100000, 2000000, 7]] * 2, np.int32),
    }
    for name, c in cases.items():
        c = np.ascontiguousarray(c, np.int32)
        ref = oracle.scde_posteriors(sub, c, g["prior_x"], n_randomizations=11, n_cores=1)
        got = api.scde_posteriors(sub, c, prior, n_randomizations=11, n_cores=1)
        assert_posterior_close(got, ref, what=name)
    # the unique build's fixed-width bitmaps widen after a rebuild for large counts: the same
    # answers again (now from the wider fixed build), counts past the widest width still take the
    # exact build, and a negative count is still rejected after widening
    huge = np.ascontiguousarray(cases["huge counts"], np.int32)
    first = api.scde_posteriors(sub, huge, prior, n_randomizations=11, n_cores=1)
    for c in (huge, np.array([[0, 1, 2, 100000, 5000000, 7]] * 2, np.int32)):
        ref = oracle.scde_posteriors(sub, c, g["prior_x"], n_randomizations=11, n_cores=1)
        for _ in range(2):
            got = api.scde_posteriors(sub, c, prior, n_randomizations=11, n_cores=1)
            assert_posterior_close(got, ref, what="huge counts again")
    np.testing.assert_array_equal(api.scde_posteriors(sub, huge, prior, n_randomizations=11, n_cores=1), first)
    with pytest.raises(Exception):
        api.scde_posteriors(sub, np.array([[0, 1, 2, 3, -4, 7]] * 2, np.int32), prior, n_randomizations=11, n_cores=1)
    empty = api.scde_posteriors(sub, np.zeros((0, 6), np.int32), prior, n_randomizations=11, n_cores=1)
    assert np.asarray(empty).shape == (0, len(g["prior_x"]))
    tab = api.scde_expression_difference(models, np.zeros((0, len(g["groups"])), np.int32), prior,
                                         groups=list(g["groups"]), n_randomizations=5, n_cores=1)
    assert len(tab) == 0
    one = {k: v[[3]] for k, v in models.items()}
    ref = oracle.scde_posteriors(one, g["counts"][:30][:, [3]], g["prior_x"], n_randomizations=5, n_cores=1)
    got = api.scde_posteriors(one, g["counts"][:30][:, [3]], prior, n_randomizations=5, n_cores=1)
    assert_posterior_close(got, ref, what="single cell")


def test_negative_counts_rejected(api):
    g = golden("esmef500.npz")
    models = {k: v[:4] for k, v in _models(g).items()}
    with pytest.raises(Exception):
        api.scde_posteriors(models, -np.ones((3, 4), np.int32), {"x": g["prior_x"], "y": g["prior_y"]}, n_cores=1)


@pytest.mark.parametrize("ncores,nlev", [(1, 2), (3, 2), (2, 3), (2, "na")])
def test_batch_corrected_difference(api, oracle, ncores, nlev):
    """Batch branch (R/functions.R:321-399) end to end against the oracle's restatement:
    batch.effect, results and batch.adjusted tables (lb/mle/ub/ce exact, Z/cZ per spec) and
    every posterior (jp, batch ratio, ratio, 1601-column batch-adjusted ratio) within 1e-6.
    "na": two levels with every seventh cell's batch NA (tapply and table drop such cells:
    never drawn in the batch posteriors, absent from the compositions)."""
    g = golden("esmef500.npz")
    models, counts, groups = _frame_inputs(g)
    counts = counts.iloc[:120]
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    if nlev == 2:
        batch = np.array(["b1" if (i * 5) % 3 else "b2" for i in range(40)])
    elif nlev == "na":
        batch = np.array([None if i % 7 == 3 else ("b1" if (i * 5) % 3 else "b2") for i in range(40)], dtype=object)
    else:
        batch = np.array([("b1", "b2", "b3")[(i * 7 + i // 5) % 3] for i in range(40)])
    out = api.scde_expression_difference(models, counts, prior, groups=groups, batch=batch, n_randomizations=10,
                                         n_cores=ncores, return_posteriors=True)
    ref = oracle.scde_expression_difference_batch(_models(g), g["counts"][:120], g["prior_x"], g["prior_y"],
                                                  g["groups"], list(batch), n_randomizations=10, n_cores=ncores,
                                                  return_posteriors=True)
    for i in range(2):
        assert_posterior_close(out["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"jp{i}")
    assert_posterior_close(out["difference.posterior"].values, ref["difference.posterior"], what="ratio")
    assert_posterior_close(out["batch.adjusted.difference.posterior"].values,
                           ref["batch.adjusted.difference.posterior"], what="batch-adjusted ratio")
    for table in ("batch.effect", "results", "batch.adjusted"):
        got, want = out[table], ref[table]
        for k in ("lb", "mle", "ub", "ce"):
            np.testing.assert_array_equal(got[k].to_numpy(), want[k], err_msg=f"{table}.{k}")
        assert_z_close(got["Z"].to_numpy(), want["Z"], what=f"{table}.Z")
        assert_cz_close(got["cZ"].to_numpy(), want["cZ"], got["Z"].to_numpy(), want["Z"], what=f"{table}.cZ")
    # the four posteriors on two lanes (default) or one after the other: the same bits
    ctx = api.default_context()
    try:
        ctx.set_option("lanes", 1)
        one = api.scde_expression_difference(models, counts, prior, groups=groups, batch=batch, n_randomizations=10,
                                             n_cores=ncores, return_posteriors=True)
    finally:
        ctx.set_option("lanes", 2)
    for i in range(2):
        np.testing.assert_array_equal(one["joint.posteriors"][i], out["joint.posteriors"][i])
    for key in ("difference.posterior", "batch.adjusted.difference.posterior"):
        np.testing.assert_array_equal(one[key].values, out[key].values)
    for table in ("batch.effect", "results", "batch.adjusted"):
        np.testing.assert_array_equal(one[table].to_numpy(dtype=float), out[table].to_numpy(dtype=float))


def test_batch_device_matches_composition(api):
    """The one-call device batch pipeline equals the composition of the per-step calls
    (batch scde.posteriors, calculate.ratio.posterior, quick.distribution.summary) on a
    larger synthetic set with 3 batch levels and NA-group cells; every table bit-equal."""
    from scde_amd.prior import expression_prior
    rng = np.random.default_rng(11)
    models, counts, _ = _synthetic(7011, 700, 90)
    C = counts.shape[1]
    codes = np.where(np.arange(C) % 9 == 4, -1, np.arange(C) % 2)
    groups = [None if c < 0 else ("a", "b")[c] for c in codes]
    batch = np.array(["x", "y", "z"])[rng.integers(0, 3, C)]
    prior = expression_prior(models, counts, length_out=400)
    out = api.scde_expression_difference(models, counts, prior, groups=groups, batch=batch, n_randomizations=40,
                                         n_cores=4, return_posteriors=True)
    bpost = []
    for lv in (0, 1):
        ii = np.nonzero(codes == lv)[0]
        comp = {b: int(np.sum(batch[ii] == b)) for b in ("x", "y", "z")}
        bpost.append(api.scde_posteriors(models, counts, prior, n_randomizations=40, batch=batch, composition=comp,
                                         n_cores=4))
    brat = api.calculate_ratio_posterior(bpost[0], bpost[1], prior)
    np.testing.assert_array_equal(out["batch.effect"]["ce"].to_numpy(),
                                  api.quick_distribution_summary(brat, 0.0)["ce"].to_numpy())
    rat = out["difference.posterior"]
    uniform = {"x": rat.columns, "y": np.full(rat.shape[1], 1.0 / rat.shape[1])}
    adj = api.calculate_ratio_posterior(rat.values, brat.values, uniform, skip_prior_adjustment=True)
    np.testing.assert_array_equal(out["batch.adjusted.difference.posterior"].values, adj.values)
    want = api.quick_distribution_summary(adj, 0.0)
    for k in ("lb", "mle", "ub", "ce", "Z", "cZ"):
        np.testing.assert_array_equal(out["batch.adjusted"][k].to_numpy(), want[k].to_numpy(), err_msg=k)


@pytest.mark.parametrize("case", ["random", "ties_nan", "tiny"])
def test_bh_cz_device(api, oracle, case):
    """Device BH (scde_bh_cz_dev: pnorm, stable radix sort, cummin scan, qnorm) against the
    oracle's p.adjust restatement."""
    import ctypes
    from scde_amd._lib import lib
    rng = np.random.default_rng(7)
    if case == "random":
        z = rng.normal(0, 2.5, 20011)
    elif case == "ties_nan":
        z = np.round(rng.normal(0, 2, 5000), 1)
        z[::37] = np.nan
        z[5::101] = 0.0
        z[7::211] = 40.0
        z[9::223] = -40.0
    else:
        z = np.array([1.3])
    ctx = api.default_context()
    for zz in ([z] if case != "tiny" else [z, np.array([np.nan, 2.0]), np.array([-0.5, 2.0])]):
        zz = np.ascontiguousarray(zz, np.float64)
        n = zz.size
        zd, cd = ctypes.c_void_p(), ctypes.c_void_p()
        api.check(lib().scde_dev_alloc(ctx.handle, 8 * n, ctypes.byref(zd)))
        api.check(lib().scde_dev_alloc(ctx.handle, 8 * n, ctypes.byref(cd)))
        try:
            api.check(lib().scde_h2d(ctx.handle, zd, zz.ctypes.data_as(ctypes.c_void_p), 8 * n))
            api.bh_cz_device(ctx, zd.value, n, cd.value)
            got = np.zeros(n)
            api.check(lib().scde_d2h(ctx.handle, got.ctypes.data_as(ctypes.c_void_p), cd, 8 * n))
        finally:
            lib().scde_dev_free(ctx.handle, zd)
            lib().scde_dev_free(ctx.handle, cd)
        want = np.zeros(n)
        oracle.lib().o_bh_cz(oracle._p(zz), n, oracle._p(want))
        np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
        ok = ~np.isnan(want)
        np.testing.assert_allclose(got[ok], want[ok], rtol=1e-12, atol=1e-12)


def _synthetic(seed, ngenes, ncells, two_groups=True):
    import bench
    return bench.synthetic(seed, ngenes, ncells, two_groups=two_groups)


def test_expression_difference_config3_shape(api, oracle):
    """1000 cells (500/500) as in config 3: long ELL rows (>> 64 entries), large unique
    tables, the o.ifm-resampled synthetic generator of bench.py."""
    from scde_amd.prior import expression_prior
    models, counts, groups = _synthetic(7003, 160, 1000)
    prior = expression_prior(models, counts, length_out=400)
    api.set_rand("glibc")
    got = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=12, n_cores=3,
                                         return_posteriors=True)
    ref = oracle.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=12,
                                            n_cores=3, return_posteriors=True)
    for i in range(2):
        assert_posterior_close(got["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"jp{i}")
    res = got["results"]
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), ref["results"][k], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), ref["results"]["Z"])
    assert_cz_close(res["cZ"].to_numpy(), ref["results"]["cZ"], res["Z"].to_numpy(), ref["results"]["Z"])


def test_posteriors_modes_config4_shape(api, oracle):
    """2000 cells in one group with posterior modes, as in config 4."""
    from scde_amd.prior import expression_prior
    models, counts, _ = _synthetic(7004, 60, 2000, two_groups=False)
    prior = expression_prior(models, counts, length_out=400)
    api.set_rand("glibc")
    got = api.scde_posteriors(models, counts, prior, n_randomizations=6, return_individual_posterior_modes=True,
                              n_cores=1)
    ref = oracle.scde_posteriors(models, counts, prior["x"], n_randomizations=6,
                                 return_individual_posterior_modes=True, n_cores=1)
    assert_posterior_close(got["jp"], ref["jp"], what="jp")
    np.testing.assert_array_equal(got["modes"], ref["modes"])


@pytest.mark.parametrize("length_out", [60, 402, 700, 1200])
def test_expression_difference_grid_sizes(api, oracle, length_out):
    """Grids other than 401 points: G = 61 (one wave), 701 (11-wave blocks, column stride
    768), 1201 (> 1024 lanes: the k_boot fallback), with wider tables and ratio rows."""
    from scde_amd.prior import expression_prior
    g = golden("esmef500.npz")
    models = _models(g)
    counts = np.ascontiguousarray(g["counts"][:70])
    prior = expression_prior(models, counts, length_out=length_out)
    api.set_rand("glibc")
    got = api.scde_expression_difference(models, counts, prior, groups=list(g["groups"]), n_randomizations=10,
                                         n_cores=2, return_posteriors=True)
    ref = oracle.scde_expression_difference(models, counts, prior["x"], prior["y"], g["groups"], n_randomizations=10,
                                            n_cores=2, return_posteriors=True)
    for i in range(2):
        assert_posterior_close(got["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"jp{i}")
    assert_posterior_close(got["difference.posterior"].values, ref["difference.posterior"], what="ratio")
    res = got["results"]
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), ref["results"][k], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), ref["results"]["Z"])
    assert_cz_close(res["cZ"].to_numpy(), ref["results"]["cZ"], res["Z"].to_numpy(), ref["results"]["Z"])
