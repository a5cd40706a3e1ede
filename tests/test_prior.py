"""scde.expression.prior (R/functions.R:225-254), SURVEY.md §8(f) row 2.

CPU: the oracle restatement (oracle/prior.py) against the priors stored in the fixtures,
which are the priors the oracle reproduced the vignette's printed table with (pinning).
GPU: the device prior (scde_expression_prior_dev, csrc/prior.hip) against the oracle:
x and max.value to 1e-14 relative, y / lp / grid.weight to 1e-9 relative (the binning is
exact fixed point, the convolution a direct sum where R uses an FFT; the prior then feeds
the posteriors, whose bar is 1e-6)."""
import numpy as np
import pytest

from conftest import golden


def _models(g):
    from oracle.prior import MODEL_COLUMNS
    m = g["models"]
    return {c: m[:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(m[:, j]))}


def test_oracle_prior_matches_fixture_vignette():
    from oracle import prior as OP
    v = golden("esmef_vignette_inputs.npz")
    p = OP.expression_prior(_models(v), v["counts"], 400, max_quantile=0.999)
    np.testing.assert_array_equal(p["x"], v["prior_x"])
    np.testing.assert_allclose(p["y"], v["prior_y"], rtol=1e-13, atol=0)


def test_oracle_prior_matches_fixture_knn():
    from oracle import prior as OP
    k = golden("knn300.npz")
    p = OP.expression_prior(_models(k), k["counts"], 400)
    np.testing.assert_array_equal(p["x"], k["prior_x"])
    np.testing.assert_allclose(p["y"], k["prior_y"], rtol=1e-13, atol=0)


def test_oracle_prior_pieces():
    """R semantics of the helpers: quantile type 7, seq.int end points, approx rule 1,
    dnorm4's split branch."""
    from oracle import prior as OP
    x = np.array([3.0, 1.0, 2.0, 10.0])
    assert OP.r_quantile7(x, 0.5) == 2.5
    assert OP.r_quantile7(x, 1.0) == 10.0
    s = OP.r_seq_len(-1.3, 1.3, 7)
    assert s[0] == -1.3 and s[-1] == 1.3
    a = OP.r_approx(np.array([0.0, 1.0, 2.0]), np.array([1.0, 3.0, 5.0]), np.array([-0.1, 0.5, 2.0, 2.1]))
    assert np.isnan(a[0]) and a[1] == 2.0 and a[2] == 5.0 and np.isnan(a[3])
    d = OP.r_dnorm(np.array([0.0, 0.6, 4.0]), 0.1)
    assert d[0] == pytest.approx(3.989422804014327) and d[2] == 0.0
    assert d[1] == pytest.approx(np.exp(-18) * 3.989422804014327, rel=1e-14)


def _check(got, want, what):
    np.testing.assert_allclose(got["max.value"], want["max.value"], rtol=1e-14, err_msg=what)
    np.testing.assert_allclose(got["x"], want["x"], rtol=1e-14, atol=1e-15, err_msg=what + ".x")
    for k in ("y", "lp", "grid.weight"):
        np.testing.assert_allclose(got[k], want[k], rtol=1e-9, atol=0, err_msg=f"{what}.{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["vignette_q999", "knn_sq", "esmef500_L60", "esmef500_maxvalue", "overflow"])
def test_device_prior(case):
    from oracle import prior as OP
    from scde_amd.prior import expression_prior
    kw = {}
    if case == "vignette_q999":
        g = golden("esmef_vignette_inputs.npz")
        kw = {"max_quantile": 0.999}
        L = 400
    elif case == "knn_sq":
        g = golden("knn300.npz")
        L = 400
    else:
        g = golden("esmef500.npz")
        L = 60 if case == "esmef500_L60" else 400
        if case == "esmef500_maxvalue":
            kw = {"max_value": 3.25}
    models, counts = _models(g), np.array(g["counts"])
    if case == "overflow":
        # counts whose magnitude overflows exp(): v = Inf, dropped from the density (totMass)
        counts = counts.copy()
        models = {k: v.copy() for k, v in models.items()}
        models["corr.a"][5] = 0.02
        counts[3, 5] = 2 ** 30
        counts[7, 5] = 2 ** 31 - 1
        kw = {"max_quantile": 0.9}
    want = OP.expression_prior(models, counts, L, **kw)
    got = expression_prior(models, counts, length_out=L, **kw)
    _check(got, want, case)


@pytest.mark.gpu
def test_device_prior_config_shape():
    """The bench generator's 20k x 200 shape, from a resident DeviceCounts."""
    import bench
    from oracle import prior as OP
    from scde_amd import api
    from scde_amd.prior import expression_prior
    models, counts, _ = bench.synthetic(2002, 20000, 200)
    want = OP.expression_prior(models, counts, 400)
    ctx = api.default_context()
    dc = api.DeviceCounts(ctx, counts)
    try:
        got = expression_prior(models, dc, length_out=400, ctx=ctx)
        again = expression_prior(models, dc, length_out=400, ctx=ctx)
    finally:
        dc.free()
    _check(got, want, "config2")
    for k in ("x", "y", "lp", "grid.weight"):  # deterministic
        np.testing.assert_array_equal(got[k], again[k])
