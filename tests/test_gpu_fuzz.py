"""Randomised GPU parity sweep: scde.expression.difference through the HIP path against
the oracle on seeded random shapes, models and seeding modes (SURVEY.md §8(d) bar:
posteriors 1e-6 relative above 1e-12 of the row max, lb/mle/ub/ce exact, Z per
assert_z_close).  Each case is small (oracle runs in well under a second).

Cases draw: genes 1-60, cells per group 1-35 (groups of unequal size), NA-group cells,
counts from a zero-inflated negative binomial with occasional huge counts, models
resampled from the es.mef (6-column) or knn (12-column: local theta, squared-logit
concentration) fixtures, n.randomizations in {1, 2, 7, 20, 33}, n.cores in {1, 2, 5},
prior length.out in {60, 401}.  Every case runs through the bootstrap kernels: k_boot2 (or
the tile path from 400 cells), and the tile path at every size (boot_tiles_cells 0).
"""
import numpy as np
import pytest

from conftest import assert_cz_close, assert_posterior_close, assert_z_close, golden

pytestmark = pytest.mark.gpu

NCASES = 12


def _case(seed):
    from oracle.oracle import MODEL_COLUMNS
    rng = np.random.default_rng(seed)
    src = golden("esmef500.npz" if seed % 3 else "knn300.npz")
    M = src["models"]
    n1, n2 = int(rng.integers(1, 36)), int(rng.integers(1, 36))
    nna = int(rng.integers(0, 4))
    C = n1 + n2 + nna
    rows = rng.integers(0, M.shape[0], C)
    models = {c: M[rows, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(M[:, j]))}
    G = int(rng.integers(1, 61))
    mu = np.exp(rng.normal(1.5, 1.8, (G, 1)))
    counts = rng.negative_binomial(2.0, 2.0 / (2.0 + mu), size=(G, C))
    counts[rng.uniform(size=(G, C)) < 0.55] = 0
    counts[rng.uniform(size=(G, C)) < 0.01] = int(rng.integers(10_000, 200_000))
    groups = np.array(["a"] * n1 + ["b"] * n2 + [None] * nna, dtype=object)
    rng.shuffle(groups)
    return models, np.ascontiguousarray(counts.astype(np.int32)), groups, dict(
        n_randomizations=int(rng.choice([1, 2, 7, 20, 33])), n_cores=int(rng.choice([1, 2, 5])),
        length_out=int(rng.choice([60, 400])))


@pytest.mark.parametrize("opts", [{}, {"boot_tiles_cells": 0}], ids=["default", "tiles"])
@pytest.mark.parametrize("seed", range(NCASES))
def test_expression_difference_fuzz(seed, opts):
    from oracle import oracle as O
    from oracle import prior as OP
    from scde_amd import api
    models, counts, groups, kw = _case(1000 + seed)
    prior = OP.expression_prior(models, counts, kw["length_out"])
    api.set_rand("glibc")
    glist = list(groups)
    ctx = api.default_context()
    for k, v in opts.items():
        ctx.set_option(k, v)
    try:
        got = api.scde_expression_difference(models, counts, {"x": prior["x"], "y": prior["y"]}, groups=glist,
                                             n_randomizations=kw["n_randomizations"], n_cores=kw["n_cores"],
                                             return_posteriors=True)
    finally:
        ctx.set_option("boot_tiles_cells", 400)
    # the oracle takes factor codes (level order a < b, NA = -1), the api R-style labels
    codes = np.array([{"a": 0, "b": 1, None: -1}[v] for v in glist])
    ref = O.scde_expression_difference(models, counts, prior["x"], prior["y"], codes,
                                       n_randomizations=kw["n_randomizations"], n_cores=kw["n_cores"],
                                       return_posteriors=True)
    for i in range(2):
        assert_posterior_close(got["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"jp{i} {kw}")
    assert_posterior_close(got["difference.posterior"].values, ref["difference.posterior"], what=f"ratio {kw}")
    res = got["results"]
    for k in ("lb", "mle", "ub", "ce"):
        np.testing.assert_array_equal(res[k].to_numpy(), ref["results"][k], err_msg=f"{k} {kw}")
    assert_z_close(res["Z"].to_numpy(), ref["results"]["Z"])
    assert_cz_close(res["cZ"].to_numpy(), ref["results"]["cZ"], res["Z"].to_numpy(), ref["results"]["Z"])
