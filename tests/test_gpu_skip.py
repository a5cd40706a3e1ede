"""Grid-stretch skipping in the bootstrap (k_stretch_mask + k_boot2 + redo launch).

The skipping is an optimisation that must not change results: a 64-point stretch is only
left out of a boot slab when a rigorous upper bound of its row values stays more than 51
below the exact row maximum (post-check), i.e. when every softmax term there falls under
the e^-50 cut that zeroes it anyway; any slab that fails the check is recomputed whole.
These tests run the same calls with skipping on (default), off (SCDE_BOOT_SKIP=0), and
with a negative heuristic slack (SCDE_SKIP_SLACK) that makes the mask drop stretches the
post-check must reject, so the redo launch carries real work -- and compare all three
with the oracle at the SURVEY §8(d) bar.
"""
import numpy as np
import pytest

from conftest import assert_posterior_close, assert_z_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


def _run(api, monkeypatch, env, models, counts, prior, groups, nrand, ncores):
    for k in ("SCDE_BOOT_SKIP", "SCDE_SKIP_SLACK"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    api.set_rand("glibc")
    return api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nrand,
                                          n_cores=ncores, return_posteriors=True)


@pytest.mark.parametrize("seed,ngenes,ncells,nrand,ncores", [(8002, 300, 200, 100, 1), (8003, 120, 1000, 40, 3)])
def test_skip_modes_match_oracle(api, oracle, monkeypatch, seed, ngenes, ncells, nrand, ncores):
    import bench
    from scde_amd.prior import expression_prior
    models, counts, groups = bench.synthetic(seed, ngenes, ncells)
    prior = expression_prior(models, counts, length_out=400)
    ref = oracle.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=nrand,
                                            n_cores=ncores, return_posteriors=True)
    runs = {
        "skip": {},
        "noskip": {"SCDE_BOOT_SKIP": "0"},
        "forced-redo": {"SCDE_SKIP_SLACK": "-45"},
    }
    for name, env in runs.items():
        got = _run(api, monkeypatch, env, models, counts, prior, groups, nrand, ncores)
        for i in range(2):
            assert_posterior_close(got["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"{name} jp{i}")
        assert_posterior_close(got["difference.posterior"].values, ref["difference.posterior"], what=f"{name} ratio")
        res = got["results"]
        for k in ("lb", "mle", "ub", "ce"):
            np.testing.assert_array_equal(res[k].to_numpy(), ref["results"][k], err_msg=f"{name} {k}")
        assert_z_close(res["Z"].to_numpy(), ref["results"]["Z"], what=f"{name} Z")
        assert_z_close(res["cZ"].to_numpy(), ref["results"]["cZ"], what=f"{name} cZ")
