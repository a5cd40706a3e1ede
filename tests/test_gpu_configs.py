"""GPU parity at every BASELINE configuration's real shape, on gene slices
small enough for the oracle to finish in seconds:

* config 3 -- 64 genes of the bench's own 20,000 x 1,000 data set (500/500 cells), B = 100
  (five 20-boot slabs, the stretch mask and its redo pass at 500 cells per group), reference
  seeding n.cores 1 and 10 (ten chunk seeds over 20,000 genes: the n.cores = 10 slice,
  genes 1968..2031, straddles the first chunk boundary, so it uses two draw lists);
* config 4 -- 48 genes x 2,000 cells in one group, B = 100, postflag 1 (posterior modes exact);
* config 5 -- the npcs = 1 multi-start weighted-PCA kernel at 3,000 cells (R = 3 register
  tiles per thread), against the C oracle on identical starts.

The oracle is the C restatement (oracle/scde_oracle.c, oracle/bwpca_oracle.c).
"""
import numpy as np
import pytest

from conftest import assert_cz_close, assert_posterior_close, assert_z_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


def _bench_slice(config, ngenes, two_groups=True, start=0):
    """The bench's synthetic data set for `config`, its prior (from all genes, on the GPU,
    as bench.py computes it), and genes start .. start + ngenes - 1."""
    import bench
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS[config]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=two_groups)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    return models, np.asfortranarray(counts[start:start + ngenes]), groups, prior, cfg["genes"]


@pytest.mark.parametrize("ncores", [1, 10])
def test_config3_slice_full_bootstrap(api, oracle, ncores):
    g0 = 0 if ncores == 1 else 1968
    models, counts, groups, prior, ntot = _bench_slice("3", 64, start=g0)
    api.set_rand("glibc")
    # n.cores seeding of the whole 20,000-gene call (global gene offsets)
    from scde_amd import sharded
    got_rows = sharded.device_shard(models, counts, prior, groups, 100, ncores, 0.0, g0, ntot)
    ref = oracle.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=100,
                                            n_cores=ncores, gene_offset=g0, ngenes_total=ntot,
                                            return_posteriors=True)
    for j, k in enumerate(("lb", "mle", "ub", "ce")):
        np.testing.assert_array_equal(got_rows[:, j], ref["results"][k], err_msg=k)
    assert_z_close(got_rows[:, 4], ref["results"]["Z"])
    if ncores == 1:
        # whole call on the slice: posteriors, ratio, cZ
        got = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=100,
                                             n_cores=1, return_posteriors=True)
        for i in range(2):
            assert_posterior_close(got["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"jp{i}")
        assert_posterior_close(got["difference.posterior"].values, ref["difference.posterior"], what="ratio")
        assert_z_close(got["results"]["Z"].to_numpy(), ref["results"]["Z"])
        assert_cz_close(got["results"]["cZ"].to_numpy(), ref["results"]["cZ"], got["results"]["Z"].to_numpy(),
                        ref["results"]["Z"])


def test_config4_slice_modes_full_bootstrap(api, oracle):
    models, counts, _, prior, _ = _bench_slice("4", 48, two_groups=False)
    api.set_rand("glibc")
    got = api.scde_posteriors(models, counts, prior, n_randomizations=100, return_individual_posterior_modes=True,
                              n_cores=1)
    ref = oracle.scde_posteriors(models, counts, prior["x"], n_randomizations=100,
                                 return_individual_posterior_modes=True, n_cores=1)
    assert_posterior_close(got["jp"], ref["jp"], what="jp")
    np.testing.assert_array_equal(got["modes"], ref["modes"])


def test_config5_ms1_kernel_3000_cells():
    """k_wpca_ms1 (npcs = 1, 10 starts, one workgroup per 5 starts) at 3,000 cells."""
    from oracle import wpca as W
    from scde_amd import pagoda as PG
    n, d, nstarts, nsh = 3000, 60, 10, 1
    rng = np.random.default_rng(3000)
    m = np.outer(rng.normal(size=n), rng.normal(size=d)) * 2.0 + 0.4 * rng.normal(size=(n, d))
    w = rng.uniform(0.05, 1.0, size=(n, d))
    w[rng.uniform(size=w.shape) < 0.15] = 1e-3
    m = m - (m * w).sum(0) / w.sum(0)
    starts = W.RState(11).unif_rand((1 + nsh) * nstarts * d)
    perms = W.shuffle_perms(5, nsh, d, n)
    ref = W.baileyWPCA(m, w, 1, nstarts, 0, 1e-6, 25, starts, nsh, perms)
    got = PG.baileyWPCA(m, w, 1, nstarts, 0, 1e-6, 25, 1, nsh, starts=starts, perms=perms)
    for key, rel in (("rotation", 1e-7), ("scores", 1e-7), ("scoreweights", 1e-9)):
        a, b = np.asarray(got[key]), np.asarray(ref[key])
        scale = np.maximum(np.abs(a).max(0), np.abs(b).max(0))
        assert np.all(np.abs(a - b).max(0) <= rel * scale), key
    np.testing.assert_allclose(got["var"], ref["var"], rtol=1e-8)
    assert got["totvar"] == pytest.approx(ref["totvar"], rel=1e-12)
    np.testing.assert_allclose(got["randvar"], ref["randvar"], rtol=1e-8)


def test_config3_host_pipeline_equals_device_resident(api):
    """Full config 3 (20,000 x 1,000: an 80 MB matrix, above the 32 MB pipelining threshold):
    scde_expression_difference_host uploads the counts in two column ranges, the first in pieces
    whose unique sets and tables start as each lands (option pieces), and builds the second
    group's unique sets and posterior on the peer lane beside the first group's
    (engine.hip de_run, lanes = 2); the table must equal, bit for bit, the device-resident entry
    on the same counts with the groups one after the other (lanes = 1, no pipelining)."""
    import ctypes
    import bench
    from scde_amd._lib import DEParams, check, lib
    from scde_amd.models import model_matrix
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS["3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    mat = np.asfortranarray(counts, dtype=np.int32)
    N, C = mat.shape
    assert mat.nbytes >= 32 << 20
    codes = np.ascontiguousarray(np.asarray(groups), np.int32)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    ctx = api.default_context()
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px), 100, 1,
                      0, N, 0.0, api.get_rand_kind(), 1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    hosts = []
    try:
        # the first group's columns in 4 (default), 3 (uneven) pieces or one; the repeat reuses the
        # context's buffers and streams
        for pieces in (4, 4, 3, 1, 8):
            ctx.set_option("pieces", pieces)
            host = np.zeros((N, 6), order="F")
            check(lib().scde_expression_difference_host(ctx.handle, vp(mat), N, N, ctypes.byref(params), vp(host),
                                                        None, None, None))
            hosts.append(host)
    finally:
        ctx.set_option("pieces", 5)
    dc = api.DeviceCounts(ctx, mat)
    try:
        dev = np.zeros((N, 6), order="F")
        ctx.set_option("lanes", 1)  # the two group posteriors one after the other
        check(lib().scde_expression_difference_dev(ctx.handle, dc.ptr, N, N, ctypes.byref(params), vp(dev), None,
                                                   None, None))
    finally:
        ctx.set_option("lanes", 2)
        dc.free()
    for host in hosts:
        assert np.isfinite(host[:, :4]).all()
        np.testing.assert_array_equal(host, dev)
