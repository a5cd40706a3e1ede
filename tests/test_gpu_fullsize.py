"""GPU parity at the BASELINE shapes, beyond the 64-gene slices of test_gpu_configs.py:

* config 3 WHOLE: the bench's own 20,000 x 1,000 data set (500/500 cells), B = 100, n.cores = 16
  seeding, through scde_expression_difference_host (two-range pipelined upload, device gene
  ordering, compacted fallback list, device BH over all genes), against the oracle's table for
  every gene (tests/golden/config3_full.npz, tools/make_config3_fixture.py): lb/mle/ub/ce exact,
  Z and the global-BH cZ (R/functions.R:5051, 3527-3531) within conftest's tolerances; the joint
  and ratio posteriors of a 48-gene window straddling the first n.cores chunk boundary (gene
  1,250) against the live oracle;
* config 4: a 1,000-gene x 2,000-cell slice, B = 100, postflag 1 (modes exact), oracle run in
  worker processes (mclapply-style contiguous chunks of the n.cores = 1 call: one draw list);
* config 2b: a 256-gene slice of the batch-corrected bench set, B = 100, all three tables and
  every posterior.
"""
import os

import numpy as np
import pytest

from conftest import assert_cz_close, assert_posterior_close, assert_z_close

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


def _posteriors_chunk(job):
    models, sub, px, nboot, lo, ntot = job
    from oracle import oracle as O
    O.set_rng(0)
    r = O.scde_posteriors(models, np.ascontiguousarray(sub), px, n_randomizations=nboot,
                          return_individual_posterior_modes=True, n_cores=1, gene_offset=lo, ngenes_total=ntot)
    return lo, r["jp"], r["modes"]


def _workers():
    # the GPU box's CPU share is 16 (os.cpu_count() shows the whole machine)
    return max(1, min(16, os.cpu_count() or 1))


def test_config3_whole_table_vs_oracle(api, oracle):
    import bench
    g = np.load(os.path.join(ROOT, "tests", "golden", "config3_full.npz"), allow_pickle=False)
    seed, ngenes, ncells, nboot, ncores = (int(v) for v in g["meta"])
    cfg = bench.CONFIGS["3"]
    assert (seed, ngenes, ncells) == (cfg["seed"], cfg["genes"], cfg["cells"])
    models, counts, groups = bench.synthetic(seed, ngenes, ncells, two_groups=True)
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    api.set_rand("glibc")
    got = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nboot,
                                         n_cores=ncores, return_posteriors=True)
    res, want = got["results"], g["results"]
    for j, k in enumerate(("lb", "mle", "ub", "ce")):
        np.testing.assert_array_equal(res[k].to_numpy(), want[:, j], err_msg=k)
    assert_z_close(res["Z"].to_numpy(), want[:, 4], what="Z")
    assert_cz_close(res["cZ"].to_numpy(), want[:, 5], res["Z"].to_numpy(), want[:, 4], what="cZ")
    # posteriors of a window across the first chunk boundary (two draw lists), live oracle
    lo, hi = 1226, 1274
    ref = oracle.scde_expression_difference(models, np.ascontiguousarray(counts[lo:hi]), prior["x"], prior["y"],
                                            groups, n_randomizations=nboot, n_cores=ncores, gene_offset=lo,
                                            ngenes_total=ngenes, return_posteriors=True)
    for i in range(2):
        assert_posterior_close(got["joint.posteriors"][i][lo:hi], ref["joint.posteriors"][i], what=f"jp{i}")
    assert_posterior_close(got["difference.posterior"].values[lo:hi], ref["difference.posterior"], what="ratio")


def test_config4_1000_gene_slice_modes(api):
    import multiprocessing as mp

    import bench
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS["4"]
    models, counts, _ = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=False)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    n = 1000
    sub = np.asfortranarray(counts[:n])
    api.set_rand("glibc")
    got = api.scde_posteriors(models, sub, prior, n_randomizations=100, return_individual_posterior_modes=True,
                              n_cores=1)
    # the host entry's piece pipeline (forced below its 32 MB threshold): the same bits
    ctx = api.default_context()
    try:
        # and the read-backs: modes piece by piece / jp in gene chunks from the read-back thread
        # (jp_chunks 1 = one bootstrap launch; modes_overlap 0 = plain copies after the bootstrap)
        for pieces, chunks, overlap in ((3, 4, 1), (8, 3, 1), (8, 1, 1), (3, 7, 1), (3, 4, 0)):
            ctx.set_option("pipeline_mb", 0)
            ctx.set_option("pieces", pieces)
            ctx.set_option("jp_chunks", chunks)
            ctx.set_option("modes_overlap", overlap)
            api.set_rand("glibc")
            pip = api.scde_posteriors(models, sub, prior, n_randomizations=100,
                                      return_individual_posterior_modes=True, n_cores=1)
            np.testing.assert_array_equal(pip["jp"], got["jp"], err_msg=f"pieces {pieces} chunks {chunks}")
            np.testing.assert_array_equal(pip["modes"], got["modes"], err_msg=f"pieces {pieces} chunks {chunks}")
        # the device-resident entry (counts in HBM; its jp read back in gene chunks, its modes once
        # the tables are done) gives the same bits
        import ctypes
        from scde_amd._lib import check, lib
        from scde_amd.models import model_matrix
        mm, lt, sq = model_matrix(models)
        px = np.ascontiguousarray(prior["x"], np.float64)
        N, C = sub.shape
        cellidx = np.arange(C, dtype=np.int32)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        dc = api.DeviceCounts(ctx, sub)
        try:
            for chunks, overlap in ((4, 1), (1, 1), (4, 0)):
                ctx.set_option("jp_chunks", chunks)
                ctx.set_option("modes_overlap", overlap)
                jp = np.zeros((N, len(px)), order="F")
                modes = np.zeros((N, C), order="F")
                api.set_rand("glibc")
                check(lib().scde_posteriors_dev(ctx.handle, dc.ptr, N, N, P(cellidx), C, P(mm), lt, sq, P(px), len(px),
                                                100, 1, 0, N, 1, 0, None, None, None, 0, P(jp), P(modes), None))
                np.testing.assert_array_equal(jp, got["jp"], err_msg=f"device entry, chunks {chunks}")
                np.testing.assert_array_equal(modes, got["modes"], err_msg=f"device entry, chunks {chunks}")
        finally:
            dc.free()
    finally:
        ctx.set_option("pipeline_mb", 32)
        ctx.set_option("pieces", 5)
        ctx.set_option("jp_chunks", 4)
        ctx.set_option("modes_overlap", 1)
    px = np.asarray(prior["x"])
    w = _workers()
    bounds = np.linspace(0, n, w + 1).astype(int)
    jobs = [(models, sub[bounds[i]:bounds[i + 1]], px, 100, int(bounds[i]), n) for i in range(w)
            if bounds[i + 1] > bounds[i]]
    with mp.get_context("spawn").Pool(len(jobs)) as pool:
        parts = pool.map(_posteriors_chunk, jobs)
    jp = np.vstack([p[1] for p in parts])
    modes = np.vstack([p[2] for p in parts])
    assert_posterior_close(got["jp"], jp, what="jp")
    np.testing.assert_array_equal(got["modes"], modes)


def test_config2b_slice_b100(api, oracle):
    import bench
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS["2b"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    batch = bench.synthetic_batch(cfg["seed"], cfg["cells"], cfg["nbatch"])
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    sub = np.asfortranarray(counts[:256])
    api.set_rand("glibc")
    out = api.scde_expression_difference(models, sub, prior, groups=list(groups), batch=batch, n_randomizations=100,
                                         n_cores=1, return_posteriors=True)
    ref = oracle.scde_expression_difference_batch(models, sub, prior["x"], prior["y"], groups, list(batch),
                                                  n_randomizations=100, n_cores=1, return_posteriors=True)
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


def test_config3_host_pipeline_after_call_history(api):
    """a full-size wrong table once appeared only after other calls in the same
    process (the dropped direct-row experiment).  The per-call state kept in grow-only buffers (the
    list pass's `wide` count and entries, the `redo` flags and list, `pmask`, partial rows, the
    unique sets' fixed-width offsets and bitmaps, the peer lane's workspace) must not leak from one
    call into the next.  So: the device-resident config-3 table on a fresh context (one lane, no
    pipelining) is the reference; then, on another fresh context, a varied history -- a batch DE,
    scde.posteriors with modes (postflag 1), a smaller DE (fewer genes: every per-gene buffer holds
    longer stale contents), a DE with the list pass forced and capped (gene_rows = 1,
    gene_list_cap = 41: stale list entries past the cap), a DE with NaN-free but wider counts --
    and then the full host pipeline twice (4 and 3 pieces, two lanes): both equal the reference bit
    for bit."""
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
    codes = np.ascontiguousarray(np.asarray(groups), np.int32)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px), 100, 1,
                      0, N, 0.0, api.get_rand_kind(), 1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    api.set_rand("glibc")
    ref_ctx = api.Context(0)
    try:
        ref_ctx.set_option("lanes", 1)
        dc = api.DeviceCounts(ref_ctx, mat)
        ref = np.zeros((N, 6), order="F")
        check(lib().scde_expression_difference_dev(ref_ctx.handle, dc.ptr, N, N, ctypes.byref(params), vp(ref), None,
                                                   None, None))
        dc.free()
    finally:
        ref_ctx.close()
    ctx = api.Context(0)
    try:
        # history: batch DE (four posteriors, 1601-column second level) on a slice
        sub = np.asfortranarray(mat[:700])
        batch = np.array(["b%d" % (c % 2) for c in range(C)], dtype=object)
        api.scde_expression_difference(models, sub, prior, groups=list(groups), batch=batch, n_randomizations=30,
                                       n_cores=3, ctx=ctx)
        # scde.posteriors with posterior modes (one group, all cells)
        api.scde_posteriors(models, np.asfortranarray(mat[:1500]), prior, n_randomizations=40,
                            return_individual_posterior_modes=True, n_cores=2, ctx=ctx)
        # a smaller DE, then one with the list pass forced and capped off a multiple of 4
        api.scde_expression_difference(models, np.asfortranarray(mat[5000:9000]), prior, groups=list(groups),
                                       n_randomizations=100, n_cores=1, ctx=ctx)
        ctx.set_option("gene_rows", 1)
        ctx.set_option("gene_list_cap", 41)
        api.scde_expression_difference(models, np.asfortranarray(mat[:3000]), prior, groups=list(groups),
                                       n_randomizations=100, n_cores=5, ctx=ctx)
        ctx.set_option("gene_rows", 4)
        ctx.set_option("gene_list_cap", 0)
        # counts past the fixed bitmaps' 65,535 in a slice of the matrix (the exact unique rebuild)
        wide = np.asfortranarray(mat[:800].copy())
        wide[::97, ::13] += 70000
        api.scde_expression_difference(models, wide, prior, groups=list(groups), n_randomizations=20, n_cores=1,
                                       ctx=ctx)
        for pieces in (4, 3):
            ctx.set_option("pieces", pieces)
            host = np.zeros((N, 6), order="F")
            check(lib().scde_expression_difference_host(ctx.handle, vp(mat), N, N, ctypes.byref(params), vp(host),
                                                        None, None, None))
            bad = np.nonzero(np.any(host != ref, axis=1))[0]
            assert bad.size == 0, (f"pieces {pieces}: {bad.size} of {N} genes differ after the call history; "
                                   f"first gene {bad[0]}: {host[bad[0]]} vs {ref[bad[0]]}")
    finally:
        ctx.close()


def test_host_upload_16bit_counts(api):
    """Host-count ranges of 8 MB and more go up as 16-bit counts (option upload_u16: narrowed on the
    host in pinned ring slots, widened on the device, the counts outside [0, 65535] listed and
    patched in).  Config 3's full host DE (whose synthetic matrix holds 3 counts past 65,535) and
    the same matrix with a count past 16 bits every 997 genes x 7 cells equal the int32 upload bit
    for bit, as does a config-4 posteriors slice with such counts; a negative count still fails the
    call as it does on the int32 path."""
    import ctypes
    import bench
    from scde_amd._lib import DEParams, check, lib
    from scde_amd.models import model_matrix
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS["3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    N, C = counts.shape
    codes = np.ascontiguousarray(np.asarray(groups), np.int32)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px), 100, 1,
                      0, N, 0.0, api.get_rand_kind(), 1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    mat = np.asfortranarray(counts, dtype=np.int32)
    wide = mat.copy(order="F")
    wide[::997, ::7] += 70000  # past 16 bits in every range
    ctx = api.Context(0)
    try:
        def de(m, u16):
            ctx.set_option("upload_u16", 2 * u16)  # (2: DE host calls too)
            out = np.zeros((N, 6), order="F")
            api.set_rand("glibc")
            check(lib().scde_expression_difference_host(ctx.handle, vp(m), N, N, ctypes.byref(params), vp(out), None,
                                                        None, None))
            return out
        for m, what in ((mat, "config 3"), (wide, "counts past 65535")):
            ref = de(m, 0)
            got = de(m, 1)
            bad = np.nonzero(np.any(got != ref, axis=1))[0]
            assert bad.size == 0, f"{what}: {bad.size} genes differ, first {bad[:3]}"
        neg = mat.copy(order="F")
        neg[123, 456] = -3
        for u16 in (0, 1):
            ctx.set_option("upload_u16", 2 * u16)
            with pytest.raises(Exception) as e:
                out = np.zeros((N, 6), order="F")
                check(lib().scde_expression_difference_host(ctx.handle, vp(neg), N, N, ctypes.byref(params), vp(out),
                                                            None, None, None))
            assert "negative" in str(e.value).lower() or "count" in str(e.value).lower(), str(e.value)
        # an error in the middle of a 16-bit upload (a slot's copy, injected through the test hook)
        # fails the call, and the next 16-bit upload on the same context completes with the same
        # table (the error path reopens the slot ring: ADVICE r05, engine.hip upload_cols_u16)
        ref_mat = de(mat, 0)
        ctx.inject_fault("u16_slot", 1)
        with pytest.raises(Exception):
            de(mat, 1)
        np.testing.assert_array_equal(de(mat, 1), ref_mat)
        # scde.posteriors host entry (one range in pieces), modes included
        c4 = bench.CONFIGS["4"]
        m4, k4, _ = bench.synthetic(c4["seed"], 4000, c4["cells"], two_groups=False)
        p4 = expression_prior(m4, k4, length_out=bench.LENGTH_OUT)
        sub = np.asfortranarray(k4)
        sub[::31, ::5] += 66000
        res = {}
        for u16 in (0, 1):
            ctx.set_option("upload_u16", u16)
            api.set_rand("glibc")
            res[u16] = api.scde_posteriors(m4, sub, p4, n_randomizations=100, return_individual_posterior_modes=True,
                                           n_cores=1, ctx=ctx)
        np.testing.assert_array_equal(res[1]["jp"], res[0]["jp"])
        np.testing.assert_array_equal(res[1]["modes"], res[0]["modes"])
    finally:
        ctx.close()
