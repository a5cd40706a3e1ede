"""Cross-stream ordering, checked deterministically.

The host pipeline hands data between streams and threads at fixed points: each piece's uploads
(copy stream -> unique-set stream), each piece's unique sets and tables (piece stream -> main
stream), the offsets/modes copies, the aux stream's set-up (-> the bootstrap), the peer lane's
start and finish (main <-> peer stream), the 16-bit upload ring and the read-back thread's events.
A missing or misplaced wait at one of them gives wrong results only when the producer happens to
run late, which a plain run rarely shows.  The test hook "handoff_spin" (include/scde_hip.h
scde_ctx_inject_fault) queues a one-wave spin kernel of ~1 ms on a stream after each of its
cross-stream waits (so the work it produces next starts late) and right before every such event, so
the producer is always late: any consumer that does not wait reads unwritten data every time.  The
pipelined layouts, the posteriors read-backs and the config-3 host pipeline after a call history
must then equal the runs without spins bit for bit; the negative control drops one wait
("skip_lane_join") and must see different results.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPIN = 2_500_000  # shader clocks (~1 ms at 2.4 GHz): longer than any consumer's kernel at these sizes


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


def _de(api, ctx, models, counts, prior, groups, nrand, ncores):
    api.set_rand("glibc")
    return api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nrand,
                                          n_cores=ncores, return_posteriors=True, ctx=ctx)


def _diff(a, b, what):
    bad = []
    for i in range(2):
        ne = int(np.sum(a["joint.posteriors"][i] != b["joint.posteriors"][i]))
        if ne:
            bad.append(f"{what} jp{i}: {ne} entries differ")
    for k in ("lb", "mle", "ub", "ce", "Z", "cZ"):
        if not np.array_equal(a["results"][k].to_numpy(), b["results"][k].to_numpy()):
            bad.append(f"{what} {k}")
    return bad


@pytest.mark.parametrize("layout", ["ordered", "reversed", "mixed"])
def test_handoff_spin_pipelined_layouts(api, layout):
    import bench
    from scde_amd.prior import expression_prior
    models, counts, groups = bench.synthetic(8004, 150, 400)
    groups = np.asarray(groups)
    if layout == "reversed":
        groups = 1 - groups
    elif layout == "mixed":
        groups = np.random.default_rng(5).permutation(groups)
    prior = expression_prior(models, counts, length_out=400)
    runs = {"default": {}, "pipelined": {"pipeline_mb": 0, "pieces": 3},
            "pipelined-one-lane": {"pipeline_mb": 0, "pieces": 2, "lanes": 1}}
    ctx = api.Context(0)
    try:
        base = _de(api, ctx, models, counts, prior, groups, 30, 1)
        bad = []
        for name, opts in runs.items():
            for k, v in opts.items():
                ctx.set_option(k, v)
            ctx.inject_fault("handoff_spin", SPIN)
            ctx.reset_stats()
            got = _de(api, ctx, models, counts, prior, groups, 30, 1)
            nspin = ctx.stat("handoff_spins")
            ctx.inject_fault("handoff_spin", 0)
            # the spins really ran at the handoffs: at least the peer lane's start and finish, or
            # (one lane, pipelined) the pieces' uploads and tables
            assert nspin >= 2, (name, nspin)
            bad += _diff(got, base, f"{layout} {name}")
            ctx.set_option("pipeline_mb", 32)
            ctx.set_option("pieces", 5)
            ctx.set_option("lanes", 2)
        assert not bad, bad
    finally:
        ctx.close()


def test_handoff_spin_posteriors_readback(api):
    """scde.posteriors with modes: the modes copies overlap the bootstrap (modes_ev) and the jp
    chunks leave through the read-back thread's events -- with spins, the same bits."""
    import bench
    from scde_amd.prior import expression_prior
    cfg = bench.CONFIGS["4"]
    models, counts, _ = bench.synthetic(cfg["seed"], 400, 600, two_groups=False)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    sub = np.asfortranarray(counts)
    ctx = api.Context(0)
    try:
        api.set_rand("glibc")
        ref = api.scde_posteriors(models, sub, prior, n_randomizations=50, return_individual_posterior_modes=True,
                                  n_cores=1, ctx=ctx)
        for pieces, chunks, overlap in ((3, 4, 1), (1, 1, 1), (3, 4, 0)):
            ctx.set_option("pipeline_mb", 0)
            ctx.set_option("pieces", pieces)
            ctx.set_option("jp_chunks", chunks)
            ctx.set_option("modes_overlap", overlap)
            ctx.inject_fault("handoff_spin", SPIN)
            ctx.reset_stats()
            api.set_rand("glibc")
            got = api.scde_posteriors(models, sub, prior, n_randomizations=50, return_individual_posterior_modes=True,
                                      n_cores=1, ctx=ctx)
            assert ctx.stat("handoff_spins") >= 1
            ctx.inject_fault("handoff_spin", 0)
            np.testing.assert_array_equal(got["jp"], ref["jp"], err_msg=f"pieces {pieces} chunks {chunks}")
            np.testing.assert_array_equal(got["modes"], ref["modes"], err_msg=f"pieces {pieces} chunks {chunks}")
    finally:
        ctx.close()


def test_handoff_spin_config3_after_call_history(api):
    """The config-3 host pipeline (two lanes, 4 pieces, 16-bit upload) after a short call history
    (a batch DE and a smaller DE on the same context), all with spins at every handoff: equal to the
    device-resident one-lane table without spins, bit for bit."""
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
        ctx.inject_fault("handoff_spin", SPIN)
        batch = np.array(["b%d" % (c % 2) for c in range(C)], dtype=object)
        api.scde_expression_difference(models, np.asfortranarray(mat[:700]), prior, groups=list(groups), batch=batch,
                                       n_randomizations=30, n_cores=3, ctx=ctx)
        api.scde_expression_difference(models, np.asfortranarray(mat[5000:9000]), prior, groups=list(groups),
                                       n_randomizations=100, n_cores=1, ctx=ctx)
        for u16 in (2, 0):
            ctx.set_option("upload_u16", u16)
            ctx.reset_stats()
            host = np.zeros((N, 6), order="F")
            check(lib().scde_expression_difference_host(ctx.handle, vp(mat), N, N, ctypes.byref(params), vp(host),
                                                        None, None, None))
            assert ctx.stat("handoff_spins") >= 8, ctx.stat("handoff_spins")  # pieces x lanes, at least
            bad = np.nonzero(np.any(host != ref, axis=1))[0]
            assert bad.size == 0, (f"upload_u16 {u16}: {bad.size} of {N} genes differ with handoff spins; "
                                   f"first gene {bad[0]}: {host[bad[0]]} vs {ref[bad[0]]}")
    finally:
        ctx.close()


def test_handoff_spin_negative_control_skipped_lane_join(api):
    """The hook really catches a missing wait: with the spins on and the main stream's wait for the
    peer lane left out ("skip_lane_join"), the ratio reads the second group's joint posterior before
    the peer lane has written it, and the results differ from the ordered run.  The call before the
    faulted one uses the other grouping, so the stale buffer never holds the right answer."""
    import bench
    from scde_amd.prior import expression_prior
    models, counts, groups = bench.synthetic(8004, 150, 400)
    groups = np.asarray(groups)
    prior = expression_prior(models, counts, length_out=400)
    ctx = api.Context(0)
    try:
        ctx.set_option("lanes", 2)
        ref = _de(api, ctx, models, counts, prior, 1 - groups, 30, 1)
        _de(api, ctx, models, counts, prior, groups, 30, 1)  # leaves the other grouping's posteriors
        ctx.inject_fault("handoff_spin", SPIN)
        ctx.inject_fault("skip_lane_join", 1)
        got = _de(api, ctx, models, counts, prior, 1 - groups, 30, 1)
        ctx.inject_fault("handoff_spin", 0)
        ctx.synchronize()  # drain the peer lane the call did not wait for
        assert _diff(got, ref, "skipped join"), "a skipped lane join went unnoticed under the spins"
        # and the next call (join restored) is exact again
        again = _de(api, ctx, models, counts, prior, 1 - groups, 30, 1)
        assert not _diff(again, ref, "after the skipped join")
    finally:
        ctx.close()
