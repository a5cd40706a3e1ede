"""Weighted PCA (bwpca / pagoda.pathway.wPCA; src/bwpca.cpp) on the GPU vs the CPU oracle.

Host-only checks (no GPU): the library's R RNG and shuffle permutations equal the
oracle's restatement and R's published outputs.

GPU parity bar (rounding-order differences only, the same random starts on both sides):
rotation / scores / scoreweights 1e-7 relative to the column scale, var 1e-8 relative,
totvar 1e-12 relative; EM iteration counts equal except where the stop test sees
rounding noise (converged runs).  "Parity unpinned" in the sense of
SURVEY.md section 8(c): no R here, the oracle is the C restatement (oracle/bwpca_oracle.c),
cross-checked against an independent numpy restatement and numpy's SVD
(tests/test_wpca_oracle.py).
"""
import numpy as np
import pytest

from oracle import wpca as W


def _problem(n, d, seed, rank=3, zero_frac=0.0):
    rng = np.random.default_rng(seed)
    L = rng.normal(size=(n, rank)) * np.array([3.0, 1.8, 1.0, 0.6, 0.4, 0.3][:rank])
    R = rng.normal(size=(rank, d))
    m = L @ R + 0.3 * rng.normal(size=(n, d))
    w = rng.uniform(0.05, 1.0, size=(n, d))
    if zero_frac:
        w[rng.uniform(size=w.shape) < zero_frac] = 0.0
    m = m - (m * w).sum(0) / w.sum(0)
    return m, w


def _close_cols(a, b, rel, what):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, what
    scale = np.maximum(np.abs(a).max(0), np.abs(b).max(0))
    err = np.abs(a - b).max(0)
    assert np.all(err <= rel * scale + 1e-300), f"{what}: max err {err} vs scale {scale}"


def _check(got, ref, what=""):
    _close_cols(got["rotation"], ref["rotation"], 1e-7, what + " rotation")
    _close_cols(got["scores"], ref["scores"], 1e-7, what + " scores")
    _close_cols(got["scoreweights"], ref["scoreweights"], 1e-9, what + " scoreweights")
    np.testing.assert_allclose(got["var"], ref["var"], rtol=1e-8, err_msg=what + " var")
    assert got["totvar"] == pytest.approx(ref["totvar"], rel=1e-12)
    if "randvar" in ref:
        np.testing.assert_allclose(got["randvar"], ref["randvar"], rtol=1e-8, err_msg=what + " randvar")


# ------------------------------------------------------------------ host only
def test_library_r_rng_matches_oracle_and_r():
    from scde_amd import pagoda as PG
    for seed in (1, 123, 42, 2**31 - 1):
        np.testing.assert_array_equal(PG.RState(seed).unif_rand(5000), W.RState(seed).unif_rand(5000))
        np.testing.assert_array_equal(PG.RState(seed).sample(1000, 300), W.RState(seed).sample(1000, 300))
    assert PG.RState(1).sample(10, 10).tolist() == [9, 4, 7, 1, 2, 5, 3, 10, 6, 8]
    np.testing.assert_allclose(PG.RState(1).unif_rand(3), [0.2655087, 0.3721239, 0.5728534], atol=5e-8)
    np.testing.assert_array_equal(PG.shuffle_perms(11, 3, 7, 64), W.shuffle_perms(11, 3, 7, 64))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("K,nstarts,smooth,tol,nsh", [
    (1, 3, 0, 1e-6, 0),
    (2, 3, 0, 1e-6, 2),
    (3, 2, 0, 0.0, 0),
    (2, 2, 5, 1e-6, 0),
    (4, 1, 0, 1e-6, 1),
])
def test_baileyWPCA_matches_oracle(K, nstarts, smooth, tol, nsh):
    """The .Call mirror (scde_baileyWPCA) against o_baileyWPCA on identical starts/perms."""
    from scde_amd import pagoda as PG
    n, d = 150, 40
    m, w = _problem(n, d, 100 + K, rank=4)
    starts = W.RState(7 + K).unif_rand((1 + nsh) * nstarts * d * K)
    perms = W.shuffle_perms(3, nsh, d, n) if nsh else None
    ref = W.baileyWPCA(m, w, K, nstarts, smooth, tol, 25, starts, nsh, perms)
    got = PG.baileyWPCA(m, w, K, nstarts, smooth, tol, 25, 1, nsh, starts=starts, perms=perms)
    _check(got, ref, f"K={K}")


@pytest.mark.gpu
def test_batch_iterations_and_problem_independence():
    """A batch of mixed problems (K 1..3, column subsets, shuffled rows) equals the
    oracle problem by problem, EM iteration counts included."""
    from scde_amd import api
    from scde_amd import pagoda as PG
    n, G = 120, 90
    m, w = _problem(n, G, 5, rank=3, zero_frac=0.05)
    rng = np.random.default_rng(1)
    ctx = api.default_context()
    dev = PG.DeviceMatrixPair(ctx, m.T, w.T)
    b = PG.WpcaBatch()
    specs = []
    rs = W.RState(99)
    for p in range(14):
        d = int(rng.integers(12, 70))  # K <= d / 4: EM from different starts stays well conditioned
        cols = rng.choice(G, size=d, replace=False)
        K = 1 + p % 3
        ns = 1 + p % 4
        k = min(K, d)
        st = rs.unif_rand(ns * d * k)
        perm = W.shuffle_perms(p, 1, d, n)[0] if p % 5 == 4 else None
        b.add(cols, K, ns, st, perm)
        specs.append((cols, K, ns, st, perm))
    try:
        res = b.run(dev, want_iterations=True)
    finally:
        dev.free()
    same = 0
    for p, (cols, K, ns, st, perm) in enumerate(specs):
        mm, ww = m[:, cols], w[:, cols]
        if perm is not None:
            mm = np.take_along_axis(mm, perm.T, axis=0)
            ww = np.take_along_axis(ww, perm.T, axis=0)
        ref = W.baileyWPCA(mm, ww, K, ns, 0, 1e-6, 25, st)
        _check(res[p], ref, f"problem {p}")
        # EM stops when the residual's relative decrease drops below em.tol while still
        # decreasing; once converged to rounding level that sign is noise, so a run may stop
        # an iteration or two apart (with the same answer, checked above)
        same += int(np.array_equal(res[p]["iterations"], ref["iterations"]))
        cm = (mm * np.abs(ref["rotation"][:, 0])).mean(axis=1)
        np.testing.assert_allclose(res[p]["colmeans"][:, 0], cm, rtol=1e-9, atol=1e-12)
    assert same >= len(specs) * 3 // 4, f"iteration counts equal for only {same}/{len(specs)} problems"


@pytest.mark.gpu
def test_coefficients_outside_lds():
    """n x K too large for LDS: the working coefficients live in global scratch."""
    from scde_amd import pagoda as PG
    n, d, K = 5200, 24, 4
    m, w = _problem(n, d, 8, rank=5)
    starts = W.RState(4).unif_rand(2 * d * K)
    ref = W.baileyWPCA(m, w, K, 2, 0, 1e-6, 25, starts)
    got = PG.baileyWPCA(m, w, K, 2, 0, 1e-6, 25, 1, 0, starts=starts)
    _check(got, ref, "global C")


@pytest.mark.gpu
def test_large_gene_set_and_zero_weight_cells():
    """d > block size (several genes per wave and thread), cells with no weight in the set
    (singular normal equations -> zero coefficients on both sides)."""
    from scde_amd import pagoda as PG
    n, d = 200, 700
    m, w = _problem(n, d, 12, rank=3)
    w[:3, :] = 0.0
    starts = W.RState(6).unif_rand(2 * d * 2)
    ref = W.baileyWPCA(m, w, 2, 2, 0, 1e-6, 25, starts)
    got = PG.baileyWPCA(m, w, 2, 2, 0, 1e-6, 25, 1, 0, starts=starts)
    _check(got, ref, "d=700")
    assert np.all(got["scores"][:3] == 0)


@pytest.mark.gpu
def test_pagoda_pathway_wPCA_matches_oracle():
    """End to end: gene-set filtering, random gene sets (R sample), internal shuffles,
    orientation flips, avar / xv normalisation -- one batched device call."""
    from scde_amd import pagoda as PG
    rng = np.random.default_rng(2024)
    G, n = 240, 96
    m, w = _problem(n, G, 77, rank=4)
    mat, matw = m.T.copy(), w.T.copy()          # genes x cells, like varinfo$mat
    mat[5] = 1.0                                # a constant row (dropped)
    genes = [f"g{i}" for i in range(G)]
    setenv = {f"GO:{k:04d}": list(rng.choice(genes, size=int(rng.integers(8, 60)), replace=False))
              for k in range(9)}
    setenv["GO:tiny"] = genes[:3]
    batch = np.array(["a", "b"] * (n // 2))
    kw = dict(n_components=2, n_randomizations=4, n_internal_shuffles=2, n_starts=3, seed=11, rand_seed=5)
    got = PG.pagoda_pathway_wPCA({"mat": mat, "matw": matw, "genes": genes, "batch": batch}, setenv, **kw)
    ref = W.pagoda_pathway_wPCA(mat, matw, genes, setenv, batch=batch, **kw)
    assert list(got) == list(ref) and "GO:tiny" not in got
    for go in ref:
        a, b = got[go], ref[go]
        assert a["n"] == b["n"]
        _check(a["xp"], b["xp"], go)
        np.testing.assert_allclose(a["z"], b["z"], rtol=1e-8, err_msg=go)
        np.testing.assert_allclose(a["xv"], b["xv"], rtol=1e-6, atol=1e-9, err_msg=go)
