"""CPU checks of the weighted-PCA oracle (oracle/bwpca_oracle.c, oracle/wpca.py).

* R's RNG restatement against R's published outputs (set.seed + runif / sample).
* The C restatement of baileyWPCA (src/bwpca.cpp) against an independent numpy
  restatement written from the same source, and against numpy's SVD where EM-PCA must
  reach the principal subspace (unit weights, many iterations).
"""
import numpy as np
import pytest

from oracle import wpca as W


# ------------------------------------------------------------------ R RNG
def test_r_runif_known_answers():
    # R >= 1.7: set.seed(1); runif(5) / set.seed(123); runif(5) / set.seed(42); runif(2)
    np.testing.assert_allclose(W.RState(1).unif_rand(5),
                               [0.2655087, 0.3721239, 0.5728534, 0.9082078, 0.2016819], atol=5e-8)
    np.testing.assert_allclose(W.RState(123).unif_rand(5),
                               [0.2875775, 0.7883051, 0.4089769, 0.8830174, 0.9404673], atol=5e-8)
    np.testing.assert_allclose(W.RState(42).unif_rand(2), [0.9148060, 0.9370754], atol=5e-8)


def test_r_sample_known_answers():
    # R >= 3.6 (sample.kind = "Rejection"): set.seed(s); sample(1:10)
    assert W.RState(1).sample(10, 10).tolist() == [9, 4, 7, 1, 2, 5, 3, 10, 6, 8]
    assert W.RState(123).sample(10, 10).tolist() == [3, 10, 2, 8, 6, 9, 1, 7, 5, 4]
    assert W.RState(42).sample(10, 10).tolist() == [1, 5, 10, 8, 2, 4, 6, 9, 7, 3]


def test_shuffle_perms_are_permutations():
    p = W.shuffle_perms(7, 3, 5, 40)
    for s in range(3):
        for c in range(5):
            assert sorted(p[s, c].tolist()) == list(range(40))
    # columns continue from the previous column's order; each call restarts from 0..n-1
    assert not np.array_equal(p[0, 0], p[0, 1])


# ------------------------------------------------------------------ numpy restatement
def _np_qr_start(X):
    """LAPACK dgeqr2 + dorg2r Q (Householder, beta = -sign(alpha) * norm)."""
    A = X.copy()
    d, K = A.shape
    vs, taus = [], []
    for i in range(K):
        x = A[i:, i].copy()
        alpha, xn = x[0], np.linalg.norm(x[1:])
        if xn == 0:
            tau, v = 0.0, np.r_[1.0, np.zeros(len(x) - 1)]
            beta = alpha
        else:
            beta = -np.copysign(np.hypot(alpha, xn), alpha)
            tau = (beta - alpha) / beta
            v = np.r_[1.0, x[1:] / (alpha - beta)]
        A[i:, i:] -= tau * np.outer(v, v @ A[i:, i:])
        vs.append(v)
        taus.append(tau)
    Q = np.eye(d, K)
    for i in reversed(range(K)):
        Q[i:, :] -= taus[i] * np.outer(vs[i], vs[i] @ Q[i:, :])
    return Q


def _np_round(m, w, nstarts, K, maxiter, tol, starts):
    n, d = m.shape
    best = None
    bestpres = -1
    for s in range(nstarts):
        E = _np_qr_start(starts[s * d * K:(s + 1) * d * K].reshape(K, d).T)
        pres = bpres = np.finfo(float).max
        bc = be = None
        ii = 0
        while ii < maxiter:
            coef = np.empty((n, K))
            for j in range(n):
                A = E.T @ (E * w[j][:, None])
                b = (m[j] * w[j]) @ E
                coef[j] = np.linalg.solve(A, b)
            dat = m.copy()
            for k in range(K):
                cw = w * coef[:, k][:, None]
                E[:, k] = (dat * cw).sum(0) / (cw * coef[:, k][:, None]).sum(0)
                if k != K - 1:
                    dat -= np.outer(coef[:, k], E[:, k])
            E[:, 0] /= np.sqrt(E[:, 0] @ E[:, 0])
            for k in range(1, K):
                for kx in range(k):
                    E[:, k] -= (E[:, k] @ E[:, kx]) * E[:, kx]
                E[:, k] /= np.sqrt(E[:, k] @ E[:, k])
            npres = (((coef @ E.T - m) * np.sqrt(w)) ** 2).sum()
            if npres < bpres:
                bpres, bc, be = npres, coef.copy(), E.copy()
            if tol > 0 and ii > 0 and (pres - npres) / npres < tol and pres > npres:
                pres = npres
                break
            ii += 1
            pres = npres
        if s == 0 or pres < bestpres:
            bestpres, best = bpres, (bc, be)
    return best


def _problem(n, d, seed, rank=2):
    rng = np.random.default_rng(seed)
    L = rng.normal(size=(n, rank)) * np.array([3.0, 1.5, 0.8][:rank])
    R = rng.normal(size=(rank, d))
    m = L @ R + 0.3 * rng.normal(size=(n, d))
    w = rng.uniform(0.05, 1.0, size=(n, d))
    m = m - (m * w).sum(0) / w.sum(0)
    return m, w


@pytest.mark.parametrize("K,nstarts,tol", [(1, 3, 1e-6), (2, 2, 1e-6), (3, 2, 0.0)])
def test_c_oracle_matches_numpy_restatement(K, nstarts, tol):
    n, d = 60, 25
    m, w = _problem(n, d, 10 + K, rank=3)
    starts = W.RState(5 + K).unif_rand(nstarts * d * K)
    r = W.baileyWPCA(m, w, K, nstarts, 0, tol, 25, starts)
    bc, be = _np_round(m, w, nstarts, K, 25, tol, starts)
    np.testing.assert_allclose(r["rotation"], be, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(r["scores"], bc, rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(r["scoreweights"], w @ np.abs(be), rtol=1e-12)
    tot = ((m * np.sqrt(w)) ** 2).sum()
    assert r["totvar"] == pytest.approx(tot, rel=1e-13)
    dat = np.zeros_like(m)
    prev = 0.0
    for k in range(K):
        dat += np.outer(bc[:, k], be[:, k])
        npres = (((dat - m) * np.sqrt(w)) ** 2).sum()
        assert r["var"][k] == pytest.approx(tot - npres - prev, rel=1e-8)
        prev = tot - npres


def test_unit_weights_reach_principal_subspace():
    """EM-PCA with unit weights converges to the SVD's leading right singular vectors."""
    n, d = 80, 12
    m, _ = _problem(n, d, 3, rank=2)
    m = m - m.mean(0)
    w = np.ones_like(m)
    starts = W.RState(9).unif_rand(d * 2)
    r = W.baileyWPCA(m, w, 2, 1, 0, 0.0, 400, starts)
    _, s, vt = np.linalg.svd(m, full_matrices=False)
    for k in range(2):
        assert abs(abs(r["rotation"][:, k] @ vt[k]) - 1) < 1e-8
    np.testing.assert_allclose(r["var"], s[:2] ** 2, rtol=1e-8)


def test_bwpca_wrapper_shuffles_and_smoothing():
    n, d = 50, 16
    m, w = _problem(n, d, 21)
    r = W.bwpca(m, w, npcs=2, nstarts=2, smooth=5, n_shuffles=3, seed=3)
    assert r["rotation"].shape == (d, 2) and r["randvar"].shape == (3,)
    assert np.all(np.isfinite(r["randvar"]))
    # orthonormal rotation
    np.testing.assert_allclose(r["rotation"].T @ r["rotation"], np.eye(2), atol=1e-12)
    # a shuffled matrix has no more structure than the real one on PC1
    assert np.all(r["randvar"] < r["var"][0])
    # unit weights: NULL matw path forces nstarts = 1
    r1 = W.bwpca(m, None, npcs=1, nstarts=5)
    assert r1["iterations"].shape[0] >= 1
