"""Host-side check of the arithmetic behind k_boot2's grid-stretch skipping,
on oracle tables -- no GPU.

The device bounds a boot's row over a 64-point stretch s by
    UB_bs = ZU_bs + sum_e W_be U_e,s,
with U the per-column stretch maxima split exactly as the bootstrap splits the row
(baseline count-0 columns in ZU, the cell's other column as "its maximum minus the
baseline column's maximum"), and leaves s out of a slab only when UB_bs < m_b - 51 for
every boot of the slab (the post-check against the exact row maximum m_b).  This test
rebuilds those quantities from the oracle's per-cell log-posterior tables and checks that
(1) UB bounds every row value of its stretch, and (2) any stretch the post-check lets go
holds only softmax terms below e^-50, the cut the kernel applies anyway -- so skipping
cannot change an output.
"""
import numpy as np

from conftest import golden


def _tables(nboot=30, ngenes=40):
    from oracle import oracle as O
    g = golden("esmef500.npz")
    from oracle.oracle import MODEL_COLUMNS
    models = {c: g["models"][:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}
    counts = np.asarray(g["counts"])[:ngenes, :20]
    models = {k: v[:20] for k, v in models.items()}
    prior_x = np.linspace(0, np.log10(counts.max() + 1) * 1.1, 401)
    r = O.scde_posteriors(models, counts, prior_x, n_randomizations=nboot, return_individual_posteriors=True,
                          n_cores=1)
    post = np.stack(r["post"])  # C x N x G: T[c, count(g, c)] rows
    C = post.shape[0]
    draws = O.draw_stream(1, C, nboot * C).reshape(nboot, C)
    W = np.zeros((nboot, C))
    for b in range(nboot):
        np.add.at(W[b], draws[b], 1.0)
    return post, W, counts


def test_stretch_bounds_and_post_check():
    post, W, counts = _tables()
    C, N, G = post.shape
    nst = (G + 63) // 64
    zero = counts == 0  # N x C: cells whose column is the count-0 (baseline) column
    checked = skipped = 0
    for g in range(N):
        T = post[:, g, :]
        rows = W @ T  # boots x G
        mx = rows.max(1)
        # per-column stretch maxima; baseline cells' count-0 maxima go to ZU, every other
        # cell enters as an explicit entry (its maximum minus its baseline maximum)
        M = np.stack([T[:, 64 * s:64 * s + 64].max(1) for s in range(nst)], 1)  # C x nst
        base = np.where(zero[g][:, None], M, 0.0)
        ZU = W @ base
        UD = np.where(zero[g][:, None], 0.0, M)
        UB = ZU + W @ UD
        for s in range(nst):
            seg = rows[:, 64 * s:64 * s + 64]
            assert np.all(seg.max(1) <= UB[:, s] + 1e-9 * np.abs(UB[:, s]) + 1e-9), (g, s)
            ok = np.all(UB[:, s] < mx - 51.0)
            checked += 1
            if ok:
                skipped += 1
                assert np.all(seg - mx[:, None] < -50.0), (g, s)
    assert checked > 0 and skipped > 0  # the check has cases on both sides
