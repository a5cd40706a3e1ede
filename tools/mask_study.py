"""Offline study of the bootstrap's grid-stretch masks (CPU; oracle tables).

For genes of a bench configuration, one boot slab of uniform draws: how many 64-point
stretches (and 16-point tiles) per slab hold a softmax term above the e^-50 cut (truth),
and how many each mask rule keeps:
  heuristic  UB_bs >= max_s' UB_bs' - 50 - slack (the current k_stretch_mask rule)
  ub-exact   UB_bs >= m_b - 51 with the exact row maxima (the best any UB-based rigorous rule can do)
  ub-probe   UB_bs >= LB_b - 51, LB_b = row_b at the mean row's argmax (rigorous, one probe point)

  python tools/mask_study.py [config] [genes] [nb]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402


def tables(mm, lt, sq, counts, mag):
    ucl, uci = O.ucl_uci(counts)
    vals, off = O._flatten_list(ucl)
    C = mm.shape[0]
    G = len(mag)
    tab = np.zeros(int(off[-1]) * G)
    O.lib().o_tables.argtypes = None
    O.lib().o_tables(O._p(mm), C, O._p(vals), O._p(off), O._p(mag), G, lt, sq, 0, O._p(tab), None)
    return tab.reshape(-1, G), off, uci


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "3"
    ngenes = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    cfg = bench.CONFIGS[cfgname]
    de = cfg["kind"] == "de"
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=de)
    cells = np.nonzero(np.asarray(groups) == groups[0])[0] if de else np.arange(counts.shape[1])
    sub = {k: np.asarray(v)[cells] for k, v in models.items()}
    mm, lt, sq = O.model_matrix(sub)
    from oracle.prior import expression_prior
    x = np.asarray(expression_prior(models, counts[:4000], length_out=400)["x"])  # the bench's grid (gene sample)
    mag = O.marginals_from_prior_x(x)
    cnt = np.ascontiguousarray(counts[:ngenes][:, cells])
    tab, off, uci = tables(mm, lt, sq, cnt, mag)
    C = len(cells)
    G = len(mag)
    rng = np.random.default_rng(1)
    W = np.zeros((nb, C))
    for b in range(nb):
        np.add.at(W[b], rng.integers(0, C, C), 1.0)
    slack = 30 + 0.4 * C
    res = {k: [] for k in ("truth64", "heur64", "ubex64", "probe64", "truth16", "heur16", "ubex16", "probe16", "truth8",
                           "ubex8")}
    for g in range(ngenes):
        X = tab[off[:-1] + uci[g]]  # C x G
        X = np.where(np.isfinite(X), X, -1e300)
        rows = W @ X
        m = rows.max(1)
        mean = X.sum(0)
        kstar = int(np.argmax(mean))
        lb = rows[:, kstar]
        for L, tag in ((64, "64"), (16, "16"), (8, "8")):
            ns = (G + L - 1) // L
            Xp = np.full((C, ns * L), -np.inf)
            Xp[:, :G] = X
            U = Xp.reshape(C, ns, L).max(2)
            UB = W @ U
            rp = np.full((nb, ns * L), -np.inf)
            rp[:, :G] = rows
            truth = (rp.reshape(nb, ns, L) >= (m - 50)[:, None, None]).any(2).any(0)
            heur = (UB >= (UB.max(1) - 50 - slack)[:, None]).any(0)
            ubex = (UB >= (m - 51)[:, None]).any(0)
            probe = (UB >= (lb - 51)[:, None]).any(0)
            if tag in ("16", "8"):
                # tile groups of 4 (one wave): the top-4 tiles by max UB, then the tiles
                # still needed against the exact maxima of what is computed
                mub = np.where(np.isfinite(UB), UB, -np.inf).max(0)
                order = np.argsort(-mub, kind="stable")
                need = (UB >= (m - 51)[:, None]).any(0)
                done = np.zeros(ns, bool)
                gs = 64 // L
                done[order[:gs]] = True
                extra = need & ~done
                res.setdefault("groups" + tag, []).append(1 + int(np.ceil(extra.sum() / gs)))
            res["truth" + tag].append(truth.sum())
            res.setdefault("heur" + tag, []).append(heur.sum())
            res["ubex" + tag].append(ubex.sum())
            res.setdefault("probe" + tag, []).append(probe.sum())
    for k, v in res.items():
        print(f"{k:8s} mean kept {np.mean(v):6.2f}  max {np.max(v)}")
    for tag in ("16", "8"):
        gr = np.bincount(res["groups" + tag])
        print(f"{tag}-point tile groups per slab:", {i: int(c) for i, c in enumerate(gr) if c})


if __name__ == "__main__":
    main()
