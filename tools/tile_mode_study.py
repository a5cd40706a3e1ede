"""Offline study for k_boot_tiles' pass width (CPU; oracle tables).

For genes of a bench configuration and boot slabs of uniform draws, with 32-point bound tiles:
  need    the bound tiles the exact post-check keeps: UB_bt >= m_b - 51 for some boot (m_b the
          exact row maximum) -- the fewest any UB-based rigorous rule can compute;
  pred(S) the heuristic set UB_bt >= max_t' UB_bt' - 51 - S for some boot (no row computed);
and, per S, how often a 2-tile pass chosen by pred(S) <= 2 would be right (need <= 2 and inside
the chosen pair) or wrong (the slab must be redone wider), against slabs pred sends wide.

  python tools/tile_mode_study.py [config] [genes] [slabs]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
from mask_study import tables  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "3"
    ngenes = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    nslab = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    nb, L = 20, 32
    cfg = bench.CONFIGS[cfgname]
    de = cfg["kind"] == "de"
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=de)
    cells = np.nonzero(np.asarray(groups) == groups[0])[0] if de else np.arange(counts.shape[1])
    sub = {k: np.asarray(v)[cells] for k, v in models.items()}
    mm, lt, sq = O.model_matrix(sub)
    from oracle.prior import expression_prior
    x = np.asarray(expression_prior(models, counts[:4000], length_out=400)["x"])
    mag = O.marginals_from_prior_x(x)
    cnt = np.ascontiguousarray(counts[:ngenes][:, cells])
    tab, off, uci = tables(mm, lt, sq, cnt, mag)
    C, G = len(cells), len(mag)
    ns = (G + L - 1) // L
    rng = np.random.default_rng(1)
    Ws = []
    for _ in range(nslab):
        W = np.zeros((nb, C))
        for b in range(nb):
            np.add.at(W[b], rng.integers(0, C, C), 1.0)
        Ws.append(W)
    Ss = [0, 10, 20, 30, 50, 80, 120, 200]
    needs = []
    preds = {S: [] for S in Ss}
    ok2 = {S: [] for S in Ss}
    for g in range(ngenes):
        X = tab[off[:-1] + uci[g]]
        X = np.where(np.isfinite(X), X, -1e300)
        Xp = np.full((C, ns * L), -np.inf)
        Xp[:, :G] = X
        U = np.ceil(Xp.reshape(C, ns, L).max(2) * 256) / 256  # the tables' rounding up
        for W in Ws:
            rows = W @ X
            m = rows.max(1)
            UB = W @ U
            need = (UB >= (m - 51)[:, None]).any(0)
            needs.append(int(need.sum()))
            mub = UB.max(1)
            for S in Ss:
                pr = (UB >= (mub - 51 - S)[:, None]).any(0)
                preds[S].append(int(pr.sum()))
                # a 2-tile pass on the two best-scored tiles when pred says <= 2
                score = UB.max(0)
                top2 = np.zeros(ns, bool)
                top2[np.argsort(-score, kind="stable")[:2]] = True
                ok2[S].append((pr.sum() <= 2, bool(np.all(top2 | ~need))))
    needs = np.array(needs)
    print(f"config {cfgname}: {len(needs)} slabs; exact need (bound tiles):",
          {i: int(c) for i, c in enumerate(np.bincount(needs)) if c})
    for S in Ss:
        p = np.array(preds[S])
        o = np.array(ok2[S])
        narrow = o[:, 0]
        right = narrow & o[:, 1]
        wrong = narrow & ~o[:, 1]
        # cost units: 2-tile pass 1, 4-tile pass 2 (a wrong narrow pass pays both)
        cost = np.where(narrow, np.where(o[:, 1], 1.0, 3.0), 2.0).mean()
        print(f"S={S:4d}: pred mean {p.mean():5.2f}; narrow {narrow.mean():.3f} (right {right.mean():.3f}, "
              f"wrong {wrong.mean():.3f}); cost {cost:.3f} (4-tile only: 2.000)")
    print("narrow pass right whenever need <= 2 and in the top two:",
          np.mean([a[1] for a in ok2[Ss[0]]]))


if __name__ == "__main__":
    main()
