"""Generate tests/golden/config3_full.npz: the oracle's scde.expression.difference table for the
WHOLE BASELINE config-3 data set (run in the dev container; ~1 min on 8 cores).

Data: bench.synthetic(2003, 20000, 1000) -- the bench's own counts (500/500 cells), regenerated
bit for bit from the PCG64 seed by the test.  Prior: oracle/prior.py (numpy restatement of
scde.expression.prior, length.out 400) over all genes; stored in the fixture so the GPU test
feeds the device the identical grid.  n.randomizations = 100, n.cores = 16 (R/functions.R:606-617:
sixteen contiguous gene chunks of 1,250, seeds 1, 1251, ...), glibc rand().

The oracle runs the chunks in worker processes, as mclapply forks them; each worker returns its
genes' lb/mle/ub/ce/Z (R/functions.R:5039-5050).  cZ is the BH adjustment over ALL 20,000 genes
(R/functions.R:5051; oracle o_bh_cz), computed here once the chunks are joined -- the quantity
the 64-gene slice tests cannot check.

Usage:  python tools/make_config3_fixture.py [--workers 8]
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NCORES = 16
NBOOT = 100
OUT = os.path.join(ROOT, "tests", "golden", "config3_full.npz")


def _chunk(job):
    models, sub, groups, px, py, lo, ntot = job
    from oracle import oracle as O
    O.set_rng(0)
    r = O.scde_expression_difference(models, np.ascontiguousarray(sub), px, py, groups, n_randomizations=NBOOT,
                                     n_cores=NCORES, gene_offset=lo, ngenes_total=ntot)
    return lo, np.column_stack([r["lb"], r["mle"], r["ub"], r["ce"], r["Z"]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    args = ap.parse_args()
    import bench
    from oracle import oracle as O
    from oracle.prior import expression_prior
    cfg = bench.CONFIGS["3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    N = counts.shape[0]
    t0 = time.time()
    prior = expression_prior(models, counts, bench.LENGTH_OUT)
    px, py = np.asarray(prior["x"], np.float64), np.asarray(prior["y"], np.float64)
    chunks = O.r_chunks(N, NCORES)
    jobs = [(models, counts[c[0]:c[-1] + 1], groups, px, py, int(c[0]), N) for c in chunks]
    with mp.get_context("spawn").Pool(args.workers) as pool:
        parts = pool.map(_chunk, jobs)
    res = np.zeros((N, 6))
    for lo, tab in parts:
        res[lo:lo + len(tab), :5] = tab
    z = np.ascontiguousarray(res[:, 4])
    cz = np.zeros(N)
    O.lib().o_bh_cz(O._p(z), N, O._p(cz))
    res[:, 5] = cz
    np.savez_compressed(OUT, prior_x=px, prior_y=py, results=res,
                        meta=np.array([cfg["seed"], cfg["genes"], cfg["cells"], NBOOT, NCORES], np.int64))
    print(f"wrote {OUT}: {N} genes in {time.time() - t0:.1f}s; {np.count_nonzero(res[:, 3])} genes with ce != 0")


if __name__ == "__main__":
    main()
