"""Generate the committed golden fixtures under tests/golden/ (run in the dev container).

Inputs come from the reference's own datasets (parsed with tools/rdata.py, which
executes nothing from the files):
  * es.mef.small + o.ifm  -- the vignette setup (vignettes/diffexp.md:21-99):
      clean.counts(min.lib.size=1000, min.reads=1, min.detected=1), prior with
      length.out=400 and max.quantile=0.999 (the grid step recovered from the
      printed table: 9.984631/251 = max.value/400/log10(2)), groups ESC/MEF.
  * knn (64 cells, local-theta + conc.a2 models) with pollen counts (data/pollen.rda).
Expected outputs come from the CPU oracle (oracle/), itself pinned against the
vignette's printed known-answer table (tests/test_oracle.py).

Usage:  python tools/make_fixtures.py [--skip-vignette]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import rdata  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.prior import expression_prior  # noqa: E402

REF = "/root/reference/data"
GOLD = os.path.join(ROOT, "tests", "golden")


def load_df(name):
    obj = rdata.read_rda(os.path.join(REF, f"{name}.rda"))[name]
    return rdata.data_frame(obj)


def esmef_vignette():
    names, genes, cols = load_df("es.mef.small")
    X = np.stack([cols[n] for n in names], 1).astype(np.int64)
    # clean.counts(counts, min.lib.size=1000, min.reads=1, min.detected=1)  R/functions.R:127-135
    keep_c = (X > 0).sum(0) > 1000
    X = X[:, keep_c]
    cnames = [n for n, k in zip(names, keep_c) if k]
    keep_g = X.sum(1) > 1
    X, genes = X[keep_g], [g for g, k in zip(genes, keep_g) if k]
    keep_g = (X > 0).sum(1) > 1
    X, genes = X[keep_g], [g for g, k in zip(genes, keep_g) if k]
    mnames, mrows, mcols = load_df("o.ifm")
    pos = {c: i for i, c in enumerate(cnames)}
    X = X[:, [pos[r] for r in mrows]]
    models = {k: np.asarray(v, np.float64) for k, v in mcols.items()}
    groups = np.array([0 if r.startswith("ESC") else 1 for r in mrows], np.int32)
    return X.astype(np.int32), genes, list(mrows), models, groups


def knn_pollen():
    obj = rdata.read_rda(os.path.join(REF, "pollen.rda"))["pollen"]
    dims = obj.attrs["dim"].value
    dn = obj.attrs["dimnames"].value
    X = np.asarray(obj.value).reshape(tuple(dims), order="F")
    genes = list(dn[0].value)
    cells = list(dn[1].value)
    mnames, mrows, mcols = load_df("knn")
    pos = {c: i for i, c in enumerate(cells)}
    X = X[:, [pos[r] for r in mrows]]
    models = {k: np.asarray(v, np.float64) for k, v in mcols.items()}
    return X.astype(np.int32), genes, list(mrows), models


def save(name, **arrs):
    os.makedirs(GOLD, exist_ok=True)
    path = os.path.join(GOLD, name)
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


def model_array(models):
    return np.stack([models.get(c, np.full(len(next(iter(models.values()))), np.nan)) for c in O.MODEL_COLUMNS], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-vignette", action="store_true")
    args = ap.parse_args()

    X, genes, cells, models, groups = esmef_vignette()
    print("es.mef.small cleaned", X.shape)
    prior = expression_prior(models, X, length_out=400, max_quantile=0.999)
    print("max.value", prior["max.value"])

    # -- small inputs fixture (first 500 genes, config 1) with oracle outputs at B=50
    sub = X[:500]
    t0 = time.time()
    res = O.scde_expression_difference(models, sub, prior["x"], prior["y"], groups, n_randomizations=50, n_cores=1,
                                       return_posteriors=True)
    print("oracle 500 genes B=50: %.1fs" % (time.time() - t0))
    r = res["results"]
    save("esmef500.npz", counts=sub, genes=np.array(genes[:500]), cells=np.array(cells),
         models=model_array(models), groups=groups, prior_x=prior["x"], prior_y=prior["y"],
         jp1=res["joint.posteriors"][0], jp2=res["joint.posteriors"][1], ratio=res["difference.posterior"],
         lb=r["lb"], mle=r["mle"], ub=r["ub"], ce=r["ce"], Z=r["Z"], cZ=r["cZ"], nboot=50)

    # -- knn / pollen: local theta + squared logit models, 300 genes, with modes
    Xp, pgenes, pcells, pmodels = knn_pollen()
    print("pollen", Xp.shape)
    keep = np.nonzero((Xp > 0).sum(1) > 5)[0][:300]
    sp = Xp[keep]
    pprior = expression_prior(pmodels, sp, length_out=400)
    t0 = time.time()
    out = O.scde_posteriors(pmodels, sp, pprior["x"], n_randomizations=20, return_individual_posterior_modes=True,
                            n_cores=1)
    print("oracle knn 300 genes B=20: %.1fs" % (time.time() - t0))
    save("knn300.npz", counts=sp, genes=np.array([pgenes[i] for i in keep]), cells=np.array(pcells),
         models=model_array(pmodels), prior_x=pprior["x"], prior_y=pprior["y"], jp=out["jp"], modes=out["modes"],
         nboot=20)

    if not args.skip_vignette:
        # -- the vignette run: all genes, n.randomizations = 100, n.cores = 1, with the
        #    Darwin rand() that produced the printed table (vignettes/diffexp.md:113-119)
        for kind, fname in ((2, "esmef_vignette_darwin.npz"), (0, "esmef_vignette_glibc.npz")):
            O.set_rng(kind)
            t0 = time.time()
            r = O.scde_expression_difference(models, X, prior["x"], prior["y"], groups, n_randomizations=100,
                                             n_cores=1)
            print("oracle vignette full run (rng %d): %.1fs" % (kind, time.time() - t0))
            save(fname, genes=np.array(genes), prior_x=prior["x"], prior_y=prior["y"], lb=r["lb"], mle=r["mle"],
                 ub=r["ub"], ce=r["ce"], Z=r["Z"], cZ=r["cZ"])
            order = np.argsort(-r["Z"], kind="stable")[:6]
            for i in order:
                print("%-14s %9.6f %9.6f %9.6f %9.6f %9.6f %9.6f" % (genes[i], r["lb"][i], r["mle"][i], r["ub"][i],
                                                                     r["ce"][i], r["Z"][i], r["cZ"][i]))
        O.set_rng(0)
        save("esmef_vignette_inputs.npz", counts=X, genes=np.array(genes), cells=np.array(cells),
             models=model_array(models), groups=groups, prior_x=prior["x"], prior_y=prior["y"])


if __name__ == "__main__":
    main()
