"""Host-side mirror of scde's weighted-PCA path (``bwpca()``, ``pagoda.pathway.wPCA()``) and
of the PAGODA helper ``.Call`` symbols (src/pagoda.cpp: ``winsorizeMatrix``, ``matWCorr``,
``matCorr``, ``plSemicompleteCor2``).

The EM iterations run in ``libscde_hip.so`` (``wpca.hip``: one workgroup per problem x
random start, the whole EM loop on chip).  This module restates the R glue around the
``.Call("baileyWPCA", ...)`` boundary (src/bwpca.cpp:59) and batches every bwpca call of
a ``pagoda.pathway.wPCA`` run -- each gene set, its ``n.randomizations`` random gene sets
and its internal shuffles -- into one device call over a resident matrix pair.

R glue restated (file:line into the reference):
  * ``bwpca``                R/functions.R:1067-1088
  * ``weighted_mat_center``  R/functions.R:5062-5072
  * ``pagoda_pathway_wPCA``  R/functions.R:1907-1975

Random inputs follow the reference's RNG use (R's RNG.c; restated natively in the library):
  * ``set.seed(seed)`` fixes .Random.seed and the in-memory state;
  * every R-level draw (``sample``) reloads .Random.seed, draws, and saves it back;
  * baileyWPCA draws ``nstarts x d x npcs`` uniforms per EM round from the in-memory state
    only (RcppArmadillo's randu -> unif_rand(); the .Call does no Get/PutRNGstate), so
    those draws are discarded by the next R-level draw;
  * internal shuffles use the platform rand(); the reference inherits the process's rand()
    state, the mirror seeds it with ``rand_seed`` (+ the gene-set index) per bwpca call.
With ``n_cores > 1`` the reference forks (mclapply) and its RNG streams depend on the
fork; this mirror always follows the n.cores = 1 (lapply) order.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import ScdeError, check, lib
from .api import Context, _p, default_context

P = ctypes.c_void_p


class RState:
    """R's Mersenne-Twister state (625 words; word 0 = mti) -- ``set.seed(seed)``."""

    def __init__(self, seed=None, words=None):
        if words is not None:
            self.w = np.array(words, dtype=np.uint32)
        else:
            self.w = np.zeros(625, np.uint32)
            check(lib().scde_r_set_seed(ctypes.c_uint32(int(seed) & 0xffffffff), _p(self.w)))

    def copy(self):
        return RState(words=self.w)

    def unif_rand(self, n):
        out = np.empty(int(n), np.float64)
        if n:
            check(lib().scde_r_unif_rand(_p(self.w), int(n), _p(out)))
        return out

    def sample(self, n, k):
        """sample.int(n, k) without replacement, 1-based (R >= 3.6)."""
        out = np.empty(int(k), np.int32)
        if k:
            check(lib().scde_r_sample(_p(self.w), int(n), int(k), _p(out)))
        return out


def shuffle_perms(rand_seed, nshuffles, d, n):
    """set_random_matrices' row permutations (src/bwpca.cpp:41-57): nshuffles x d x n."""
    out = np.zeros((max(int(nshuffles), 0), d, n), np.int32)
    if nshuffles > 0 and d > 0 and n > 0:
        check(lib().scde_shuffle_perms(int(rand_seed), int(nshuffles), int(d), int(n), _p(out)))
    return out


def baileyWPCA(Mat, Matw, Npcs, Nstarts, Smooth, EMtol, EMmaxiter, Seed, Nshuffles, rstate=None, rand_seed=1,
               starts=None, perms=None):
    """``.Call("baileyWPCA", ...)`` (src/bwpca.cpp:59-182) through ``scde_baileyWPCA``.

    ``Seed`` is accepted and unused, as in the reference (arma_rng::set_seed is a no-op
    under RcppArmadillo).  The starts come from ``rstate`` (R's in-memory RNG state,
    advanced in place; default ``set.seed(1)``) unless given explicitly."""
    m = np.asfortranarray(Mat, dtype=np.float64)
    w = np.asfortranarray(Matw, dtype=np.float64)
    if m.shape != w.shape or m.ndim != 2:
        raise ValueError("Mat and Matw must be matrices of the same dimensions")
    n, d = m.shape
    K = min(int(Npcs), d)
    ns = int(Nshuffles)
    if starts is None:
        rs = rstate if rstate is not None else RState(1)
        starts = rs.unif_rand((1 + ns) * int(Nstarts) * d * K)
    starts = np.ascontiguousarray(starts, dtype=np.float64)
    if starts.size < (1 + ns) * int(Nstarts) * d * K:
        raise ValueError("starts: too few uniforms")
    if ns > 0 and perms is None:
        perms = shuffle_perms(rand_seed, ns, d, n)
    pr = np.ascontiguousarray(perms, dtype=np.int32) if ns > 0 else np.zeros(1, np.int32)
    rot = np.zeros((d, K), order="F")
    sc = np.zeros((n, K), order="F")
    pcw = np.zeros((n, K), order="F")
    var = np.zeros(K)
    tot = np.zeros(1)
    rv = np.zeros(max(ns, 1))
    check(lib().scde_baileyWPCA(_p(m), _p(w), n, d, int(Npcs), int(Nstarts), int(Smooth), float(EMtol),
                                int(EMmaxiter), _p(starts), ns, _p(pr), _p(rot), _p(sc), _p(pcw), _p(var), _p(tot),
                                _p(rv)))
    res = {"rotation": rot, "scores": sc, "scoreweights": pcw, "var": var, "totvar": float(tot[0])}
    if ns > 0:
        res["randvar"] = rv[:ns]
    return res


def bwpca(mat, matw=None, npcs=2, nstarts=1, smooth=0, em_tol=1e-6, em_maxiter=25, seed=1, center=True,
          n_shuffles=0, rstate=None, rand_seed=1):
    """R/functions.R:1067-1088.  mat: observations (cells) x variables (genes)."""
    colnames = list(mat.columns) if hasattr(mat, "columns") else None
    rownames = list(mat.index) if hasattr(mat, "index") else None
    mat = np.array(mat, dtype=np.float64)
    if smooth < 4:
        smooth = 0
    if matw is not None and np.any(np.isnan(np.asarray(matw, dtype=np.float64))):
        raise ScdeError("bwpca: weight matrix contains NaN values")
    if np.any(np.isnan(mat)):
        raise ScdeError("bwpca: value matrix contains NaN values")
    if matw is None:
        matw = np.ones_like(mat)
        nstarts = 1
    matw = np.asarray(matw, dtype=np.float64)
    if center:
        mat = mat - (mat * matw).sum(axis=0) / matw.sum(axis=0)
    res = baileyWPCA(mat, matw, npcs, nstarts, smooth, em_tol, em_maxiter, seed, n_shuffles, rstate=rstate,
                     rand_seed=rand_seed)
    res["sd"] = np.sqrt(res["var"])[None, :]
    res["rotation_names"] = colnames
    res["scores_names"] = rownames
    return res


def weighted_mat_center(mat, matw, batch=None):
    """R/functions.R:5062-5072: per-row (gene) weighted centering, per batch level."""
    mat = np.asarray(mat, dtype=np.float64)
    matw = np.asarray(matw, dtype=np.float64)
    if batch is None:
        return mat - ((mat * matw).sum(axis=1) / matw.sum(axis=1))[:, None]
    cmat = mat.copy()
    b = np.asarray(batch)
    for lev in sorted(set(b.tolist())):
        ii = np.where(b == lev)[0]
        cmat[:, ii] = cmat[:, ii] - ((cmat[:, ii] * matw[:, ii]).sum(axis=1) / matw[:, ii].sum(axis=1))[:, None]
    return cmat


def _r_sd(x):
    x = np.asarray(x, dtype=np.float64)
    return float(np.std(x, ddof=1)) if x.size > 1 else float("nan")


def _r_cor(x, y):
    x = np.asarray(x, dtype=np.float64) - np.mean(x)
    y = np.asarray(y, dtype=np.float64) - np.mean(y)
    return float((x * y).sum() / np.sqrt((x * x).sum() * (y * y).sum()))


class DeviceMatrixPair:
    """pagoda's t(varinfo$mat) / t(varinfo$matw) resident in HBM: cells x genes column-major
    (= genes x cells row-major), column stride ncells."""

    def __init__(self, ctx: Context, mat_genes_x_cells, matw_genes_x_cells):
        m = np.ascontiguousarray(mat_genes_x_cells, dtype=np.float64)
        w = np.ascontiguousarray(matw_genes_x_cells, dtype=np.float64)
        if m.shape != w.shape or m.ndim != 2:
            raise ValueError("mat and matw must be genes x cells matrices of the same shape")
        self.ctx = ctx
        self.ngenes, self.ncells = m.shape
        self.M, self.W = P(), P()
        for ptr, a in ((self.M, m), (self.W, w)):
            check(lib().scde_dev_alloc(ctx.handle, max(1, a.nbytes), ctypes.byref(ptr)))
            if a.nbytes:
                check(lib().scde_h2d(ctx.handle, ptr, _p(a), a.nbytes))

    def free(self):
        for ptr in (self.M, self.W):
            if ptr:
                check(lib().scde_dev_free(self.ctx.handle, ptr))
        self.M, self.W = P(), P()


class WpcaBatch:
    """Problems for one ``scde_bwpca_batch_dev`` call (column subsets of a resident pair)."""

    def __init__(self):
        self.d, self.npcs, self.nstarts, self.col_off, self.perm_off, self.start_off = [], [], [], [], [], []
        self.cols, self.perms, self.starts = [], [], []
        self._nc = self._np = self._ns = 0

    def add(self, cols, npcs, nstarts, starts, perm=None):
        cols = np.asarray(cols, dtype=np.int32)
        self.d.append(len(cols))
        self.npcs.append(int(npcs))
        self.nstarts.append(int(nstarts))
        self.col_off.append(self._nc)
        self.cols.append(cols)
        self._nc += len(cols)
        if perm is None:
            self.perm_off.append(-1)
        else:
            perm = np.ascontiguousarray(perm, dtype=np.int32).ravel()
            self.perm_off.append(self._np)
            self.perms.append(perm)
            self._np += perm.size
        starts = np.asarray(starts, dtype=np.float64).ravel()
        self.start_off.append(self._ns)
        self.starts.append(starts)
        self._ns += starts.size
        return len(self.d) - 1

    def run(self, dev: DeviceMatrixPair, smooth=0, em_tol=1e-6, em_maxiter=25, want_iterations=False):
        nprob = len(self.d)
        n = dev.ncells
        K = np.minimum(np.array(self.npcs, np.int32), np.array(self.d, np.int32)) if nprob else np.zeros(0, np.int32)
        d = np.array(self.d, np.int32)
        cols = np.concatenate(self.cols) if self.cols else np.zeros(1, np.int32)
        perms = np.concatenate(self.perms) if self.perms else np.zeros(1, np.int32)
        starts = np.concatenate(self.starts) if self.starts else np.zeros(1)
        rot = np.zeros(max(int((d * K).sum()), 1))
        nk = int(K.sum())
        sco = np.zeros(max(n * nk, 1))
        pcw = np.zeros(max(n * nk, 1))
        cm = np.zeros(max(n * nk, 1))
        stats = np.zeros(max(nk + 2 * nprob, 1))
        its = np.zeros(max(int(np.sum(self.nstarts)), 1), np.int32)
        if nprob:
            i64 = lambda a: np.ascontiguousarray(a, dtype=np.int64)  # noqa: E731
            i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)  # noqa: E731
            npcs_a, ns_a, co, po, so = (i32(self.npcs), i32(self.nstarts), i64(self.col_off), i64(self.perm_off),
                                        i64(self.start_off))
            check(lib().scde_bwpca_batch_dev(dev.ctx.handle, dev.M, dev.W, n, n, dev.ngenes, nprob, _p(d),
                                             _p(npcs_a), _p(ns_a), _p(co), _p(cols), self._nc, _p(po), _p(perms),
                                             self._np, _p(so), _p(starts), self._ns, int(smooth), float(em_tol),
                                             int(em_maxiter), _p(rot), _p(sco), _p(pcw), _p(cm), _p(stats),
                                             _p(its) if want_iterations else None))
        out = []
        ro = so_ = vo = it = 0
        for p in range(nprob):
            k, dp = int(K[p]), int(d[p])
            r = {"rotation": rot[ro:ro + dp * k].reshape(k, dp).T,
                 "scores": sco[so_:so_ + n * k].reshape(k, n).T,
                 "scoreweights": pcw[so_:so_ + n * k].reshape(k, n).T,
                 "colmeans": cm[so_:so_ + n * k].reshape(k, n).T,
                 "var": stats[vo:vo + k].copy(), "totvar": float(stats[vo + k]), "npres1": float(stats[vo + k + 1])}
            if want_iterations:
                r["iterations"] = its[it:it + self.nstarts[p]].copy()
            it += self.nstarts[p]
            ro += dp * k
            so_ += n * k
            vo += k + 2
            out.append(r)
        return out


def pathway_gene_sets(gene_names, setenv, min_size=10, max_size=1000):
    """gsl (R/functions.R:1929-1934): ls(envir) -- sorted names -- kept when the number of
    unique members present is within [min, max]."""
    present = set(gene_names)
    out = []
    for go in sorted(setenv):
        ng = len({g for g in setenv[go] if g in present})
        if min_size <= ng <= max_size:
            out.append(go)
    return out


class PagodaDevice:
    """``varinfo`` prepared as pagoda.pathway.wPCA does before its gene-set loop
    (R/functions.R:1916-1927: weighted centering per batch, constant rows dropped) and
    resident in HBM as t(mat) / t(matw)."""

    def __init__(self, varinfo, ctx=None, center=True, batch_center=True, proper_gene_names=None):
        mat = np.asarray(varinfo["mat"], dtype=np.float64)
        matw = np.asarray(varinfo["matw"], dtype=np.float64)
        genes = varinfo.get("genes")
        names = list(proper_gene_names) if proper_gene_names is not None else (
            list(genes) if genes is not None else [str(i) for i in range(mat.shape[0])])
        batch = varinfo.get("batch") if batch_center else None
        if center:
            mat = weighted_mat_center(mat, matw, batch)
        vi = np.abs(np.diff(mat, axis=1)).sum(axis=1) > 0
        vi[np.isnan(vi)] = False
        if not vi.all():
            mat, matw = mat[vi], matw[vi]
        self.names = [g for g, k in zip(names, vi) if k]
        self.ngenes, self.ncells = mat.shape
        self.ctx = ctx or default_context()
        self.dev = DeviceMatrixPair(self.ctx, mat, matw)

    def free(self):
        self.dev.free()


def pagoda_pathway_wPCA(varinfo, setenv, n_components=2, n_cores=1, min_pathway_size=10, max_pathway_size=1000,
                        n_randomizations=10, n_internal_shuffles=0, n_starts=10, center=True, batch_center=True,
                        proper_gene_names=None, verbose=0, seed=1, rand_seed=1, ctx=None, em_tol=1e-6,
                        em_maxiter=25, device=None):
    """R/functions.R:1907-1975.  varinfo: {"mat": genes x cells, "matw": genes x cells,
    "batch": per-cell labels or None, "genes": row names}; setenv: {name: [gene, ...]}.
    Returns {name: {"xv", "xp", "z", "sd", "n"}} in gsl order (None for an empty set).
    Every bwpca call of the run goes to the device in one batch.  ``device``: a
    PagodaDevice prepared from varinfo earlier (reused, not freed)."""
    own = device is None
    pdev = PagodaDevice(varinfo, ctx, center, batch_center, proper_gene_names) if own else device
    try:
        return _pathway_wpca(pdev, setenv, n_components, min_pathway_size, max_pathway_size, n_randomizations,
                             n_internal_shuffles, n_starts, verbose, seed, rand_seed, em_tol, em_maxiter)
    finally:
        if own:
            pdev.free()


def _pathway_wpca(pdev, setenv, n_components, min_pathway_size, max_pathway_size, n_randomizations,
                  n_internal_shuffles, n_starts, verbose, seed, rand_seed, em_tol, em_maxiter):
    names = pdev.names
    gsl = pathway_gene_sets(names, setenv, min_pathway_size, max_pathway_size)
    if verbose:
        print(f"processing {len(gsl)} valid pathways")
    ncells, ngenes = pdev.ncells, pdev.ngenes
    pos = {}
    for i, g in enumerate(names):
        pos.setdefault(g, []).append(i)
    # walk the RNG in the reference's order, building every problem up front
    batch_ = WpcaBatch()
    saved = RState(seed)
    mem = saved.copy()
    plan = []
    for gi, go in enumerate(gsl):
        # lab <- proper.gene.names %in% get(x): columns in matrix order
        cols = np.array(sorted({i for g in set(setenv[go]) for i in pos.get(g, ())}), dtype=np.int32)
        if len(cols) < 1:
            plan.append(None)
            continue
        d = len(cols)
        K = min(int(n_components), d)
        starts = mem.unif_rand((1 + n_internal_shuffles) * n_starts * d * K)
        main = batch_.add(cols, n_components, n_starts, starts[:n_starts * d * K])
        shuf = []
        if n_internal_shuffles > 0:
            perms = shuffle_perms(rand_seed + gi, n_internal_shuffles, d, ncells)
            for s in range(n_internal_shuffles):
                o = (1 + s) * n_starts * d * K
                shuf.append(batch_.add(cols, n_components, n_starts, starts[o:o + n_starts * d * K], perms[s]))
        rnd = []
        for _ in range(n_randomizations):
            mem = saved.copy()                       # GetRNGstate()
            si = mem.sample(ngenes, d) - 1
            saved = mem.copy()                       # PutRNGstate()
            rnd.append(batch_.add(si, 1, n_starts, mem.unif_rand(n_starts * d)))
        plan.append((go, cols, main, shuf, rnd))
    res = batch_.run(pdev.dev, smooth=0, em_tol=em_tol, em_maxiter=em_maxiter)
    out = {}
    for go, pl in zip(gsl, plan):
        if pl is None:
            out[go] = None
            continue
        _, cols, main, shuf, rnd = pl
        r = res[main]
        xp = {"rotation": r["rotation"].copy(), "scores": r["scores"].copy(), "scoreweights": r["scoreweights"],
              "var": r["var"], "totvar": r["totvar"], "sd": np.sqrt(r["var"])[None, :],
              "rotation_names": [names[c] for c in cols]}
        if shuf:
            xp["randvar"] = np.array([r["totvar"] - res[q]["npres1"] for q in shuf])
        z = np.array([np.sqrt(res[q]["var"][0]) for q in rnd])[:, None] if rnd else np.zeros((0, 1))
        K = xp["scores"].shape[1]
        cs = np.array([np.sign(_r_cor(xp["scores"][:, i], r["colmeans"][:, i])) for i in range(K)])
        xp["scores"] = xp["scores"] * cs
        xp["rotation"] = xp["rotation"] * cs
        z2 = z[:, 0] ** 2
        avar = np.maximum(0.0, (xp["sd"][0] ** 2 - np.mean(z2)) / _r_sd(z2)) if len(z2) else np.full(K, np.nan)
        xv = xp["scores"].T.copy()
        sds = np.array([_r_sd(row) for row in xv])
        xv = xv / sds[:, None] * np.sqrt(avar)[:, None]
        out[go] = {"xv": xv, "xp": xp, "z": z, "sd": xp["sd"], "n": len(cols)}
    return out


# ================================================================== PAGODA helpers (src/pagoda.cpp)
def winsorizeMatrix(Mat, Trim):
    """.Call("winsorizeMatrix", Mat, Trim) (src/pagoda.cpp:6-31)."""
    m = np.asfortranarray(Mat, dtype=np.float64)
    if m.ndim != 2:
        raise ValueError("Mat must be a matrix")
    out = np.empty_like(m, order="F")
    check(lib().scde_winsorizeMatrix(_p(m), m.shape[0], m.shape[1], float(Trim), _p(out)))
    return out


def winsorize_matrix(mat, trim):
    """winsorize.matrix (R/functions.R:1109-1115): trim > 0.5 is a count of values."""
    rows = list(mat.index) if hasattr(mat, "index") else None
    cols = list(mat.columns) if hasattr(mat, "columns") else None
    m = np.asarray(mat, dtype=np.float64)
    if trim > 0.5:
        trim = trim / m.shape[1]
    wm = winsorizeMatrix(m, trim)
    if rows is not None or cols is not None:
        import pandas as pd
        return pd.DataFrame(wm, index=rows, columns=cols)
    return wm


def matWCorr(Mat, Matw):
    """.Call("matWCorr", Mat, Matw) (src/pagoda.cpp:41-65): ncol x ncol, lower triangle."""
    m = np.asfortranarray(Mat, dtype=np.float64)
    w = np.asfortranarray(Matw, dtype=np.float64)
    if m.shape != w.shape or m.ndim != 2:
        raise ValueError("Mat and Matw must be matrices of the same dimensions")
    out = np.empty((m.shape[1], m.shape[1]), order="F")
    check(lib().scde_matWCorr(_p(m), _p(w), m.shape[0], m.shape[1], _p(out)))
    return out


def matCorr(X, Y):
    """.Call("matCorr", X, Y) = arma::cor(X, Y) (src/pagoda.cpp:33-38)."""
    x = np.asfortranarray(X, dtype=np.float64)
    y = np.asarray(Y, dtype=np.float64)
    if y.ndim == 1:
        y = y[:, None]
    y = np.asfortranarray(y)
    if x.ndim != 2 or x.shape[0] != y.shape[0]:
        raise ValueError("X and Y must have the same number of rows")
    out = np.empty((x.shape[1], y.shape[1]), order="F")
    check(lib().scde_matCorr(_p(x), x.shape[0], x.shape[1], _p(y), y.shape[1], _p(out)))
    return out


def plSemicompleteCor2(pl):
    """.Call("plSemicompleteCor2", pl) (src/pagoda.cpp:67-117); pl: [(i, v), ...] with
    increasing integer gene indices i.  Returns {"r", "n"}."""
    npl = len(pl)
    off = np.zeros(npl + 1, np.int64)
    for k, (i, _) in enumerate(pl):
        off[k + 1] = off[k] + len(i)
    idx = np.ascontiguousarray(np.concatenate([np.asarray(i).astype(np.int32) for i, _ in pl]) if off[-1] else
                               np.zeros(1, np.int32))
    val = np.ascontiguousarray(np.concatenate([np.asarray(v, np.float64) for _, v in pl]) if off[-1] else
                               np.zeros(1))
    r = np.zeros((npl, npl), order="F")
    n = np.zeros((npl, npl), np.int32, order="F")
    check(lib().scde_plSemicompleteCor2(npl, _p(off), _p(idx), _p(val), _p(r), _p(n)))
    return {"r": r, "n": n}


def pagoda_varnorm_weights(models, counts, prior, batch=None, n_cores=1, n_randomizations=100,
                           use_expected_value=True, ctx=None):
    """pagoda.varnorm's posterior-mode consumer (R/functions.R:1401-1507), on the device:
    scde.posteriors over all cells (and over each batch level's cells), the modes
    ``jp %*% as.numeric(colnames(jp))`` (or the magnitude of each row's maximum with
    ``use_expected_value=False``), and the weight matrix ``matw = 1 - mfp * sfp``
    (mfp = scde.failure.probability at log(modes), sfp = ppois(count - 1, exp(fail.r),
    lower.tail = FALSE)), plus the batch version ``bmatw``.  Batch levels with fewer than
    2 cells join the largest level first (1404-1410).  Returns a dict: avmodes (genes),
    modes (levels x genes with a batch, else None), matw, bmatw (genes x cells; bmatw None
    without a batch)."""
    import ctypes
    from . import api
    from ._lib import check, lib
    from .models import model_matrix
    ctx = ctx or api.default_context()
    mat, _ = api._align_counts(models, counts)
    N, C = mat.shape
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    codes = None
    nb = 0
    if batch is not None:
        b = np.asarray(batch)
        levels = sorted(set(b.tolist()))
        counts_per = {lv: int(np.sum(b == lv)) for lv in levels}
        big = max(levels, key=lambda lv: counts_per[lv])
        b = np.array([big if counts_per[x] < 2 else x for x in b.tolist()])
        levels = sorted(set(b.tolist()))
        if len(levels) > 1:
            codes = np.ascontiguousarray([levels.index(x) for x in b.tolist()], np.int32)
            nb = len(levels)
    nm = 1 + nb if nb > 1 else 1
    modes = np.zeros(nm * N)
    matw = np.zeros((N, C), order="F")
    bmatw = np.zeros((N, C), order="F") if nb > 1 else None
    P = ctypes.c_void_p

    def p(a):
        return None if a is None else a.ctypes.data_as(P)
    check(lib().scde_pagoda_varnorm_weights_host(ctx.handle, p(mat), N, N, C, p(mm), lt, sq, p(px), len(px),
                                                 int(n_randomizations), int(n_cores), p(codes), nb,
                                                 int(bool(use_expected_value)), p(modes), p(matw), p(bmatw)))
    modes = modes.reshape(nm, N)
    return {"avmodes": modes[0].copy(), "modes": modes[1:].copy() if nm > 1 else None, "matw": matw,
            "bmatw": bmatw}
