"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the scde DE hot path.

Python side of the oracle: ctypes bindings to ``oracle/liboracle.so`` (the C
restatement in ``scde_oracle.c``) plus a restatement of the R glue on the path.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product (``scde_amd``) never
does.

R glue restated here (file:line into the reference):
  * ``scde_posteriors``            R/functions.R:566-669
      - marginals  log(pmax(10^x - 1, 0))            :575-577
      - slope clamp corr.a < 1e-10                   :579-583
      - postflag / ensemble / model-matrix ``mm``    :585-604
      - gene chunking ``split(x, sort(rank(x) %% n.cores))`` and seed ii[1] :606-617
      - ``ucl`` (first-appearance unique) / ``uci`` (match-1)               :609-610, 631-632
  * ``calculate_ratio_posterior``  R/functions.R:3491-3510
  * ``quick_distribution_summary`` R/functions.R:5039-5053 (+ Z 3514-3531)
  * ``scde_expression_difference`` R/functions.R:304-407
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SCDE_ORACLE_LIB: another build of the same sources (the sanitizer build, oracle/Makefile)
_LIB_PATH = os.environ.get("SCDE_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

MODEL_COLUMNS = ["conc.b", "conc.a", "fail.r", "corr.b", "corr.a", "corr.theta",
                 "corr.ltheta.b", "corr.ltheta.t", "corr.ltheta.m", "corr.ltheta.s",
                 "corr.ltheta.r", "conc.a2"]

_lib = None


def build():
    """Compile the C restatement (``make -C oracle``)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        d, i, P = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        L.o_stirlerr.restype = d
        L.o_stirlerr.argtypes = [d]
        L.o_bd0.restype = d
        L.o_bd0.argtypes = [d, d]
        L.o_dnbinom_log.restype = d
        L.o_dnbinom_log.argtypes = [d, d, d]
        L.o_dpois_log.restype = d
        L.o_dpois_log.argtypes = [d, d]
        L.o_qnorm.restype = d
        L.o_qnorm.argtypes = [d, i]
        L.o_pnorm.restype = d
        L.o_pnorm.argtypes = [d, i]
        L.o_rand_stream.argtypes = [ctypes.c_uint, i, P]
        L.o_draw_stream.argtypes = [ctypes.c_uint, i, i, P]
        L.o_logBootPosterior.argtypes = [P, i, P, P, P, i, P, i, i, i, i, i, i, i, P, P, P]
        L.o_logBootBatchPosterior.argtypes = [P, i, P, P, P, i, P, i, P, P, P, i, i, i, i, i, i, P, P, P]
        L.o_jpmatLogBoot.argtypes = [P, i, i, i, i, i, P]
        L.o_jpmatLogBatchBoot.argtypes = [P, P, P, i, i, i, i, i, P]
        L.o_matSlideMult.argtypes = [P, P, i, i, P]
        L.o_ratio_posterior.argtypes = [P, P, P, i, i, P]
        L.o_summary.argtypes = [P, i, i, P, d, P]
        L.o_bh_cz.argtypes = [P, i, P]
        L.o_set_rng_kind.argtypes = [i]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f64(a):
    return np.require(a, dtype=np.float64, requirements=["F", "A"])


def _i32(a):
    return np.require(a, dtype=np.int32, requirements=["F", "A"])


# ---------------------------------------------------------------- scalars
def set_rng(kind):
    """0 = glibc TYPE_3 (Linux), 2 = Darwin/BSD Park-Miller (macOS; the vignette's platform)."""
    lib().o_set_rng_kind(int(kind))


def rand_stream(seed, n):
    out = np.zeros(n, np.int32)
    lib().o_rand_stream(seed, n, _p(out))
    return out


def draw_stream(seed, n, count):
    out = np.zeros(count, np.int32)
    lib().o_draw_stream(seed, n, count, _p(out))
    return out


def dnbinom_log(x, size, prob):
    return lib().o_dnbinom_log(float(x), float(size), float(prob))


def dpois_log(x, lam):
    return lib().o_dpois_log(float(x), float(lam))


def qnorm(p, lower_tail=True):
    return lib().o_qnorm(float(p), int(bool(lower_tail)))


def pnorm(x, lower_tail=True):
    return lib().o_pnorm(float(x), int(bool(lower_tail)))


# ---------------------------------------------------------------- .Call restatements
def _flatten_list(lst):
    vals = np.ascontiguousarray(np.concatenate([np.asarray(v, np.int32) for v in lst]) if lst else np.zeros(0, np.int32), np.int32)
    off = np.zeros(len(lst) + 1, np.int64)
    off[1:] = np.cumsum([len(v) for v in lst])
    return vals, off


def logBootPosterior(models, ucl, uci, magnitudes, nboot, seed, returnpost=0, localtheta=0,
                     squarelogit=0, ensemble=0):
    """Restates src/jpmatLogBoot.cpp:100-331; mirrors its return shapes."""
    mm = _f64(models)
    C = mm.shape[0]
    uci = _i32(uci)
    N = uci.shape[0]
    mag = _f64(magnitudes)
    G = mag.shape[0]
    vals, off = _flatten_list(ucl)
    jp = np.zeros((N, G), order="F")
    modes = np.zeros((N, C), order="F") if returnpost in (1, 3) else None
    post_buf = np.zeros(C * N * G) if returnpost in (2, 3) else None
    lib().o_logBootPosterior(_p(mm), C, _p(vals), _p(off), _p(uci), N, _p(mag), G, int(nboot), int(seed),
                             int(returnpost), int(localtheta), int(squarelogit), int(ensemble), _p(jp),
                             _p(modes) if modes is not None else None,
                             _p(post_buf) if post_buf is not None else None)
    return _pack(jp, modes, post_buf, returnpost, C, N, G)


def _pack(jp, modes, post_buf, returnpost, C, N, G):
    if returnpost == 0:
        return jp
    out = {"jp": jp}
    if modes is not None:
        out["modes"] = modes
    if post_buf is not None:
        out["post"] = [post_buf[i * N * G:(i + 1) * N * G].reshape((N, G), order="F") for i in range(C)]
    return out


def logBootBatchPosterior(models, ucl, uci, magnitudes, batchil, composition, nboot, seed, returnpost=0,
                          localtheta=0, squarelogit=0):
    """Restates src/jpmatLogBoot.cpp:343-531."""
    mm = _f64(models)
    C = mm.shape[0]
    uci = _i32(uci)
    N = uci.shape[0]
    mag = _f64(magnitudes)
    G = mag.shape[0]
    vals, off = _flatten_list(ucl)
    bvals, boff = _flatten_list(batchil)
    comp = np.ascontiguousarray(composition, np.int32)
    jp = np.zeros((N, G), order="F")
    rp = returnpost if returnpost in (1, 2) else 0
    modes = np.zeros((N, C), order="F") if rp == 1 else None
    post_buf = np.zeros(C * N * G) if rp == 2 else None
    lib().o_logBootBatchPosterior(_p(mm), C, _p(vals), _p(off), _p(uci), N, _p(mag), G, _p(bvals), _p(boff),
                                  _p(comp), len(comp), int(nboot), int(seed), int(returnpost), int(localtheta),
                                  int(squarelogit), _p(jp), _p(modes) if modes is not None else None,
                                  _p(post_buf) if post_buf is not None else None)
    return _pack(jp, modes, post_buf, rp, C, N, G)


def jpmatLogBoot(matl, nboot, seed):
    mats = [_f64(m) for m in matl]
    nr, nc = mats[0].shape
    ptrs = (ctypes.c_void_p * len(mats))(*[m.ctypes.data for m in mats])
    out = np.zeros((nr, nc), order="F")
    lib().o_jpmatLogBoot(ptrs, len(mats), nr, nc, int(nboot), int(seed), _p(out))
    return out


def jpmatLogBatchBoot(matll, comp, nboot, seed):
    mats = [_f64(m) for lst in matll for m in lst]
    toff = np.zeros(len(matll) + 1, np.int32)
    toff[1:] = np.cumsum([len(lst) for lst in matll])
    nr, nc = mats[0].shape
    ptrs = (ctypes.c_void_p * len(mats))(*[m.ctypes.data for m in mats])
    comp = np.ascontiguousarray(comp, np.int32)
    out = np.zeros((nr, nc), order="F")
    lib().o_jpmatLogBatchBoot(ptrs, _p(toff), _p(comp), len(matll), nr, nc, int(nboot), int(seed), _p(out))
    return out


def matSlideMult(m1, m2):
    a, b = _f64(m1), _f64(m2)
    nr, n = a.shape
    out = np.zeros((nr, 2 * n - 1), order="F")
    lib().o_matSlideMult(_p(a), _p(b), nr, n, _p(out))
    return out


# ---------------------------------------------------------------- R glue
def marginals_from_prior_x(x):
    """R/functions.R:575-577.  R's `^` is libm pow() (R_pow), so use math.pow, not numpy."""
    m = np.array([math.pow(10.0, v) for v in np.asarray(x, np.float64)]) - 1
    m[m < 0] = 0
    with np.errstate(divide="ignore"):
        return np.log(m)


def model_matrix(models):
    """R/functions.R:579-604.  `models`: dict name -> per-cell vector."""
    C = len(next(iter(models.values())))
    mm = np.full((C, 12), np.nan, order="F")
    for j, nm in enumerate(MODEL_COLUMNS):
        if nm in models:
            mm[:, j] = np.asarray(models[nm], np.float64)
    ca = mm[:, 4]
    ca[ca < 1e-10] = 1e-10
    return mm, int("corr.ltheta.b" in models), int("conc.a2" in models)


def r_chunks(N, n):
    """split(seq_len(N), sort(rank(x) %% n)) -> list of 0-based index arrays (R/functions.R:606)."""
    labels = np.sort((np.arange(1, N + 1)) % n)
    return [np.nonzero(labels == k)[0] for k in range(n) if np.any(labels == k)]


def ucl_uci(counts_sub):
    """unique() in first-appearance order and match()-1, per cell (R/functions.R:609-610)."""
    N, C = counts_sub.shape
    ucl = []
    uci = np.zeros((N, C), np.int32, order="F")
    for i in range(C):
        col = counts_sub[:, i]
        u, first, inv = np.unique(col, return_index=True, return_inverse=True)
        order = np.argsort(first, kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        ucl.append(u[order].astype(np.int32))
        uci[:, i] = rank[inv.reshape(-1)]
    return ucl, uci


def scde_posteriors(models, counts, prior_x, n_randomizations=100, batch=None, composition=None,
                    return_individual_posteriors=False, return_individual_posterior_modes=False,
                    ensemble_posterior=False, n_cores=20, gene_offset=0, ngenes_total=None):
    """Restates scde.posteriors (R/functions.R:566-669).  counts: N x C int, columns = model rows.

    gene_offset / ngenes_total (test harness for sharding): ``counts`` holds rows
    [gene_offset, gene_offset + N) of an ngenes_total-gene call; chunks and seeds are those of
    the whole call (R/functions.R:606-617), restricted to this row range."""
    counts = np.asarray(counts)
    N, C = counts.shape
    NT = N if ngenes_total is None else int(ngenes_total)
    marg = marginals_from_prior_x(prior_x)
    mm, lt, sq = model_matrix(models)
    postflag = 0
    if return_individual_posteriors:
        postflag = 3 if return_individual_posterior_modes else 2
    elif return_individual_posterior_modes:
        postflag = 1
    ens = 1 if ensemble_posterior else 0
    if batch is not None:
        # None is an NA batch label: tapply (R/functions.R:570) leaves such cells out of BatchIL
        levels = sorted(set(b for b in batch if b is not None))
        batchil = [np.array([i for i in range(C) if batch[i] == lv], np.int32) for lv in levels]

    def call(ii, seed):
        ucl, uci = ucl_uci(counts[ii, :])
        if batch is not None:
            return logBootBatchPosterior(mm, ucl, uci, marg, batchil, composition, n_randomizations, seed,
                                         postflag, lt, sq)
        return logBootPosterior(mm, ucl, uci, marg, n_randomizations, seed, postflag, lt, sq, ens)

    if n_cores > 1 and NT > n_cores:
        parts = []
        for ii in r_chunks(NT, n_cores):
            loc = ii[(ii >= gene_offset) & (ii < gene_offset + N)] - gene_offset
            if len(loc):
                parts.append(call(loc, int(ii[0]) + 1))
        if postflag == 0:
            return np.vstack(parts)
        out = {"jp": np.vstack([p["jp"] for p in parts])}
        if "modes" in parts[0]:
            out["modes"] = np.vstack([p["modes"] for p in parts])
        if "post" in parts[0]:
            out["post"] = [np.vstack([p["post"][i] for p in parts]) for i in range(C)]
        return out
    return call(np.arange(N), 1)


def r_seq(frm, to, n):
    """seq(from, to, length.out = n) (R >= 3.x seq.default)."""
    by = (to - frm) / (n - 1)
    out = frm + np.arange(n, dtype=np.float64) * by
    out[0] = frm
    out[-1] = to
    return out


def r_as_character_roundtrip(v):
    """as.numeric(as.character(v)): R formats doubles with 15 significant digits."""
    return np.array([float("%.15g" % x) for x in v])


def ratio_grid(prior_x):
    x = np.asarray(prior_x, np.float64)
    n = len(x)
    rv = r_seq(x[0] - x[-1], x[-1] - x[0], 2 * n - 1)
    return r_as_character_roundtrip(rv)


def calculate_ratio_posterior(pmat1, pmat2, prior_y, skip_prior_adjustment=False):
    a, b = _f64(pmat1), _f64(pmat2)
    nr, n = a.shape
    out = np.zeros((nr, 2 * n - 1), order="F")
    y = None if skip_prior_adjustment else np.ascontiguousarray(prior_y, np.float64)
    lib().o_ratio_posterior(_p(a), _p(b), _p(y) if y is not None else None, nr, n, _p(out))
    return out


def quick_distribution_summary(rpost, diffv, expectation=0.0):
    r = _f64(rpost)
    nr, m = r.shape
    dv = np.ascontiguousarray(diffv, np.float64)
    out = np.zeros((nr, 5), order="F")
    lib().o_summary(_p(r), nr, m, _p(dv), float(expectation), _p(out))
    z = np.ascontiguousarray(out[:, 4])
    cz = np.zeros(nr)
    lib().o_bh_cz(_p(z), nr, _p(cz))
    return {"lb": out[:, 0].copy(), "mle": out[:, 1].copy(), "ub": out[:, 2].copy(),
            "ce": out[:, 3].copy(), "Z": z, "cZ": cz}


def scde_expression_difference(models, counts, prior_x, prior_y, groups, n_randomizations=150, n_cores=10,
                               return_posteriors=False, expectation=0.0, gene_offset=0, ngenes_total=None):
    """Restates scde.expression.difference (R/functions.R:304-407), no batch.

    groups: per-cell labels in {0, 1} (level order) or -1 for NA."""
    groups = np.asarray(groups)
    jpl = []
    for lv in (0, 1):
        ii = np.nonzero(groups == lv)[0]
        sub = {k: np.asarray(v)[ii] for k, v in models.items()}
        jpl.append(scde_posteriors(sub, np.asarray(counts)[:, ii], prior_x, n_randomizations=n_randomizations,
                                   n_cores=n_cores, gene_offset=gene_offset, ngenes_total=ngenes_total))
    bdiffp = calculate_ratio_posterior(jpl[0], jpl[1], prior_y)
    res = quick_distribution_summary(bdiffp, ratio_grid(prior_x), expectation)
    if return_posteriors:
        return {"results": res, "difference.posterior": bdiffp, "joint.posteriors": jpl}
    return res


def scde_expression_difference_batch(models, counts, prior_x, prior_y, groups, batch, batch_models=None,
                                     n_randomizations=150, n_cores=10, expectation=0.0, return_posteriors=False,
                                     gene_offset=0, ngenes_total=None):
    """Restates the batch-corrected branch of scde.expression.difference (R/functions.R:321-399):
    batch posteriors over all cells with each group's batch composition (table(batch[ii])),
    their ratio posterior and summary (batch.effect); the group posteriors, ratio and summary
    (results); the second-level ratio of the two 801-column posteriors with skip.prior.adjustment
    and its summary over the 1601 columns (batch.adjusted)."""
    groups = np.asarray(groups)
    batch = list(batch)
    levels = sorted(set(b for b in batch if b is not None))  # None: NA (no level; table() drops it)
    bm = models if batch_models is None else batch_models
    cnt = np.asarray(counts)
    diffv = ratio_grid(prior_x)
    bjp = []
    for lv in (0, 1):
        ii = np.nonzero(groups == lv)[0]
        comp = [int(sum(1 for i in ii if batch[i] == b)) for b in levels]
        bjp.append(scde_posteriors(bm, cnt, prior_x, n_randomizations=n_randomizations, batch=batch, composition=comp,
                                   n_cores=n_cores, gene_offset=gene_offset, ngenes_total=ngenes_total))
    batch_bdiffp = calculate_ratio_posterior(bjp[0], bjp[1], prior_y)
    batch_rep = quick_distribution_summary(batch_bdiffp, diffv, 0.0)
    jpl = []
    for lv in (0, 1):
        ii = np.nonzero(groups == lv)[0]
        sub = {k: np.asarray(v)[ii] for k, v in models.items()}
        jpl.append(scde_posteriors(sub, cnt[:, ii], prior_x, n_randomizations=n_randomizations, n_cores=n_cores,
                                   gene_offset=gene_offset, ngenes_total=ngenes_total))
    bdiffp = calculate_ratio_posterior(jpl[0], jpl[1], prior_y)
    rep = quick_distribution_summary(bdiffp, diffv, expectation)
    a_bdiffp = calculate_ratio_posterior(bdiffp, batch_bdiffp, None, skip_prior_adjustment=True)
    a_rep = quick_distribution_summary(a_bdiffp, ratio_grid(diffv), expectation)
    out = {"batch.adjusted": a_rep, "results": rep, "batch.effect": batch_rep}
    if return_posteriors:
        out.update({"difference.posterior": bdiffp, "batch.adjusted.difference.posterior": a_bdiffp,
                    "joint.posteriors": jpl, "batch.difference.posterior": batch_bdiffp})
    return out
