"""TEST INFRASTRUCTURE ONLY -- CPU oracle for scde's PAGODA helper kernels
(src/pagoda.cpp: winsorizeMatrix, matCorr, matWCorr, plSemicompleteCor2), as ctypes
bindings to ``oracle/pagoda_oracle.c``.  Only ``tests/`` import this module.

R glue restated: ``winsorize_matrix`` (R/functions.R:1109-1115: trim > 0.5 means a
count, divided by ncol); ``varnorm_weights`` (pagoda.varnorm's posterior-mode consumer,
R/functions.R:1414-1507) on the C restatement's joint posteriors, with R's ppois upper tail
restated as scipy's Poisson survival function (both the regularised incomplete gamma).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import oracle as _o

_bound = False


def lib():
    global _bound
    L = _o.lib()
    if not _bound:
        P, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        L.o_winsorizeMatrix.argtypes = [P, i, i, d, P]
        L.o_matWCorr.argtypes = [P, P, i, i, P]
        L.o_matCorr.argtypes = [P, i, i, P, i, P]
        L.o_plSemicompleteCor2.argtypes = [i, P, P, P, P, P]
        _bound = True
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def winsorizeMatrix(mat, trim):
    m = np.asfortranarray(mat, dtype=np.float64)
    out = np.empty_like(m, order="F")
    if m.size:
        lib().o_winsorizeMatrix(_p(m), m.shape[0], m.shape[1], float(trim), _p(out))
    return out


def winsorize_matrix(mat, trim):
    if trim > 0.5:
        trim = trim / np.asarray(mat).shape[1]
    return winsorizeMatrix(mat, trim)


def matWCorr(mat, matw):
    m = np.asfortranarray(mat, dtype=np.float64)
    w = np.asfortranarray(matw, dtype=np.float64)
    k, n = m.shape
    out = np.empty((n, n), order="F")
    lib().o_matWCorr(_p(m), _p(w), k, n, _p(out))
    return out


def matCorr(x, y):
    x = np.asfortranarray(x, dtype=np.float64)
    y = np.asfortranarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y[:, None].copy(order="F")
    out = np.empty((x.shape[1], y.shape[1]), order="F")
    lib().o_matCorr(_p(x), x.shape[0], x.shape[1], _p(y), y.shape[1], _p(out))
    return out


def plSemicompleteCor2(pl):
    """pl: list of (i, v) pairs (increasing integer gene indices, values)."""
    npl = len(pl)
    off = np.zeros(npl + 1, np.int64)
    for k, (i, _) in enumerate(pl):
        off[k + 1] = off[k] + len(i)
    idx = np.ascontiguousarray(np.concatenate([np.asarray(i, np.int32) for i, _ in pl]) if npl else np.zeros(1),
                               dtype=np.int32)
    val = np.ascontiguousarray(np.concatenate([np.asarray(v, np.float64) for _, v in pl]) if npl else np.zeros(1),
                               dtype=np.float64)
    r = np.zeros((npl, npl), order="F")
    n = np.zeros((npl, npl), np.int32, order="F")
    if npl:
        lib().o_plSemicompleteCor2(npl, _p(off), _p(idx), _p(val), _p(r), _p(n))
    return {"r": r, "n": n}


def varnorm_weights(models, counts, prior_x, batch_codes=None, n_randomizations=100, n_cores=1,
                    use_expected_value=True):
    """pagoda.varnorm's modes and weight matrices (R/functions.R:1423-1507).

    modes: dataset-wide (1423-1431), then per batch level (1433-1450): jp %*% magnitudes, or the
    magnitude of the row maximum (the first maximum; R's max.col breaks ties at random);
    magnitudes = as.numeric(colnames(jp)) = exp(marginals) through as.character (15 digits).
    matw = 1 - mfp * sfp (1466-1474): mfp = scde.failure.probability(models, log(modes))
    (725-748, NaN -> 0), sfp = ppois(count - 1, exp(fail.r), lower.tail = FALSE); bmatw the
    same with each cell's batch modes (1485-1506)."""
    from scipy.stats import poisson
    from .oracle import MODEL_COLUMNS, marginals_from_prior_x, model_matrix, r_as_character_roundtrip, scde_posteriors
    counts = np.asarray(counts)
    N, C = counts.shape
    mm, lt, sq = model_matrix(models)
    mag = r_as_character_roundtrip(np.exp(marginals_from_prior_x(prior_x)))

    def modes_of(cells):
        sub = {k: np.asarray(v)[cells] for k, v in models.items()}
        jp = scde_posteriors(sub, np.ascontiguousarray(counts[:, cells]), prior_x, n_randomizations=n_randomizations,
                             n_cores=n_cores)
        if use_expected_value:
            out = np.zeros(N)
            for k in range(len(mag)):  # R's %*%: multiply then add, k in order
                out = out + jp[:, k] * mag[k]
            return out
        return mag[np.argmax(jp, axis=1)]

    allc = np.arange(C)
    modes = [modes_of(allc)]
    nb = 0 if batch_codes is None else int(np.max(batch_codes)) + 1
    if nb > 1:
        modes += [modes_of(np.nonzero(np.asarray(batch_codes) == k)[0]) for k in range(nb)]
    col = {c: j for j, c in enumerate(MODEL_COLUMNS)}

    def matw_of(mode_for_cell):
        out = np.zeros((N, C))
        for c in range(C):
            m = np.log(mode_for_cell(c))
            e = mm[c, col["conc.a"]] * m
            if sq:
                e = e + mm[c, col["conc.a2"]] * (m * m)
            with np.errstate(over="ignore", invalid="ignore"):
                mfp = 1.0 / (np.exp(e + mm[c, col["conc.b"]]) + 1.0)
            mfp[np.isnan(mfp)] = 0.0
            sfp = poisson.sf(counts[:, c] - 1, np.exp(mm[c, col["fail.r"]]))
            out[:, c] = 1.0 - mfp * sfp
        return out

    res = {"modes": np.vstack(modes), "matw": matw_of(lambda c: modes[0])}
    if nb > 1:
        res["bmatw"] = matw_of(lambda c: modes[1 + int(batch_codes[c])])
    return res
