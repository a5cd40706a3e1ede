"""TEST INFRASTRUCTURE ONLY -- CPU oracle for scde's PAGODA helper kernels
(src/pagoda.cpp: winsorizeMatrix, matCorr, matWCorr, plSemicompleteCor2), as ctypes
bindings to ``oracle/pagoda_oracle.c``.  Only ``tests/`` import this module.

R glue restated: ``winsorize_matrix`` (R/functions.R:1109-1115: trim > 0.5 means a
count, divided by ncol).
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
