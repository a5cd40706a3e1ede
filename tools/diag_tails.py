"""Diagnostic: relative error of jp (layer-1 logBootPosterior) against the oracle by
magnitude band, for two library builds (e.g. before/after a numerics change)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402
from scde_amd.prior import expression_prior  # noqa: E402

import torch  # noqa: E402,F401  (HIP runtime first, as scde_amd._lib does)


def run_lib(path, mm, ucl, uci, mag, nboot, seed, lt, sq):
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    i = ctypes.c_int
    L.scde_logBootPosterior.argtypes = [P, i, P, P, P, i, P, i, i, i, i, i, i, i, P, P, P]
    L.scde_last_error.restype = ctypes.c_char_p
    vals = np.ascontiguousarray(np.concatenate(ucl), np.int32)
    off = np.zeros(len(ucl) + 1, np.int64)
    off[1:] = np.cumsum([len(u) for u in ucl])
    N, C = uci.shape
    G = len(mag)
    jp = np.zeros((N, G), order="F")
    ci = np.asfortranarray(uci, np.int32)
    rc = L.scde_logBootPosterior(mm.ctypes.data, C, vals.ctypes.data, off.ctypes.data, ci.ctypes.data, N,
                                 mag.ctypes.data, G, nboot, seed, 0, lt, sq, 0, jp.ctypes.data, None, None)
    assert rc == 0, L.scde_last_error()
    return jp


def bands(a, b):
    rowmax = np.maximum(np.abs(a).max(1), np.abs(b).max(1))[:, None]
    rel = np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-300)
    out = {}
    for lo, hi in ((1e-6, 2), (1e-12, 1e-6), (1e-16, 1e-12), (1e-20, 1e-16)):
        m = (np.maximum(np.abs(a), np.abs(b)) >= lo * rowmax) & (np.maximum(np.abs(a), np.abs(b)) < hi * rowmax)
        out[f"[{lo:g},{hi:g})"] = (float(rel[m].max()) if m.any() else None, int(m.sum()))
    return out


def main():
    models, counts, groups = bench.synthetic(7003, 160, 1000)
    prior = expression_prior(models, counts, length_out=400)
    ii = np.nonzero(groups == 0)[0]
    sub = {k: v[ii] for k, v in models.items()}
    mm, lt, sq = O.model_matrix(sub)
    mm = np.asfortranarray(mm)
    mag = np.ascontiguousarray(O.marginals_from_prior_x(prior["x"]))
    ucl, uci = O.ucl_uci(counts[:, ii])
    O.set_rng(0)  # glibc
    ref = O.logBootPosterior(mm, ucl, uci, mag, 12, 1, 0, lt, sq, 0)
    for path in sys.argv[1:]:
        jp = run_lib(path, mm, ucl, uci, mag, 12, 1, lt, sq)
        print(path, bands(jp, ref))


if __name__ == "__main__":
    main()
