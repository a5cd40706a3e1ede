"""CPU restatement of scde.expression.prior (R/functions.R:225-254) -- TEST INFRASTRUCTURE.

The checker for the device prior (scde_amd/csrc/prior.hip).  Only tests/, smoke() and
bench.py's cpu_baseline leg use it.  Pinned: the vignette fixtures
(tests/golden/vignette_*.npz) hold priors made by this code (max.quantile = 0.999), and the
oracle reproduces all 30 values the vignette prints from them exactly
(tests/test_oracle.py::test_vignette_*), so a prior that differed would have shown there.

  * ``expression_magnitude``  scde.expression.magnitude  R/functions.R:694-697
  * ``failure_probability``   scde.failure.probability   R/functions.R:725-750
  * ``expression_prior``      scde.expression.prior      R/functions.R:225-254, with
      - ``r_density``  stats::density.default (gaussian kernel, weights, the pre-4.4 grid
        lo = from - 4 bw): C_BinDist linear binning (src/library/stats/src/massdist.c),
        FFT cross-correlation with dnorm(kords, sd = bw), approx(rule = 1);
      - ``r_quantile7`` stats::quantile(type = 7).
"""
from __future__ import annotations

import math

import numpy as np

MODEL_COLUMNS = ["conc.b", "conc.a", "fail.r", "corr.b", "corr.a", "corr.theta", "corr.ltheta.b", "corr.ltheta.t",
                 "corr.ltheta.m", "corr.ltheta.s", "corr.ltheta.r", "conc.a2"]


def _model_dict(models):
    if isinstance(models, dict):
        return {k: np.asarray(v, np.float64) for k, v in models.items()}
    if hasattr(models, "columns"):
        return {k: models[k].to_numpy(np.float64) for k in models.columns}
    mm = np.asarray(models, np.float64)
    return {c: mm[:, j] for j, c in enumerate(MODEL_COLUMNS) if j < mm.shape[1] and not np.all(np.isnan(mm[:, j]))}


def expression_magnitude(models, counts):
    """t((t(log(counts)) - corr.b) / corr.a)   (natural-log FPM; log(0) = -inf)."""
    m = _model_dict(models)
    c = np.asarray(counts, np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (np.log(c) - m["corr.b"][None, :]) / m["corr.a"][None, :]


def failure_probability(models, magnitudes=None, counts=None):
    """R/functions.R:725-750 (matrix and common-vector forms); NaN -> 0."""
    m = _model_dict(models)
    if magnitudes is None:
        if counts is None:
            raise ValueError("ERROR: either magnitudes or counts should be provided")
        magnitudes = expression_magnitude(models, counts)
    mags = np.asarray(magnitudes, np.float64)
    with np.errstate(over="ignore", invalid="ignore"):
        if mags.ndim == 2:
            e = mags * m["conc.a"][None, :]
            if "conc.a2" in m:
                e = e + mags ** 2 * m["conc.a2"][None, :]
            x = 1.0 / (np.exp(e + m["conc.b"][None, :]) + 1.0)
        else:
            e = np.outer(m["conc.a"], mags)
            if "conc.a2" in m:
                e = e + np.outer(m["conc.a2"], mags ** 2)
            x = (1.0 / (np.exp(e + m["conc.b"][:, None]) + 1.0)).T
    x[np.isnan(x)] = 0
    return x


def r_quantile7(x, p):
    """quantile(x, p, type = 7) for one p."""
    xs = np.sort(np.asarray(x, np.float64))
    n = len(xs)
    index = 1 + max(n - 1, 0) * p
    lo = int(np.floor(index))
    hi = int(np.ceil(index))
    qs = xs[lo - 1]
    h = index - lo
    if index > lo and xs[hi - 1] != qs:
        qs = (1 - h) * qs + h * xs[hi - 1]
    return qs


def r_seq_len(frm, to, n):
    """seq.int(from, to, length.out = n)."""
    if n == 1:
        return np.array([frm], np.float64)
    by = (to - frm) / (n - 1)
    out = frm + np.arange(n, dtype=np.float64) * by
    out[-1] = to
    return out


def _bindist(x, w, lo, hi, n):
    """C_BinDist (massdist.c): linear binning into 2n cells, in input order."""
    y = np.zeros(2 * n)
    xdelta = (hi - lo) / (n - 1)
    ok = np.isfinite(x)
    x, w = x[ok], w[ok]
    xpos = (x - lo) / xdelta
    ix = np.floor(xpos).astype(np.int64)
    fx = xpos - ix
    ixmax = n - 2
    mid = (ix >= 0) & (ix <= ixmax)
    np.add.at(y, ix[mid], w[mid] * (1 - fx[mid]))
    np.add.at(y, ix[mid] + 1, w[mid] * fx[mid])
    left = ix == -1
    np.add.at(y, np.zeros(left.sum(), np.int64), w[left] * fx[left])
    right = ix == ixmax + 1
    np.add.at(y, ix[right], w[right] * (1 - fx[right]))
    return y


_DNORM_SPLIT_MAX = math.sqrt(-2 * math.log(2) * (-1021 + 1 - 53))
_M_1_SQRT_2PI = 0.398942280401432677939946059934


def r_dnorm(x, sd):
    """dnorm(x, 0, sd) as nmath dnorm4 (R >= 3.1: split x = x1 + x2 for x >= 5)."""
    x = np.abs(np.asarray(x, np.float64) / sd)
    out = _M_1_SQRT_2PI * np.exp(-0.5 * x * x) / sd
    big = x >= 5
    xb = x[big]
    x1 = np.ldexp(np.rint(np.ldexp(xb, 16)), -16)
    x2 = xb - x1
    out[big] = _M_1_SQRT_2PI / sd * (np.exp(-0.5 * x1 * x1) * np.exp((-0.5 * x2 - x1) * x2))
    out[x > _DNORM_SPLIT_MAX] = 0.0
    return out


def r_approx(x, y, v):
    """approx(x, y, xout = v, rule = 1): R's approx1 bisection and interpolation formula."""
    out = np.empty(len(v))
    n = len(x)
    for k, vk in enumerate(v):
        if vk < x[0] or vk > x[n - 1]:
            out[k] = np.nan
            continue
        i, j = 0, n - 1
        while i < j - 1:
            ij = (i + j) // 2
            if vk < x[ij]:
                j = ij
            else:
                i = ij
        if vk == x[j]:
            out[k] = y[j]
        elif vk == x[i]:
            out[k] = y[i]
        else:
            out[k] = y[i] + (y[j] - y[i]) * ((vk - x[i]) / (x[j] - x[i]))
    return out


def r_density(x, bw, weights, n_user, frm, to):
    """density.default(x, bw, weights=, n=, from=, to=) with the gaussian kernel (R < 4.4 grid)."""
    x = np.asarray(x, np.float64)
    w = np.asarray(weights, np.float64)
    fin = np.isfinite(x)
    wsum = w.sum()
    tot_mass = w[fin].sum() / wsum if not fin.all() else 1.0
    n = max(n_user, 512)
    if n > 512:
        n = int(2 ** np.ceil(np.log2(n)))
    lo = frm - 4 * bw
    up = to + 4 * bw
    y = _bindist(x, w, lo, up, n) * tot_mass
    kords = r_seq_len(0.0, 2 * (up - lo), 2 * n)
    kords[n + 1:2 * n] = -kords[n - 1:0:-1]
    kords = r_dnorm(kords, bw)
    conv = np.fft.ifft(np.fft.fft(y) * np.conj(np.fft.fft(kords)))
    kords = np.maximum(0.0, conv.real[:n])
    xords = r_seq_len(lo, up, n)
    xo = r_seq_len(frm, to, n_user)
    return xo, r_approx(xords, kords, xo)


def expression_prior(models, counts, length_out=400, pseudo_count=1, bw=0.1, max_quantile=1.0, max_value=None):
    """scde.expression.prior (R/functions.R:225-254).  Returns dict x, y, lp, grid.weight, max.value."""
    fpkm = expression_magnitude(models, counts)
    fail = failure_probability(models, counts=counts)
    with np.errstate(over="ignore"):
        fpkm = np.log10(np.exp(fpkm) + 1)
    wts = (1 - fail).ravel(order="F")
    wts = wts / wts.sum()
    if max_value is None:
        xv = fpkm.ravel(order="F")
        max_value = r_quantile7(xv[xv < np.inf], max_quantile)
    xs = fpkm.ravel(order="F")
    mx, my = r_density(np.concatenate([-xs, xs]), bw, np.concatenate([wts / 2, wts / 2]),
                       2 * length_out + 1, -max_value, max_value)
    gx = mx[length_out:]
    gy = my[length_out:].copy()
    gy[np.isnan(gy)] = 0
    gy = gy + pseudo_count / fpkm.shape[0]
    gy = gy / gy.sum()
    lp = np.log(gy)
    xe = np.concatenate([[gx[0]], gx + np.concatenate([np.diff(gx) / 2, [0.0]])])
    gw = np.diff(10.0 ** xe - 1)
    return {"x": gx, "y": gy, "lp": lp, "grid.weight": gw, "max.value": max_value}
