"""The producers of the DE path's inputs.

  * ``expression_prior``      scde.expression.prior      R/functions.R:225-254, on the GPU
                              (``scde_expression_prior_dev``, csrc/prior.hip); counts may be
                              host arrays or a resident ``DeviceCounts``.
  * ``expression_magnitude``  scde.expression.magnitude  R/functions.R:694-697
  * ``failure_probability``   scde.failure.probability   R/functions.R:725-750
    (elementwise R-API helpers returning genes x cells matrices, numpy on the host).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import api
from ._lib import check, lib
from .models import as_model_dict, model_matrix


def expression_magnitude(models, counts):
    """t((t(log(counts)) - corr.b) / corr.a)   (natural-log FPM; log(0) = -inf)."""
    m = as_model_dict(models)
    c = np.asarray(counts, np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return (np.log(c) - m["corr.b"][None, :]) / m["corr.a"][None, :]


def failure_probability(models, magnitudes=None, counts=None):
    m = as_model_dict(models)
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


def expression_prior(models, counts, length_out=400, show_plot=False, pseudo_count=1, bw=0.1, max_quantile=1.0,
                     max_value=None, ctx: api.Context | None = None):
    """scde.expression.prior (R/functions.R:225-254) -> dict x, y, lp, grid.weight (and
    max.value, the value used).  Computed on the GPU; ``counts`` is a genes x cells matrix
    (columns matched to the model rows) or a ``DeviceCounts`` already in HBM."""
    ctx = ctx or api.default_context()
    mm, _, sq = model_matrix(models)
    own = not isinstance(counts, api.DeviceCounts)
    if own:
        mat, _ = api._align_counts(models, counts)
        dc = api.DeviceCounts(ctx, mat)
    else:
        dc = counts
    N, C = dc.ngenes, dc.ncells
    if C != mm.shape[0]:
        raise ValueError("counts and models disagree on the number of cells")
    L = int(length_out)
    out = np.zeros((4, L + 1))
    mv_out = ctypes.c_double()
    mv_in = None if max_value is None else ctypes.byref(ctypes.c_double(float(max_value)))
    try:
        check(lib().scde_expression_prior_dev(ctx.handle, dc.ptr, N, N, C, api._p(mm), sq, L, float(pseudo_count),
                                              float(bw), float(max_quantile), mv_in, api._p(out[0]), api._p(out[1]),
                                              api._p(out[2]), api._p(out[3]), ctypes.byref(mv_out)))
    finally:
        if own:
            dc.free()
    return {"x": out[0].copy(), "y": out[1].copy(), "lp": out[2].copy(), "grid.weight": out[3].copy(),
            "max.value": mv_out.value}
