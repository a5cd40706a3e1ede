"""Error-model table handling (the `models` data.frame of the R API).

The R code builds the ncells x 12 model matrix `mm` from named columns
(R/functions.R:600-604); absent columns are NA.  Column presence selects the
local-theta and squared-logit code paths (R/functions.R:597-598).
"""
from __future__ import annotations

import numpy as np

MODEL_COLUMNS = ["conc.b", "conc.a", "fail.r", "corr.b", "corr.a", "corr.theta",
                 "corr.ltheta.b", "corr.ltheta.t", "corr.ltheta.m", "corr.ltheta.s",
                 "corr.ltheta.r", "conc.a2"]


def as_model_dict(models) -> dict:
    """Accept a pandas DataFrame (rows = cells), a dict of column -> vector, or a
    numpy structured array; return {column: float64 vector}."""
    if hasattr(models, "columns") and hasattr(models, "index"):
        return {str(c): np.asarray(models[c], np.float64) for c in models.columns}
    if isinstance(models, dict):
        return {str(k): np.asarray(v, np.float64) for k, v in models.items()}
    if getattr(models, "dtype", None) is not None and models.dtype.names:
        return {n: np.asarray(models[n], np.float64) for n in models.dtype.names}
    raise TypeError("models must be a DataFrame, a dict of columns or a structured array")


def model_rownames(models):
    if hasattr(models, "index"):
        return [str(x) for x in models.index]
    return None


def model_matrix(models):
    """(mm [ncells x 12, Fortran order, NaN where absent], local_theta, square_logit_conc)."""
    m = as_model_dict(models)
    ncells = len(next(iter(m.values())))
    mm = np.full((ncells, 12), np.nan, order="F")
    for j, nm in enumerate(MODEL_COLUMNS):
        if nm in m:
            mm[:, j] = m[nm]
    return mm, int("corr.ltheta.b" in m), int("conc.a2" in m)


def subset_models(models, idx):
    m = as_model_dict(models)
    return {k: v[idx] for k, v in m.items()}
