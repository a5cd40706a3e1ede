"""Python mirror of the R-level scde API on the DE hot path, backed by HIP.

Same names (dots -> underscores), argument meaning and return shapes as the
reference R functions; every numeric step runs in ``libscde_hip.so``:

  * ``scde_expression_difference``  R/functions.R:304-407
  * ``scde_posteriors``             R/functions.R:566-669
  * ``calculate_ratio_posterior``   R/functions.R:3491-3510
  * ``quick_distribution_summary``  R/functions.R:5039-5053
  * ``.Call`` entry points          ``logBootPosterior`` / ``logBootBatchPosterior`` /
    ``jpmatLogBoot`` / ``jpmatLogBatchBoot`` / ``matSlideMult``
    (src/jpmatLogBoot.cpp, src/matSlideMult.cpp)

Inputs follow R's conventions: ``models`` rows are cells, ``counts`` is a
genes x cells integer matrix whose columns are named by cell, ``prior`` has
``x`` (log10 grid) and ``y`` (prior density).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from . import _lib
from ._lib import DEParams, ScdeError, check, lib
from .models import as_model_dict, model_matrix, model_rownames

P = ctypes.c_void_p


def _p(a):
    return None if a is None else a.ctypes.data_as(P)


def _f64(a):
    return np.require(a, dtype=np.float64, requirements=["F", "A", "W"])


def _i32(a):
    return np.require(a, dtype=np.int32, requirements=["F", "A"])


def _flatten_list(lst):
    if len(lst) == 0:
        return np.zeros(1, np.int32), np.zeros(1, np.int64)
    vals = np.ascontiguousarray(np.concatenate([np.asarray(v, np.int32).ravel() for v in lst]), np.int32)
    if vals.size == 0:
        vals = np.zeros(1, np.int32)
    off = np.zeros(len(lst) + 1, np.int64)
    off[1:] = np.cumsum([np.asarray(v).size for v in lst])
    return vals, off


# ================================================================== .Call mirrors
def logBootPosterior(Models, Ucl, CountsI, Magnitudes, Nboot, Seed, ReturnIndividualPosteriors=0,
                     LocalThetaFit=0, SquareLogitConc=0, EnsembleProbability=0):
    """src/jpmatLogBoot.cpp:100.  Returns jp (ngenes x ngrid) or a dict with jp/modes/post."""
    mm = _f64(Models)
    C = mm.shape[0]
    uci = _i32(CountsI)
    N = uci.shape[0]
    mag = _f64(Magnitudes)
    G = mag.shape[0]
    vals, off = _flatten_list(Ucl)
    rp = int(ReturnIndividualPosteriors)
    jp = np.zeros((N, G), order="F")
    modes = np.zeros((N, C), order="F") if rp in (1, 3) else None
    post = np.zeros(C * N * G) if rp in (2, 3) else None
    check(lib().scde_logBootPosterior(_p(mm), C, _p(vals), _p(off), _p(uci), N, _p(mag), G, int(Nboot), int(Seed),
                                      rp, int(LocalThetaFit), int(SquareLogitConc), int(EnsembleProbability),
                                      _p(jp), _p(modes), _p(post)))
    return _pack(jp, modes, post, rp, C, N, G)


def _pack(jp, modes, post, rp, C, N, G):
    if rp == 0:
        return jp
    out = {"jp": jp}
    if modes is not None:
        out["modes"] = modes
    if post is not None:
        out["post"] = [post[i * N * G:(i + 1) * N * G].reshape((N, G), order="F") for i in range(C)]
    return out


def logBootBatchPosterior(Models, Ucl, CountsI, Magnitudes, BatchIL, Composition, Nboot, Seed,
                          ReturnIndividualPosteriors=0, LocalThetaFit=0, SquareLogitConc=0):
    """src/jpmatLogBoot.cpp:343."""
    mm = _f64(Models)
    C = mm.shape[0]
    uci = _i32(CountsI)
    N = uci.shape[0]
    mag = _f64(Magnitudes)
    G = mag.shape[0]
    vals, off = _flatten_list(Ucl)
    bvals, boff = _flatten_list(BatchIL)
    comp = np.ascontiguousarray(Composition, np.int32)
    rp = int(ReturnIndividualPosteriors)
    rpe = rp if rp in (1, 2) else 0
    jp = np.zeros((N, G), order="F")
    modes = np.zeros((N, C), order="F") if rpe == 1 else None
    post = np.zeros(C * N * G) if rpe == 2 else None
    check(lib().scde_logBootBatchPosterior(_p(mm), C, _p(vals), _p(off), _p(uci), N, _p(mag), G, _p(bvals),
                                           _p(boff), _p(comp), len(comp), int(Nboot), int(Seed), rp,
                                           int(LocalThetaFit), int(SquareLogitConc), _p(jp), _p(modes), _p(post)))
    return _pack(jp, modes, post, rpe, C, N, G)


def jpmatLogBoot(Matl, Nboot, Seed):
    """src/jpmatLogBoot.cpp:11."""
    mats = [_f64(m) for m in Matl]
    nr, nc = mats[0].shape
    ptrs = (P * len(mats))(*[m.ctypes.data for m in mats])
    out = np.zeros((nr, nc), order="F")
    check(lib().scde_jpmatLogBoot(ptrs, len(mats), nr, nc, int(Nboot), int(Seed), _p(out)))
    return out


def jpmatLogBatchBoot(Matll, Comp, Nboot, Seed):
    """src/jpmatLogBoot.cpp:48."""
    mats = [_f64(m) for lst in Matll for m in lst]
    toff = np.zeros(len(Matll) + 1, np.int32)
    toff[1:] = np.cumsum([len(lst) for lst in Matll])
    nr, nc = mats[0].shape
    ptrs = (P * len(mats))(*[m.ctypes.data for m in mats])
    comp = np.ascontiguousarray(Comp, np.int32)
    out = np.zeros((nr, nc), order="F")
    check(lib().scde_jpmatLogBatchBoot(ptrs, _p(toff), _p(comp), len(Matll), nr, nc, int(Nboot), int(Seed), _p(out)))
    return out


def matSlideMult(Mat1, Mat2):
    """src/matSlideMult.cpp:5."""
    a, b = _f64(Mat1), _f64(Mat2)
    nr, n = a.shape
    out = np.zeros((nr, 2 * n - 1), order="F")
    check(lib().scde_matSlideMult(_p(a), _p(b), nr, n, _p(out)))
    return out


# ================================================================== platform rand()
RAND_KINDS = {"glibc": 0, "darwin": 2}


def set_rand(kind: str):
    """Select which C-library rand() the bootstrap reproduces: "glibc" (Linux, default) or
    "darwin" (macOS/BSD Park-Miller; the generator behind the vignette's printed numbers)."""
    check(lib().scde_set_rand_kind(RAND_KINDS[kind]))


def get_rand_kind() -> int:
    return int(lib().scde_get_rand_kind())


# ================================================================== R glue helpers (host)
def marginals(prior_x):
    """R/functions.R:575-577: log(pmax(10^x - 1, 0)); R's `^` is libm pow()."""
    m = np.array([math.pow(10.0, v) for v in np.asarray(prior_x, np.float64)]) - 1
    m[m < 0] = 0
    with np.errstate(divide="ignore"):
        return np.log(m)


def _r_seq(frm, to, n):
    out = frm + np.arange(n, dtype=np.float64) * ((to - frm) / (n - 1))
    out[0], out[-1] = frm, to
    return out


def ratio_columns(prior_x):
    """as.numeric(colnames(ratio)): seq(x1-xn, xn-x1, length = 2n-1) round-tripped through
    R's 15-significant-digit as.character (R/functions.R:3506, 5040)."""
    x = np.asarray(prior_x, np.float64)
    rv = _r_seq(x[0] - x[-1], x[-1] - x[0], 2 * len(x) - 1)
    return np.array([float("%.15g" % v) for v in rv])


def expectation_column(diffv, expectation=0.0):
    """which.min(abs(diffv - expectation/log2(10))) - 1 (R/functions.R:3524)."""
    return int(np.argmin(np.abs(np.asarray(diffv) - expectation / np.log2(10.0))))


class RatioPosterior:
    """A ratio (fold-difference) posterior: ``values`` ngenes x ncol, ``columns`` numeric colnames."""

    def __init__(self, values, columns, rownames=None):
        self.values = values
        self.columns = np.asarray(columns, np.float64)
        self.rownames = rownames

    @property
    def shape(self):
        return self.values.shape


def _frame(cols: dict, rownames):
    try:
        import pandas as pd
        return pd.DataFrame(cols, index=rownames)
    except Exception:  # pragma: no cover
        return cols


# ================================================================== device context
class Context:
    """A device + HIP stream + workspace (``scde_ctx``)."""

    def __init__(self, device: int = 0):
        self.handle = P()
        check(lib().scde_ctx_create(int(device), ctypes.byref(self.handle)))
        self.device = device

    def close(self):
        if self.handle:
            lib().scde_ctx_destroy(self.handle)
            self.handle = P()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        check(lib().scde_ctx_synchronize(self.handle))

    def set_profiling(self, on: bool):
        check(lib().scde_ctx_set_profiling(self.handle, int(bool(on))))

    SLOT_NAMES = ["tables", "boot", "ratio_summary", "unique", "other", "prior_stats", "prior_bin", "prior_tail",
                  "wpca_em", "wpca_final"]

    def kernel_times(self):
        """{slot: (total ms, launches)} from HIP events on the context's stream."""
        names = self.SLOT_NAMES
        ms = np.zeros(len(names))
        n = np.zeros(len(names), np.int64)
        check(lib().scde_ctx_kernel_times(self.handle, _p(ms), _p(n), len(names)))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(names)}

    def reset_kernel_times(self):
        check(lib().scde_ctx_reset_kernel_times(self.handle))

    def set_option(self, name: str, value: float):
        """Tuning / test switches (include/scde_hip.h scde_ctx_set_option)."""
        check(lib().scde_ctx_set_option(self.handle, name.encode(), float(value)))

    def stat(self, name: str) -> float:
        v = ctypes.c_double()
        check(lib().scde_ctx_get_stat(self.handle, name.encode(), ctypes.byref(v)))
        return v.value

    def inject_fault(self, where: str, count: int = 1):
        """Test hook (include/scde_hip.h scde_ctx_inject_fault): the next `count` failures at `where`."""
        check(lib().scde_ctx_inject_fault(self.handle, where.encode(), int(count)))

    def reset_stats(self):
        check(lib().scde_ctx_reset_stats(self.handle))


class DeviceCounts:
    """An int32 genes x cells count matrix resident in HBM (R column-major layout)."""

    def __init__(self, ctx: Context, counts):
        c = np.asfortranarray(np.asarray(counts), dtype=np.int32)
        if c.ndim != 2:
            raise ValueError("counts must be a genes x cells matrix")
        self.ctx = ctx
        self.ngenes, self.ncells = c.shape
        self.ptr = P()
        nbytes = max(1, c.nbytes)
        check(lib().scde_dev_alloc(ctx.handle, nbytes, ctypes.byref(self.ptr)))
        if c.nbytes:
            check(lib().scde_h2d(ctx.handle, self.ptr, _p(c), c.nbytes))

    def free(self):
        if self.ptr:
            check(lib().scde_dev_free(self.ctx.handle, self.ptr))
            self.ptr = P()


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


def _counts_matrix(counts):
    """(int32 genes x cells array, gene names, cell names)."""
    if hasattr(counts, "columns") and hasattr(counts, "index"):
        return (np.asarray(counts.values), [str(x) for x in counts.index], [str(x) for x in counts.columns])
    return np.asarray(counts), None, None


def _align_counts(models, counts):
    """Reorder counts columns to the model rows (R/functions.R:305-310)."""
    mat, genes, cells = _counts_matrix(counts)
    rn = model_rownames(models)
    if rn is not None and cells is not None:
        missing = [r for r in rn if r not in cells]
        if missing:
            raise ValueError("ERROR: provided count data does not cover all of the cells specified in the model matrix")
        pos = {c: i for i, c in enumerate(cells)}
        mat = mat[:, [pos[r] for r in rn]]
    mat = np.asarray(mat)
    if not np.issubdtype(mat.dtype, np.integer) and np.any(mat != np.round(mat)):
        raise ValueError("counts must be integers")
    return np.asfortranarray(mat, dtype=np.int32), genes


# ================================================================== R API
def scde_posteriors(models, counts, prior, n_randomizations=100, batch=None, composition=None,
                    return_individual_posteriors=False, return_individual_posterior_modes=False,
                    ensemble_posterior=False, n_cores=20, ctx: Context | None = None):
    """scde.posteriors (R/functions.R:566-669).  ``n_cores`` only selects the reference's
    per-chunk bootstrap seeds (results depend on it exactly as in R); all chunks run in one
    device pass."""
    ctx = ctx or default_context()
    mat, genes = _align_counts(models, counts)
    N, C = mat.shape
    mm, lt, sq = model_matrix(models)
    postflag = 0
    if return_individual_posteriors:
        postflag = 3 if return_individual_posterior_modes else 2
    elif return_individual_posterior_modes:
        postflag = 1
    prior_x = np.ascontiguousarray(prior["x"], np.float64)
    G = len(prior_x)
    bvals = boff = comp = None
    nbatch = 0
    if batch is not None:
        if composition is None:
            raise ValueError("ERROR: group composition must be provided if the batch argument is passed")
        batch = np.asarray(batch)
        levels = sorted(set(batch.tolist()))
        bvals, boff = _flatten_list([np.nonzero(batch == lv)[0] for lv in levels])
        if isinstance(composition, dict):
            comp = np.array([composition.get(lv, 0) for lv in levels], np.int32)
        else:
            comp = np.ascontiguousarray(composition, np.int32)
        nbatch = len(levels)
    jp = np.zeros((N, G), order="F")
    bt = batch is not None
    want_modes = postflag == 1 if bt else postflag in (1, 3)
    want_post = postflag == 2 if bt else postflag in (2, 3)
    modes = np.zeros((N, C), order="F") if want_modes else None
    post = np.zeros(C * N * G) if want_post else None
    cellidx = np.arange(C, dtype=np.int32)
    check(lib().scde_posteriors_host(ctx.handle, _p(mat), N, N, C, _p(cellidx), C, _p(mm), lt, sq, _p(prior_x), G,
                                     int(n_randomizations), int(n_cores), 0, N, postflag,
                                     int(bool(ensemble_posterior)), _p(bvals), _p(boff), _p(comp), nbatch,
                                     _p(jp), _p(modes), _p(post)))
    if postflag == 0 or (bt and postflag == 3):
        return jp
    out = {"jp": jp}
    if modes is not None:
        out["modes"] = modes
    if post is not None:
        out["post"] = [post[i * N * G:(i + 1) * N * G].reshape((N, G), order="F") for i in range(C)]
    return out


def calculate_ratio_posterior(pmat1, pmat2, prior, n_cores=15, skip_prior_adjustment=False):
    """calculate.ratio.posterior (R/functions.R:3491-3510) -> RatioPosterior."""
    a, b = _f64(pmat1), _f64(pmat2)
    nr, n = a.shape
    y = None if skip_prior_adjustment else np.ascontiguousarray(prior["y"], np.float64)
    out = np.zeros((nr, 2 * n - 1), order="F")
    check(lib().scde_ratio_summary(_p(a), _p(b), nr, n, _p(y), None, 0, _p(out), None))
    return RatioPosterior(out, ratio_columns(prior["x"]))


def _bh(z):
    z = np.ascontiguousarray(z, np.float64)
    cz = np.zeros_like(z)
    check(lib().scde_bh_cz(_p(z), z.size, _p(cz)))
    return cz


def quick_distribution_summary(s_bdiffp, expectation=0.0, rownames=None):
    """quick.distribution.summary (R/functions.R:5039-5053) of a RatioPosterior."""
    r = _f64(s_bdiffp.values)
    nr, m = r.shape
    diffv = np.ascontiguousarray(s_bdiffp.columns, np.float64)
    zi = expectation_column(diffv, expectation)
    res = np.zeros((nr, 5), order="F")
    check(lib().scde_distribution_summary(_p(r), nr, m, _p(diffv), zi, _p(res)))
    return _result_frame(res, _bh(res[:, 4]), rownames or s_bdiffp.rownames)


def _result_frame(res, cz, rownames):
    return _frame({"lb": res[:, 0].copy(), "mle": res[:, 1].copy(), "ub": res[:, 2].copy(),
                   "ce": res[:, 3].copy(), "Z": res[:, 4].copy(), "cZ": cz}, rownames)


def _groups_vector(models, groups):
    """groups factor -> per-cell level code (0/1, -1 = NA), levels in factor order."""
    if groups is None:
        raise ValueError("ERROR: groups factor is not provided")
    rn = model_rownames(models)
    if hasattr(groups, "cat") and hasattr(groups, "index"):  # pandas categorical Series
        levels = list(groups.cat.categories)
        codes = groups.cat.codes.to_numpy()
        if rn is not None:
            pos = {str(k): i for i, k in enumerate(groups.index)}
            if all(r in pos for r in rn):
                codes = np.array([codes[pos[r]] for r in rn])
        codes = np.where(codes < 0, -1, codes)
    else:
        g = list(groups)
        levels = sorted(set(x for x in g if x is not None and x == x))
        codes = np.array([levels.index(x) if (x is not None and x == x) else -1 for x in g])
    if len(levels) != 2:
        raise ValueError("ERROR: wrong number of levels in the grouping factor (%s), but must be two."
                         % " ".join(map(str, levels)))
    return np.ascontiguousarray(codes, np.int32)


def scde_expression_difference(models, counts, prior, groups=None, batch=None, n_randomizations=150, n_cores=10,
                               batch_models=None, return_posteriors=False, expectation=0, verbose=0,
                               ctx: Context | None = None):
    """scde.expression.difference (R/functions.R:304-407)."""
    ctx = ctx or default_context()
    mat, genes = _align_counts(models, counts)
    N, C = mat.shape
    if groups is None and hasattr(models, "attrs") and "groups" in getattr(models, "attrs", {}):
        groups = models.attrs["groups"]
    codes = _groups_vector(models, groups)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    G = len(px)
    correct_batch = batch is not None and len(set(b for b in np.asarray(batch, dtype=object).tolist()
                                                  if b is not None)) > 1
    if correct_batch:
        return _expression_difference_batch(models, mat, genes, prior, codes, np.asarray(batch, dtype=object),
                                            n_randomizations,
                                            n_cores, batch_models if batch_models is not None else models,
                                            return_posteriors, expectation, ctx)
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, G,
                      int(n_randomizations), int(n_cores), 0, N, float(expectation), get_rand_kind(), 1)
    res = np.zeros((N, 6), order="F")  # lb, mle, ub, ce, Z, cZ (BH on device)
    jp1 = np.zeros((N, G), order="F") if return_posteriors else None
    jp2 = np.zeros((N, G), order="F") if return_posteriors else None
    ratio = np.zeros((N, 2 * G - 1), order="F") if return_posteriors else None
    check(lib().scde_expression_difference_host(ctx.handle, _p(mat), N, N, ctypes.byref(params), _p(res), _p(jp1),
                                                _p(jp2), _p(ratio)))
    table = _result_frame(res[:, :5], res[:, 5].copy(), genes)
    if return_posteriors:
        return {"results": table, "difference.posterior": RatioPosterior(ratio, ratio_columns(px), genes),
                "joint.posteriors": [jp1, jp2]}
    return table


def _expression_difference_batch(models, mat, genes, prior, codes, batch, nrand, n_cores, batch_models,
                                 return_posteriors, expectation, ctx):
    """Batch-corrected branch (R/functions.R:321-399) as one device-resident call
    (scde_expression_difference_batch_dev): batch posteriors over all cells with each
    group's batch composition, the group posteriors, the three ratio posteriors and their
    summaries with BH, all in HBM."""
    N, C = mat.shape
    # None is an NA batch label: the cell joins no level (code -1), as tapply/table drop it
    levels = sorted(set(b for b in batch.tolist() if b is not None))
    bcodes = np.ascontiguousarray([-1 if b is None else levels.index(b) for b in batch.tolist()], np.int32)
    mm, lt, sq = model_matrix(models)
    bmm, blt, bsq = model_matrix(batch_models)
    if (blt, bsq) != (lt, sq):
        raise ValueError("batch.models must be of the same model type as models")
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    G = len(px)
    codes = np.ascontiguousarray(codes, np.int32)
    res = np.zeros((N, 18), order="F")
    rp = return_posteriors
    jp1 = np.zeros((N, G), order="F") if rp else None
    jp2 = np.zeros((N, G), order="F") if rp else None
    ratio = np.zeros((N, 2 * G - 1), order="F") if rp else None
    adj = np.zeros((N, 4 * G - 3), order="F") if rp else None
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, G,
                      int(nrand), int(n_cores), 0, N, float(expectation), get_rand_kind(), 1)
    check(lib().scde_expression_difference_batch_host(ctx.handle, _p(mat), N, N, ctypes.byref(params), _p(bmm),
                                                      _p(bcodes), len(levels), _p(res), _p(jp1), _p(jp2), _p(ratio),
                                                      _p(adj), None))
    tables = [_result_frame(res[:, 6 * k: 6 * k + 5], res[:, 6 * k + 5].copy(), genes) for k in range(3)]
    out = {"batch.adjusted": tables[0], "results": tables[1], "batch.effect": tables[2]}
    if rp:
        cols = ratio_columns(px)
        out.update({"difference.posterior": RatioPosterior(ratio, cols, genes),
                    "batch.adjusted.difference.posterior": RatioPosterior(adj, ratio_columns(cols), genes),
                    "joint.posteriors": [jp1, jp2]})
    return out


def bh_cz(z):
    """cZ from Z (R/functions.R:5051), computed by the library's host code."""
    return _bh(z)


def bh_cz_device(ctx: Context, z_ptr: int, n: int, cz_ptr: int):
    """cZ from Z for device buffers (HBM pointers, n doubles each), on the context's stream."""
    check(lib().scde_bh_cz_dev(ctx.handle, ctypes.c_void_p(z_ptr), int(n), ctypes.c_void_p(cz_ptr)))


__all__ = ["scde_posteriors", "scde_expression_difference", "calculate_ratio_posterior", "quick_distribution_summary",
           "logBootPosterior", "logBootBatchPosterior", "jpmatLogBoot", "jpmatLogBatchBoot", "matSlideMult",
           "marginals", "ratio_columns", "expectation_column", "Context", "DeviceCounts", "RatioPosterior",
           "ScdeError", "bh_cz", "bh_cz_device", "set_rand"]
