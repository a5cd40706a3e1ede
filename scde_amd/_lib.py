"""ctypes binding of ``libscde_hip.so`` (the C ABI in ``include/scde_hip.h``).

The product has no CPU fallback: if the HIP library is missing or no GPU is
visible, calls raise ``ScdeError`` instead of computing something else.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SCDE_LIB overrides the library path (tuning builds); the default is the in-tree build.
LIB_PATH = os.environ.get("SCDE_LIB") or os.path.join(_HERE, "libscde_hip.so")

# Symbols declared in include/scde_hip.h (checked by tests/test_abi.py).
EXPORTS = [
    "scde_last_error", "scde_version", "scde_set_rand_kind", "scde_get_rand_kind",
    "scde_logBootPosterior", "scde_logBootBatchPosterior", "scde_jpmatLogBoot", "scde_jpmatLogBatchBoot",
    "scde_matSlideMult", "scde_ratio_summary", "scde_distribution_summary", "scde_bh_cz",
    "scde_ctx_create", "scde_ctx_destroy", "scde_ctx_synchronize", "scde_ctx_set_profiling",
    "scde_ctx_kernel_times", "scde_ctx_reset_kernel_times", "scde_ctx_set_option", "scde_ctx_get_stat",
    "scde_ctx_reset_stats", "scde_ctx_inject_fault",
    "scde_dev_alloc", "scde_dev_free", "scde_h2d", "scde_d2h",
    "scde_expression_difference_dev", "scde_posteriors_dev", "scde_bh_cz_dev",
    "scde_expression_difference_batch_dev", "scde_expression_prior_dev",
    "scde_expression_difference_host", "scde_expression_difference_batch_host", "scde_posteriors_host",
    "scde_pagoda_varnorm_weights_dev", "scde_pagoda_varnorm_weights_host",
    "scde_baileyWPCA", "scde_bwpca_batch_dev", "scde_r_set_seed", "scde_r_unif_rand", "scde_r_sample",
    "scde_shuffle_perms", "scde_winsorizeMatrix", "scde_matWCorr", "scde_matCorr", "scde_plSemicompleteCor2",
]


class ScdeError(RuntimeError):
    pass


class DEParams(ctypes.Structure):
    _fields_ = [
        ("ncells", ctypes.c_int),
        ("models", ctypes.c_void_p),
        ("local_theta", ctypes.c_int),
        ("square_logit_conc", ctypes.c_int),
        ("groups", ctypes.c_void_p),
        ("prior_x", ctypes.c_void_p),
        ("prior_y", ctypes.c_void_p),
        ("ngrid", ctypes.c_int),
        ("nboot", ctypes.c_int),
        ("n_cores", ctypes.c_int),
        ("gene_offset", ctypes.c_int64),
        ("ngenes_total", ctypes.c_int64),
        ("expectation", ctypes.c_double),
        ("rand_kind", ctypes.c_int),
        ("compute_cz", ctypes.c_int),
    ]


_lib = None


def lib():
    """Load the library (raises ScdeError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ScdeError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                        " or `make -C scde_amd/csrc`")
    if not os.environ.get("SCDE_SKIP_TORCH"):  # host-only sanitizer runs load the library alone
        try:  # share torch's HIP runtime when torch is present (same SONAME)
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is optional plumbing
            pass
    L = ctypes.CDLL(LIB_PATH)
    P, i, i64, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
    L.scde_last_error.restype = ctypes.c_char_p
    L.scde_version.restype = i
    L.scde_set_rand_kind.argtypes = [i]
    L.scde_get_rand_kind.restype = i
    L.scde_logBootPosterior.argtypes = [P, i, P, P, P, i, P, i, i, i, i, i, i, i, P, P, P]
    L.scde_logBootBatchPosterior.argtypes = [P, i, P, P, P, i, P, i, P, P, P, i, i, i, i, i, i, P, P, P]
    L.scde_jpmatLogBoot.argtypes = [P, i, i, i, i, i, P]
    L.scde_jpmatLogBatchBoot.argtypes = [P, P, P, i, i, i, i, i, P]
    L.scde_matSlideMult.argtypes = [P, P, i, i, P]
    L.scde_ratio_summary.argtypes = [P, P, i, i, P, P, i, P, P]
    L.scde_bh_cz.argtypes = [P, i64, P]
    L.scde_distribution_summary.argtypes = [P, i, i, P, i, P]
    L.scde_ctx_create.argtypes = [i, ctypes.POINTER(P)]
    L.scde_ctx_destroy.argtypes = [P]
    L.scde_ctx_destroy.restype = None
    L.scde_ctx_synchronize.argtypes = [P]
    L.scde_ctx_set_profiling.argtypes = [P, i]
    L.scde_ctx_kernel_times.argtypes = [P, P, P, i]
    L.scde_ctx_reset_kernel_times.argtypes = [P]
    L.scde_ctx_set_option.argtypes = [P, ctypes.c_char_p, d]
    L.scde_ctx_get_stat.argtypes = [P, ctypes.c_char_p, P]
    L.scde_ctx_reset_stats.argtypes = [P]
    if hasattr(L, "scde_ctx_inject_fault"):  # (study builds of earlier rounds lack the test hook)
        L.scde_ctx_inject_fault.argtypes = [P, ctypes.c_char_p, i]
    L.scde_dev_alloc.argtypes = [P, i64, ctypes.POINTER(P)]
    L.scde_dev_free.argtypes = [P, P]
    L.scde_h2d.argtypes = [P, P, P, i64]
    L.scde_d2h.argtypes = [P, P, P, i64]
    L.scde_bh_cz_dev.argtypes = [P, P, i64, P]
    L.scde_expression_difference_dev.argtypes = [P, P, i64, i, ctypes.POINTER(DEParams), P, P, P, P]
    L.scde_expression_difference_batch_dev.argtypes = [P, P, i64, i, ctypes.POINTER(DEParams), P, P, i, P, P, P, P,
                                                       P, P]
    L.scde_expression_difference_host.argtypes = [P, P, i64, i, ctypes.POINTER(DEParams), P, P, P, P]
    L.scde_expression_difference_batch_host.argtypes = [P, P, i64, i, ctypes.POINTER(DEParams), P, P, i, P, P, P, P,
                                                        P, P]
    L.scde_posteriors_host.argtypes = [P, P, i64, i, i, P, i, P, i, i, P, i, i, i, i64, i64, i, i, P, P, P, i, P, P,
                                       P]
    L.scde_pagoda_varnorm_weights_dev.argtypes = [P, P, i64, i, i, P, i, i, P, i, i, i, P, i, i, P, P, P]
    L.scde_pagoda_varnorm_weights_host.argtypes = [P, P, i64, i, i, P, i, i, P, i, i, i, P, i, i, P, P, P]
    L.scde_expression_prior_dev.argtypes = [P, P, i64, i, i, P, i, i, d, d, d, P, P, P, P, P, P]
    L.scde_posteriors_dev.argtypes = [P, P, i64, i, P, i, P, i, i, P, i, i, i, i64, i64, i, i, P, P, P, i, P, P, P]
    L.scde_baileyWPCA.argtypes = [P, P, i, i, i, i, i, d, i, P, i, P, P, P, P, P, P, P]
    L.scde_bwpca_batch_dev.argtypes = [P, P, P, i64, i, i64, i, P, P, P, P, P, i64, P, P, i64, P, P, i64, i, d, i,
                                       P, P, P, P, P, P]
    L.scde_r_set_seed.argtypes = [ctypes.c_uint32, P]
    L.scde_r_unif_rand.argtypes = [P, i64, P]
    L.scde_r_sample.argtypes = [P, i, i, P]
    L.scde_shuffle_perms.argtypes = [ctypes.c_uint, i, i, i, P]
    L.scde_winsorizeMatrix.argtypes = [P, i, i, d, P]
    L.scde_matWCorr.argtypes = [P, P, i, i, P]
    L.scde_matCorr.argtypes = [P, i, i, P, i, P]
    L.scde_plSemicompleteCor2.argtypes = [i, P, P, P, P, P]
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        msg = lib().scde_last_error().decode("utf-8", "replace")
        raise ScdeError(f"scde_hip error {rc}: {msg}")
