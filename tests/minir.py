"""TEST INFRASTRUCTURE: drive R/src/scde_hip_shim.c's .Call entry points from Python through
tests/rstub/minir.c (a minimal stand-in for the R C API; R is absent from this image).  The
shim and minir are built into tests/rstub/libshim_minir.so by __graft_entry__.build() and
linked against scde_amd/libscde_hip.so, exactly as R would load the shim with the library.

R objects are made from numpy arrays (column-major matrices keep their dims, Python lists
become VECSXP lists, bools logical scalars, None R_NilValue); results come back as numpy
arrays, or dicts for named lists."""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "rstub", "libshim_minir.so")
INTSXP, LGLSXP, REALSXP, STRSXP, VECSXP, NILSXP = 13, 10, 14, 16, 19, 0

_L = None


def build():
    import subprocess
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-O1", "-std=gnu99", "-Wall", "-Wno-unused-parameter",
                           "-I", os.path.join(ROOT, "tests", "rstub"), "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "R", "src", "scde_hip_shim.c"),
                           os.path.join(ROOT, "tests", "rstub", "minir.c"), "-o", SO,
                           "-L", os.path.join(ROOT, "scde_amd"), "-lscde_hip",
                           "-Wl,-rpath," + os.path.join("$ORIGIN", "..", "..", "scde_amd")])


def lib():
    global _L
    if _L is not None:
        return _L
    from scde_amd import _lib
    _lib.lib()  # libscde_hip.so (and torch's HIP runtime) first, as R's dyn.load order would have it
    L = ctypes.CDLL(SO)
    P, x = ctypes.c_void_p, ctypes.c_ssize_t
    for name, res, args in [
        ("minir_nil", P, []), ("minir_real", P, [x, P]), ("minir_int", P, [x, P]), ("minir_lgl", P, [ctypes.c_int]),
        ("minir_real_matrix", P, [ctypes.c_int, ctypes.c_int, P]),
        ("minir_int_matrix", P, [ctypes.c_int, ctypes.c_int, P]), ("minir_list", P, [x]),
        ("minir_set", None, [P, x, P]), ("minir_type", ctypes.c_int, [P]), ("minir_length", x, [P]),
        ("minir_nrow", ctypes.c_int, [P]), ("minir_ncol", ctypes.c_int, [P]), ("minir_data", P, [P]),
        ("minir_elt", P, [P, x]), ("minir_name", ctypes.c_char_p, [P, x]), ("minir_error", ctypes.c_char_p, []),
        ("minir_call", P, [P, ctypes.c_int, P]), ("minir_set_seed", None, [ctypes.c_uint]),
        ("minir_protect_depth", ctypes.c_int, []),
    ]:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _L = L
    return L


class RError(RuntimeError):
    pass


def to_r(v):
    L = lib()
    if v is None:
        return L.minir_nil()
    if isinstance(v, bool):
        return L.minir_lgl(int(v))
    if isinstance(v, (list, tuple)):
        lst = L.minir_list(len(v))
        for i, e in enumerate(v):
            L.minir_set(lst, i, to_r(e))
        return lst
    if isinstance(v, (int, np.integer)):
        a = np.array([v], np.int32)
        return L.minir_int(1, a.ctypes.data)
    if isinstance(v, (float, np.floating)):
        a = np.array([v], np.float64)
        return L.minir_real(1, a.ctypes.data)
    a = np.asarray(v)
    if a.ndim == 2:
        if np.issubdtype(a.dtype, np.integer):
            a = np.asfortranarray(a, np.int32)
            return L.minir_int_matrix(a.shape[0], a.shape[1], a.ctypes.data)
        a = np.asfortranarray(a, np.float64)
        return L.minir_real_matrix(a.shape[0], a.shape[1], a.ctypes.data)
    if np.issubdtype(a.dtype, np.integer):
        a = np.ascontiguousarray(a, np.int32)
        return L.minir_int(a.size, a.ctypes.data)
    a = np.ascontiguousarray(a, np.float64)
    return L.minir_real(a.size, a.ctypes.data)


def from_r(x):
    L = lib()
    t, n = L.minir_type(x), L.minir_length(x)
    if t == NILSXP:
        return None
    if t == VECSXP:
        items = [from_r(L.minir_elt(x, i)) for i in range(n)]
        names = [L.minir_name(x, i).decode() for i in range(n)]
        return dict(zip(names, items)) if any(names) else items
    ctype = {INTSXP: ctypes.c_int32, LGLSXP: ctypes.c_int32, REALSXP: ctypes.c_double}[t]
    buf = (ctype * max(n, 1)).from_address(L.minir_data(x))
    a = np.ctypeslib.as_array(buf)[:n].copy()
    nr, nc = L.minir_nrow(x), L.minir_ncol(x)
    if nr >= 0:
        a = a.reshape((nr, nc), order="F")
    return a


def call(name: str, *args):
    """.Call(name, args...) on the shim; raises RError with the Rf_error message."""
    L = lib()
    fp = ctypes.cast(getattr(L, name), ctypes.c_void_p).value
    rargs = (ctypes.c_void_p * len(args))(*[to_r(a) for a in args])
    depth = L.minir_protect_depth()
    r = L.minir_call(fp, len(args), rargs)
    if not r:
        raise RError(L.minir_error().decode())
    assert L.minir_protect_depth() == depth, f"{name}: PROTECT/UNPROTECT unbalanced"
    return from_r(r)
