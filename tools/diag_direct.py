"""Config-3 DE tables through the host and device-resident entries under context options
(GPU box): tools/diag_direct.py -> mismatch counts against the default host run."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from scde_amd import api  # noqa: E402
from scde_amd._lib import DEParams, check, lib  # noqa: E402
from scde_amd.models import model_matrix  # noqa: E402
from scde_amd.prior import expression_prior  # noqa: E402

cfg = bench.CONFIGS["3"]
models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
mat = np.asfortranarray(counts, dtype=np.int32)
N, C = mat.shape
codes = np.ascontiguousarray(np.asarray(groups), np.int32)
mm, lt, sq = model_matrix(models)
px = np.ascontiguousarray(prior["x"], np.float64)
py = np.ascontiguousarray(prior["y"], np.float64)
ctx = api.default_context()
params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px), 100, 1,
                  0, N, 0.0, api.get_rand_kind(), 1)
vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
dc = api.DeviceCounts(ctx, mat)


def run(mode, **opts):
    for k, v in opts.items():
        ctx.set_option(k, v)
    out = np.zeros((N, 6), order="F")
    try:
        if mode == "host":
            check(lib().scde_expression_difference_host(ctx.handle, vp(mat), N, N, ctypes.byref(params), vp(out),
                                                        None, None, None))
        else:
            check(lib().scde_expression_difference_dev(ctx.handle, dc.ptr, N, N, ctypes.byref(params), vp(out),
                                                       None, None, None))
    finally:
        ctx.set_option("lanes", 2)
        ctx.set_option("gene_direct", 1)
    return out


if "--prep" in sys.argv:  # the full-size test's calls first (api entry with posteriors, staged upload)
    api.set_rand("glibc")
    g = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=100, n_cores=16,
                                       return_posteriors=True)
    print("prep done", flush=True)
ref = run("host", gene_direct=0, lanes=1)
for mode, opts in (("host", {}), ("dev", {}), ("dev", {"lanes": 1}), ("dev", {"lanes": 1, "gene_direct": 0}),
                   ("dev", {"gene_direct": 0}), ("host", {"gene_direct": 0}), ("host", {"lanes": 1}),
                   ("dev", {"lanes": 1}), ("host", {})):
    o = run(mode, **opts)
    print(mode, opts, "mismatched rows", int((o != ref).any(axis=1).sum()), flush=True)
dc.free()
