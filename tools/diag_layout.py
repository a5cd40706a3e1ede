"""GPU diagnostic: the fused pipelined DE on the reversed-group layout after a config-3 host-pipeline
history on the same context (tests: test_gpu_configs + test_gpu_fullsize, then test_gpu_skip)."""
import ctypes
import math
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from scde_amd import api  # noqa: E402
from scde_amd._lib import DEParams, check, lib  # noqa: E402
from scde_amd.models import model_matrix  # noqa: E402
from scde_amd.prior import expression_prior  # noqa: E402

api.set_rand("glibc")
ctx = api.default_context()
hist = sys.argv[1] if len(sys.argv) > 1 else "pieces"
if hist != "none":
    cfg = bench.CONFIGS["3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    prior = expression_prior(models, counts, length_out=bench.LENGTH_OUT)
    mat = np.asfortranarray(counts, dtype=np.int32)
    N, C = mat.shape
    codes = np.ascontiguousarray(np.asarray(groups), np.int32)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px), 100, 1,
                      0, N, 0.0, api.get_rand_kind(), 1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    for pieces in ([4, 4, 3, 1, 8] if hist == "pieces" else [int(x) for x in hist.split(",")]):
        ctx.set_option("pieces", pieces)
        host = np.zeros((N, 6), order="F")
        check(lib().scde_expression_difference_host(ctx.handle, vp(mat), N, N, ctypes.byref(params), vp(host), None,
                                                    None, None))
    ctx.set_option("pieces", 4)
    print("history done", hist, flush=True)

models, counts, groups = bench.synthetic(8004, 150, 400)
groups = 1 - np.asarray(groups)
prior = expression_prior(models, counts, length_out=400)


def run(**opts):
    base = {"boot_tiles_cells": 0, "pipeline_mb": 32, "pieces": 4, "fuse_groups": 1}
    base.update(opts)
    for k, v in base.items():
        ctx.set_option(k, v)
    try:
        return api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=30,
                                              n_cores=1, return_posteriors=True)
    finally:
        ctx.set_option("boot_tiles_cells", 400)
        ctx.set_option("pipeline_mb", 32)
        ctx.set_option("pieces", 4)
        ctx.set_option("fuse_groups", 1)


ref = run(fuse_groups=0)
for name, o in [("fused", {}), ("fp3", dict(pipeline_mb=0, pieces=3)), ("fp3b", dict(pipeline_mb=0, pieces=3)),
                ("fp1", dict(pipeline_mb=0, pieces=1)), ("fp4", dict(pipeline_mb=0, pieces=4)),
                ("fp3_t64", dict(pipeline_mb=0, pieces=3, task_cols=64)),
                ("fp3_single", dict(pipeline_mb=0, pieces=3, tables_pair=0)),
                ("fp3_unfixed", dict(pipeline_mb=0, pieces=3, unique_fixed=0)),
                ("unfused_p3", dict(pipeline_mb=0, pieces=3, fuse_groups=0))]:
    got = run(**o)
    ctx.set_option("task_cols", 0)
    ctx.set_option("tables_pair", 1)
    ctx.set_option("unique_fixed", 1)
    d = [int(np.sum(got["joint.posteriors"][i] != ref["joint.posteriors"][i])) for i in range(2)]
    rows = [np.nonzero(np.any(got["joint.posteriors"][i] != ref["joint.posteriors"][i], axis=1))[0] for i in range(2)]
    print(name, "jp diffs", d, "rows", [len(r) for r in rows], "first", [r[:5].tolist() for r in rows], flush=True)
