"""Per-phase cycle attribution of k_tables_reg on the GPU box (diagnostic build with
-DSCDE_KT_STAMP=1, loaded through SCDE_LIB): sums of s_memtime deltas per wave-column over
three config-3 DE calls, printed per column.

  SCDE_LIB=build_diag/libkts.so python tools/ktstamp.py [config]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from scde_amd import api  # noqa: E402
from scde_amd.models import model_matrix  # noqa: E402
from scde_amd.prior import expression_prior  # noqa: E402

PHASES = ["consts", "loop1 dnbinom", "max reduce", "loop2 exp", "sum+log", "loop3 log+store+tiles", "epilogue"]


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=True)
    ctx = api.Context(0)
    dc = api.DeviceCounts(ctx, counts)
    prior = expression_prior(models, dc, length_out=400, ctx=ctx)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    codes = np.ascontiguousarray(groups, np.int32)
    NG, NC = counts.shape
    L = api.lib()
    res = np.zeros((NG, 6), order="F")
    params = api.DEParams(NC, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px),
                          100, 1, 0, NG, 0.0, api.get_rand_kind(), 1)

    def run():
        api.check(L.scde_expression_difference_dev(ctx.handle, dc.ptr, NG, NG, ctypes.byref(params), api._p(res), None,
                                                   None, None))

    buf = (ctypes.c_ulonglong * 16)()
    run()
    ctx.synchronize()
    L.scde_diag_kt_stamps(buf, 1)
    for _ in range(3):
        run()
    ctx.synchronize()
    L.scde_diag_kt_stamps(buf, 1)
    ncol = max(buf[7], 1)
    tot = sum(buf[i] for i in range(7))
    print(f"columns {ncol}  cycles/column (s_memtime ticks) total {tot / ncol:.0f}")
    for i, n in enumerate(PHASES):
        print(f"  {n:24s} {buf[i] / ncol:9.0f}  {100 * buf[i] / max(tot, 1):5.1f}%")
    print("chunk events per column (waves whose ballot is non-zero):")
    for i, n in [(13, "chunks"), (12, "own-count point"), (11, "bad lanes"), (8, "bd0 series X"),
                 (9, "bd0 series n-x"), (14, "loop2 exp"), (10, "loop3 mixed|tiny"), (15, "loop3 tiny")]:
        print(f"  {n:24s} {buf[i] / ncol:7.3f}")


if __name__ == "__main__":
    main()
