"""Bootstrap diagnostics on the GPU box: kept-tile statistics and per-slot kernel times of one
config's DE call under a few context options (tile vs stretch bootstrap, skipping off).

  python tools/qdiag.py [config] [option=value ...]
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


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "3"
    extra = dict(kv.split("=") for kv in sys.argv[2:])
    cfg = bench.CONFIGS[cfgname]
    de = cfg["kind"] == "de"
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"], two_groups=de)
    ctx = api.Context(0)
    dc = api.DeviceCounts(ctx, counts)
    prior = expression_prior(models, dc, length_out=400, ctx=ctx)
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    codes = np.ascontiguousarray(groups, np.int32)
    NG, NC = counts.shape
    L = api.lib()
    P = api._p
    res = np.zeros((NG, 6), order="F")
    jp = np.zeros((NG, 401), order="F")
    modes = np.zeros((NG, NC), order="F")
    cellidx = np.arange(NC, dtype=np.int32)
    params = api.DEParams(NC, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px),
                          100, 1, 0, NG, 0.0, api.get_rand_kind(), 1)

    def run():
        if de:
            api.check(L.scde_expression_difference_dev(ctx.handle, dc.ptr, NG, NG, ctypes.byref(params), P(res), None,
                                                       None, None))
        else:
            api.check(L.scde_posteriors_dev(ctx.handle, dc.ptr, NG, NG, P(cellidx), NC, P(mm), lt, sq, P(px), 401,
                                            100, 1, 0, NG, 1, 0, None, None, None, 0, P(jp), P(modes), None))

    variants = [("tiles", {}), ("stretch", {"boot_tiles": 0}), ("noskip", {"boot_skip": 0})]
    if extra:
        variants = [("custom", {k: float(v) for k, v in extra.items()})]
    for name, opts in variants:
        for k, v in (("boot_skip", 1), ("boot_tiles", 1)):
            ctx.set_option(k, v)
        for k, v in opts.items():
            ctx.set_option(k, v)
        run()
        ctx.set_option("skip_stats", 1)
        ctx.reset_stats()
        run()
        st = {k: ctx.stat(k) for k in ("skip_slabs", "skip_kept", "skip_stretches", "skip_redo", "degen")}
        hist = [int(ctx.stat(f"tiles_{i}")) for i in range(29)]
        ctx.set_option("skip_stats", 0)
        ctx.reset_stats()
        for _ in range(3):  # host phases without the profiling events
            run()
        ctx.synchronize()
        host = {k: round(ctx.stat(f"host_{k}_ms") / 3, 3) for k in ("setup", "unique", "post", "tail")}
        ctx.set_profiling(True)
        ctx.reset_kernel_times()
        for _ in range(3):
            run()
        ctx.synchronize()
        kt = {k: round(v[0] / 3, 3) for k, v in ctx.kernel_times().items() if v[1]}
        ctx.set_profiling(False)
        kept = st["skip_kept"] / max(st["skip_stretches"], 1)
        print(f"{name}: kept {kept:.3f} rounds/slab {st['skip_redo'] / max(st['skip_slabs'], 1):.3f} "
              f"degen {st['degen']:.0f} ms/step {kt}", flush=True)
        if any(hist):
            print("   tiles/slab histogram:", {i: h for i, h in enumerate(hist) if h}, flush=True)
        print("   host ms/step by phase:", host, flush=True)


if __name__ == "__main__":
    main()
