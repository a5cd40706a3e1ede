"""Where the host-buffer scde.expression.difference call spends its time (GPU box).

Times, on config 3 (20k x 1000): the API's input checks, the counts allocation + upload,
the device call, and the result-frame build, each over a few repeats.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from scde_amd import api  # noqa: E402
from scde_amd.prior import expression_prior  # noqa: E402


def t(fn, n=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        r = fn()
    return (time.perf_counter() - t0) / n * 1e3, r


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "3"]
    models, counts, groups = bench.synthetic(cfg["seed"], cfg["genes"], cfg["cells"])
    ctx = api.Context(0)
    dc = api.DeviceCounts(ctx, counts)
    prior = expression_prior(models, dc, length_out=400, ctx=ctx)
    dc.free()
    ms, _ = t(lambda: api._align_counts(models, counts))
    print(f"align_counts {ms:.2f} ms")

    def up():
        d = api.DeviceCounts(ctx, counts)
        ctx.synchronize()
        d.free()
    ms, _ = t(up)
    print(f"alloc+h2d+free {ms:.2f} ms ({counts.nbytes / 1e6:.0f} MB)")
    kw = dict(groups=list(groups), n_randomizations=100, n_cores=1, ctx=ctx)
    ms, _ = t(lambda: api.scde_expression_difference(models, counts, prior, **kw))
    print(f"host api call {ms:.2f} ms")
    ms, _ = t(lambda: api._result_frame(np.zeros((counts.shape[0], 5)), np.zeros(counts.shape[0]), None))
    print(f"result frame {ms:.2f} ms")
    ctx.close()


if __name__ == "__main__":
    main()
