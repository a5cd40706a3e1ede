import sys, math
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import bench
from scde_amd import api
from scde_amd.prior import expression_prior
api.set_rand("glibc")
for seed, ng, nc, nr, ncores in [(8002, 300, 200, 100, 1), (8003, 120, 1000, 40, 3), (2004, 300, 2000, 100, 1)]:
    models, counts, groups = bench.synthetic(seed, ng, nc)
    prior = expression_prior(models, counts, length_out=400)
    outs = {}
    for name, opts in [("tiles", {}), ("pairs", {"pair_cells": 1})]:
        ctx = api.default_context()
        ctx.set_option("boot_tiles_cells", 0)
        ctx.set_option("pair_cells", opts.get("pair_cells", 1000))
        ctx.set_option("skip_stats", 1)
        ctx.reset_stats()
        api.set_rand("glibc")
        out = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nr,
                                             n_cores=ncores, return_posteriors=True)
        st = {k: ctx.stat(k) for k in ("skip_slabs", "skip_redo", "pair_redo", "boot_path")}
        st["hist"] = {i: ctx.stat("tiles_%d" % i) for i in range(0, 29) if ctx.stat("tiles_%d" % i)}
        outs[name] = out
        print(seed, nc, name, st, flush=True)
    same = all(np.array_equal(outs["tiles"]["joint.posteriors"][i], outs["pairs"]["joint.posteriors"][i]) for i in range(2))
    print("  identical jp:", same, flush=True)
