"""cProfile of one config-5 step (pagoda.pathway.wPCA) on the GPU box: where the host time goes."""
import cProfile
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pstats
import time

import bench
from scde_amd import api
from scde_amd import pagoda as PG

cfg = bench.CONFIGS["5"]
vinfo, sets = bench.synthetic_varinfo(cfg["seed"], cfg["genes"], cfg["cells"], cfg["nsets"])
ctx = api.Context(0)
pdev = PG.PagodaDevice(vinfo, ctx)
kw = dict(n_components=2, n_randomizations=10, n_starts=10, seed=1, device=pdev)
PG.pagoda_pathway_wPCA(None, sets, **kw)
ctx.synchronize()
t0 = time.perf_counter()
PG.pagoda_pathway_wPCA(None, sets, **kw)
ctx.synchronize()
print("step %.1f ms" % ((time.perf_counter() - t0) * 1e3))
pr = cProfile.Profile()
pr.enable()
PG.pagoda_pathway_wPCA(None, sets, **kw)
ctx.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
