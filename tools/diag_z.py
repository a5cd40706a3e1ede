import sys
sys.path.insert(0, ".")
import numpy as np
import bench
from oracle import oracle as O
from scde_amd import api
from scde_amd.prior import expression_prior
models, counts, groups = bench.synthetic(7003, 160, 1000)
prior = expression_prior(models, counts, length_out=400)
api.set_rand("glibc")
got = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=12, n_cores=3,
                                     return_posteriors=True)
ref = O.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=12, n_cores=3,
                                   return_posteriors=True)
zg = got["results"]["Z"].to_numpy(); zr = ref["results"]["Z"]
bad = np.nonzero(~np.isclose(zg, zr, rtol=1e-6, atol=1e-9))[0]
print("bad", bad, zg[bad], zr[bad])
rg = got["difference.posterior"].values; rr = ref["difference.posterior"]
for g in bad:
    a, b = rg[g], rr[g]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    print(g, "ratio max rel err", rel.max(), "at", rel.argmax(), "vals", a[rel.argmax()], b[rel.argmax()], "rowmax", b.max())
    diffv = O.ratio_grid(prior["x"])
    zi = int(np.argmin(np.abs(diffv - 0.0)))
    for name, r in (("gpu", a), ("ora", b)):
        rp = (r + 1e-15) / np.sum(r + 1e-15)
        gs = np.sum(rp[:zi]) if zi > 0 else rp[0]
        print("  ", name, "zi", zi, "gs", gs, "zv", rp[zi], "tail p sum", np.sum(r[:zi]))
    for i in range(2):
        ja, jb = got["joint.posteriors"][i][g], ref["joint.posteriors"][i][g]
        relj = np.abs(ja - jb) / np.maximum(np.abs(jb), 1e-300)
        print("   jp", i, "max rel", relj.max(), "at", relj.argmax(), ja[relj.argmax()], jb[relj.argmax()])
