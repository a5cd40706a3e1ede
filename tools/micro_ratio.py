"""Timing study of k_ratio_summary (run under rocprofv3 --kernel-trace): 20,000 genes x
401-point posteriors, ratio + summary, then ratio only (res = NULL)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scde_amd import _lib  # noqa: E402

N, G = 20000, 401
rng = np.random.default_rng(0)
x = np.arange(G)
mu1 = rng.uniform(50, 350, N)[:, None]
mu2 = mu1 + rng.normal(0, 20, N)[:, None]
p1 = np.exp(-0.5 * ((x - mu1) / 15) ** 2)
p2 = np.exp(-0.5 * ((x - mu2) / 15) ** 2)
p1 = np.asfortranarray(p1 / p1.sum(1, keepdims=True))
p2 = np.asfortranarray(p2 / p2.sum(1, keepdims=True))
py = np.ones(G) / G
m = 2 * G - 1
diffv = np.linspace(-8.7, 8.7, m)
zi = G - 1
L = _lib.lib()
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
res = np.zeros((N, 6), order="F")
for mode in ("summary", "ratio_only", "summary", "ratio_only"):
    _lib.check(L.scde_ratio_summary(P(p1), P(p2), N, G, P(py), P(diffv), zi, None,
                                    P(res) if mode == "summary" else None))
    print(mode, "done", flush=True)
