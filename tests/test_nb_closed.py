"""The closed form of the NB log-pmf that the tables kernels (k_tables_lpc, tables_column_reg) evaluate per grid point (SCDE_NB_CLOSED,
kernels.hip k_col_consts / tables_column_reg), against the oracle's restatement of R nmath's
saddle-point dnbinom (src/jpmatLogBoot.cpp:174 calls Rf_dnbinom; oracle/scde_oracle.c
o_dnbinom_log): log dnbinom(x; size, p) = C(x, size) + size log p + x log q with q = 1 - p as
dbinom_raw forms it and C the per-column constant

    C = log(size / (size + x)) + S - lf / 2 - size (log size - log n) - x (log x - log n),
    n = size + x, S = stirlerr(n) - stirlerr(size) - stirlerr(x),
    lf = log(2 pi) + log(size) + log1p(-size / n),

i.e. dbinom_raw with bd0(y, n r) = y log(y / n) - y log r + n r - y summed over both terms
(p + q = 1).  The two forms agree to rounding; the bound checked here (absolute, log space) is
what DESIGN.md §4.0d states, far below the 1e-6 relative parity bar on the posteriors."""
import math

import numpy as np


def _closed(oracle, x, size, p):
    L = oracle.lib()
    q = 1.0 - p
    if x == 0:
        return size * math.log(p)
    n = x + size
    S = L.o_stirlerr(n) - L.o_stirlerr(size) - L.o_stirlerr(n - size)
    lf = math.log(2 * math.pi) + math.log(size) + math.log1p(-size / n)
    lp = math.log(size / (size + x))
    C = ((lp + S) - 0.5 * lf) - size * (math.log(size) - math.log(n)) - (n - size) * (math.log(n - size) - math.log(n))
    lq = math.log(q) if q > 0 else -math.inf
    return C + size * math.log(p) + x * lq


def test_closed_form_matches_saddle_point(oracle):
    rng = np.random.default_rng(20261017)
    worst = 0.0
    for _ in range(4000):
        size = float(np.exp(rng.uniform(np.log(0.01), np.log(1000.0))))  # MIN_THETA..MAX_THETA
        x = float(rng.integers(0, 5000) if rng.random() < 0.4 else rng.integers(0, 30))
        mu = float(np.exp(rng.uniform(-12.0, 12.0)))
        p = size / (size + mu)
        ref = oracle.dnbinom_log(x, size, p)
        got = _closed(oracle, x, size, p)
        if math.isinf(ref):
            assert got == ref
            continue
        worst = max(worst, abs(got - ref))
    assert worst < 5e-11, worst


def test_closed_form_grid_point_zero(oracle):
    # mu = 0 at the -inf grid point: p = 1, q = 0 -> log 1 = 0 for x = 0, -inf otherwise (dbinom_raw)
    for size in (0.5, 3.0, 250.0):
        assert _closed(oracle, 0.0, size, 1.0) == oracle.dnbinom_log(0.0, size, 1.0) == 0.0
        assert _closed(oracle, 4.0, size, 1.0) == oracle.dnbinom_log(4.0, size, 1.0) == -math.inf
