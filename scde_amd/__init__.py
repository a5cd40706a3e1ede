"""scde_amd -- MI355X-native (gfx950) implementation of scde's Bayesian
differential-expression hot path (logBootPosterior / jpmatLogBoot / matSlideMult
behind scde.posteriors() and scde.expression.difference()).

The numeric work runs in ``libscde_hip.so`` (hand-written HIP kernels, C ABI in
``include/scde_hip.h``); this package is the host-side mirror of the R API.
"""
from .api import (Context, DeviceCounts, RatioPosterior, ScdeError, bh_cz, calculate_ratio_posterior,  # noqa: F401
                  expectation_column, jpmatLogBatchBoot, jpmatLogBoot, logBootBatchPosterior, logBootPosterior,
                  marginals, matSlideMult, quick_distribution_summary, ratio_columns, scde_expression_difference,
                  scde_posteriors, set_rand)
from .prior import expression_prior  # noqa: F401

__version__ = "0.1.0"
