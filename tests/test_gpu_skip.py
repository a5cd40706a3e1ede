"""Grid-stretch skipping in the bootstrap (k_stretch_mask + k_boot2 + redo launch).

The skipping is an optimisation that must not change results: a 64-point stretch is only
left out of a boot slab when a rigorous upper bound of its row values stays more than 51
below the exact row maximum (post-check), i.e. when every softmax term there falls under
the e^-50 cut that zeroes it anyway; any slab that fails the check is recomputed whole.
These tests run the same calls, for the bootstrap kernels (k_boot_tiles on 4 bounded 32-point
tiles, the default; k_boot2 with its 64-point stretch mask, boot_tiles = 0), with skipping on
(default), off (boot_skip = 0), and forced onto the second-chance paths so that the extra work
really happens (its count is read back and must be > 0): a negative heuristic slack
(skip_slack) that makes the masks drop stretches the post-check must reject, the tile kernel
limited to 2 bound tiles (tile_groups = 2) so slabs needing more go to k_boot2's fallback launch,
gene blocks limited to one row per slab (gene_rows = 1) whose slabs needing more take the
four-tile list pass, or a multiplicity limit of 1 (tile_max_mult) so the call, with its tables set up
for the tile path, runs plain k_boot2 instead (the "multiplicity above 127" fallback) -- and
compare every run with the oracle at the SURVEY §8(d) bar, and the runs with each other bit
for bit (the kernels share rows, maxima and tile-ordered sums).
"""
import math

import numpy as np
import pytest

from conftest import assert_cz_close, assert_posterior_close, assert_z_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def api():
    from scde_amd import api as A
    A.set_rand("glibc")
    return A


# every context option (include/scde_hip.h) with its default: _run sets the call's own values and
# restores these afterwards (the module shares the default context)
OPTION_DEFAULTS = {"boot_skip": 1, "tile_max_mult": 127, "skip_slack": math.nan, "boot_tiles": 1, "tile_groups": 4,
                   "boot_tiles_cells": 400, "tile_order": 3, "gene_rows": 4, "gene_list_cap": 0, "unique_fixed": 1,
                   "lanes": 2, "pipeline_mb": 32, "pieces": 5, "tables_nt": 2, "skip_stats": 0}


def _run(api, opts, models, counts, prior, groups, nrand, ncores):
    ctx = api.default_context()
    for k, v in OPTION_DEFAULTS.items():
        ctx.set_option(k, v)
    ctx.set_option("boot_tiles_cells", opts.get("boot_tiles_cells", 0))
    for k, v in opts.items():
        ctx.set_option(k, v)
    ctx.set_option("skip_stats", 1)
    ctx.reset_stats()
    api.set_rand("glibc")
    try:
        out = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nrand,
                                             n_cores=ncores, return_posteriors=True)
        stats = {k: ctx.stat(k) for k in ("skip_slabs", "skip_kept", "skip_stretches", "skip_redo", "boot_path",
                                          "pair_redo")}
    finally:
        for k, v in OPTION_DEFAULTS.items():
            ctx.set_option(k, v)
    return out, stats


@pytest.mark.parametrize("seed,ngenes,ncells,nrand,ncores", [(8002, 300, 200, 100, 1), (8003, 120, 1000, 40, 3)])
def test_skip_modes_match_oracle(api, oracle, seed, ngenes, ncells, nrand, ncores):
    import bench
    from scde_amd.prior import expression_prior
    models, counts, groups = bench.synthetic(seed, ngenes, ncells)
    prior = expression_prior(models, counts, length_out=400)
    ref = oracle.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=nrand,
                                            n_cores=ncores, return_posteriors=True)
    runs = {
        "tiles": {},
        "noskip": {"boot_skip": 0},
        "tiles-forced-redo": {"tile_groups": 2},
        "gene-forced-list": {"gene_rows": 1},
        "gene-list-overflow": {"gene_rows": 1, "gene_list_cap": 40},
        # a cap that is not a multiple of the list pass's 4 waves per block (rounded down to 40)
        "gene-list-overflow-odd": {"gene_rows": 1, "gene_list_cap": 41},
        "tiles-unordered": {"tile_order": 0},
        "tiles-ascending": {"tile_order": 1},
        "tiles-descending": {"tile_order": 2},
        "unique-exact": {"unique_fixed": 0},
        "one-lane": {"lanes": 1},
        "pipelined-pieces": {"pipeline_mb": 0, "pieces": 3},
        "pipelined-one-lane": {"pipeline_mb": 0, "pieces": 1, "lanes": 1},
        "tiles-mult-fallback": {"tile_max_mult": 1},
        "stretch": {"boot_tiles": 0},
        "stretch-forced-redo": {"boot_tiles": 0, "skip_slack": -45.0},
        # the table rows as non-temporal stores (the default only above 256 MB of rows)
        "tables-nt": {"tables_nt": 1},
    }
    got = {}
    for name, opts in runs.items():
        got[name], stats = _run(api, opts, models, counts, prior, groups, nrand, ncores)
        if name == "noskip":
            assert stats["skip_slabs"] == 0 and stats["boot_path"] == 0, stats
        elif name == "tiles-mult-fallback":  # plain k_boot2 on the tile path's columns, no skipping
            assert stats["boot_path"] == 0 and stats["skip_slabs"] == 0, stats
        elif name == "tiles-forced-redo":
            # 2 bound tiles (64 points): slabs needing more go through the list pass (itself limited
            # to 2) to k_boot2
            assert stats["boot_path"] == 1 and stats["skip_redo"] > 0, stats
        elif name == "gene-forced-list":  # gene blocks with one row per slab: the list pass finishes the rest
            assert stats["boot_path"] == 1 and stats["pair_redo"] > 0 and stats["skip_slabs"] > 0, stats
        elif name in ("gene-list-overflow", "gene-list-overflow-odd"):  # past 40 slabs: k_boot2 directly
            assert stats["boot_path"] == 1 and 0 < stats["pair_redo"] <= 80 and stats["skip_redo"] > 0, stats  # 40 per lane
        else:
            assert stats["skip_slabs"] > 0 and stats["skip_kept"] < stats["skip_stretches"], (name, stats)
            assert stats["boot_path"] == (0 if name.startswith("stretch") else 1), (name, stats)
        if name.endswith("forced-redo"):
            assert stats["skip_redo"] > 0, stats  # the second-chance path really adds work
        g = got[name]
        for i in range(2):
            assert_posterior_close(g["joint.posteriors"][i], ref["joint.posteriors"][i], what=f"{name} jp{i}")
        assert_posterior_close(g["difference.posterior"].values, ref["difference.posterior"], what=f"{name} ratio")
        res = g["results"]
        for k in ("lb", "mle", "ub", "ce"):
            np.testing.assert_array_equal(res[k].to_numpy(), ref["results"][k], err_msg=f"{name} {k}")
        assert_z_close(res["Z"].to_numpy(), ref["results"]["Z"], what=f"{name} Z")
        assert_cz_close(res["cZ"].to_numpy(), ref["results"]["cZ"], res["Z"].to_numpy(), ref["results"]["Z"],
                        what=f"{name} cZ")
    # skipping leaves out only terms the e^-50 cut zeroes anyway: the outputs are identical
    for base, others in (("tiles", tuple(n for n in runs if n != "tiles")),):
        for name in others:
            for i in range(2):
                np.testing.assert_array_equal(got[name]["joint.posteriors"][i], got[base]["joint.posteriors"][i])
            np.testing.assert_array_equal(got[name]["difference.posterior"].values,
                                          got[base]["difference.posterior"].values)
            for k in ("Z", "cZ"):
                np.testing.assert_array_equal(got[name]["results"][k].to_numpy(), got[base]["results"][k].to_numpy())


@pytest.mark.parametrize("layout", ["reversed", "mixed"])
def test_pipelined_group_layouts(api, layout):
    """The host-count pipeline (pieces of the first group's range, then the second group's): with
    the groups' cells reversed (the second group's range first) and with the groups' cells mixed
    (no separable ranges: the sequential upload), the table equals the unpipelined one bit for bit."""
    import bench
    from scde_amd.prior import expression_prior
    models, counts, groups = bench.synthetic(8004, 150, 400)
    groups = np.asarray(groups)
    if layout == "reversed":
        groups = 1 - groups
    else:
        groups = np.random.default_rng(5).permutation(groups)
    prior = expression_prior(models, counts, length_out=400)
    base, _ = _run(api, {}, models, counts, prior, groups, 30, 1)
    runs = {"pipelined": {"pipeline_mb": 0, "pieces": 3},
            "pipelined-one-lane": {"pipeline_mb": 0, "pieces": 2, "lanes": 1}}
    bad = []
    for name, opts in runs.items():
        got, _ = _run(api, opts, models, counts, prior, groups, 30, 1)
        for i in range(2):
            ne = int(np.sum(got["joint.posteriors"][i] != base["joint.posteriors"][i]))
            if ne:
                bad.append(f"{name} jp{i}: {ne} entries differ")
        for k in ("lb", "mle", "ub", "ce", "Z", "cZ"):
            if not np.array_equal(got["results"][k].to_numpy(), base["results"][k].to_numpy()):
                bad.append(f"{name} {k}")
    assert not bad, bad
