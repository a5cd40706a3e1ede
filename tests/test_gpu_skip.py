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
the pair mode (two slabs per wave, two bound tiles each; pair_cells = 1) whose slabs needing more
take the four-tile list pass, or a multiplicity limit of 1 (tile_max_mult) so the call, with its tables set up
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


def _run(api, opts, models, counts, prior, groups, nrand, ncores):
    ctx = api.default_context()
    ctx.set_option("boot_skip", opts.get("boot_skip", 1))
    ctx.set_option("tile_max_mult", opts.get("tile_max_mult", 127))
    ctx.set_option("skip_slack", opts.get("skip_slack", math.nan))
    ctx.set_option("boot_tiles", opts.get("boot_tiles", 1))
    ctx.set_option("tile_groups", opts.get("tile_groups", 4))
    ctx.set_option("boot_tiles_cells", opts.get("boot_tiles_cells", 0))
    ctx.set_option("tile_order", opts.get("tile_order", 3))
    ctx.set_option("pair_cells", opts.get("pair_cells", 1000))
    ctx.set_option("gene_blocks", opts.get("gene_blocks", 1))
    ctx.set_option("gene_rows", opts.get("gene_rows", 4))
    ctx.set_option("gene_list_cap", opts.get("gene_list_cap", 0))
    ctx.set_option("gene_waves", opts.get("gene_waves", 0))
    ctx.set_option("unique_fixed", opts.get("unique_fixed", 1))
    ctx.set_option("lanes", opts.get("lanes", 2))
    ctx.set_option("pipeline_mb", opts.get("pipeline_mb", 32))
    ctx.set_option("pieces", opts.get("pieces", 4))
    ctx.set_option("defer_boot", opts.get("defer_boot", 0))
    ctx.set_option("upload_staged", opts.get("upload_staged", 0))
    ctx.set_option("lane_thread", opts.get("lane_thread", 0))
    ctx.set_option("interleave", opts.get("interleave", 1))
    ctx.set_option("rest_thread", opts.get("rest_thread", 1))
    ctx.set_option("boot_chunks", opts.get("boot_chunks", 1))
    ctx.set_option("fuse_groups", opts.get("fuse_groups", 0))
    ctx.set_option("tables_pair", opts.get("tables_pair", 1))
    ctx.set_option("tables_nt", opts.get("tables_nt", 2))
    ctx.set_option("lane_prio", opts.get("lane_prio", 0))
    ctx.set_option("task_cols", opts.get("task_cols", 0))
    ctx.set_option("boot2_rows", opts.get("boot2_rows", 0))
    ctx.set_option("ell_chunks", opts.get("ell_chunks", 1))
    ctx.set_option("gene_direct", opts.get("gene_direct", 1))
    ctx.set_option("skip_stats", 1)
    ctx.reset_stats()
    api.set_rand("glibc")
    try:
        out = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=nrand,
                                             n_cores=ncores, return_posteriors=True)
        stats = {k: ctx.stat(k) for k in ("skip_slabs", "skip_kept", "skip_stretches", "skip_redo", "boot_path",
                                          "pair_redo")}
    finally:
        ctx.set_option("tile_max_mult", 127)
        ctx.set_option("boot_skip", 1)
        ctx.set_option("skip_slack", math.nan)
        ctx.set_option("boot_tiles", 1)
        ctx.set_option("tile_groups", 4)
        ctx.set_option("boot_tiles_cells", 400)
        ctx.set_option("tile_order", 3)
        ctx.set_option("pair_cells", 1000)
        ctx.set_option("gene_blocks", 1)
        ctx.set_option("gene_rows", 4)
        ctx.set_option("gene_list_cap", 0)
        ctx.set_option("gene_waves", 0)
        ctx.set_option("unique_fixed", 1)
        ctx.set_option("lanes", 2)
        ctx.set_option("pipeline_mb", 32)
        ctx.set_option("pieces", 4)
        ctx.set_option("defer_boot", 0)
        ctx.set_option("upload_staged", 0)
        ctx.set_option("lane_thread", 0)
        ctx.set_option("interleave", 1)
        ctx.set_option("rest_thread", 1)
        ctx.set_option("boot_chunks", 1)
        ctx.set_option("fuse_groups", 0)
        ctx.set_option("tables_pair", 1)
        ctx.set_option("tables_nt", 2)
        ctx.set_option("lane_prio", 0)
        ctx.set_option("task_cols", 0)
        ctx.set_option("boot2_rows", 0)
        ctx.set_option("ell_chunks", 1)
        ctx.set_option("gene_direct", 1)
        ctx.set_option("skip_stats", 0)
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
        "tiles-slab-waves": {"gene_blocks": 0},
        "tiles-slab-waves-redo": {"gene_blocks": 0, "tile_groups": 2},
        "gene-forced-list": {"gene_rows": 1},
        "gene-list-overflow": {"gene_rows": 1, "gene_list_cap": 40},
        # a cap that is not a multiple of the list pass's 4 waves per block (rounded down to 40)
        "gene-list-overflow-odd": {"gene_rows": 1, "gene_list_cap": 41},
        "gene-3waves": {"gene_waves": 3},
        "gene-4waves": {"gene_waves": 4},
        "gene-chunks": {"boot_chunks": 3},
        "tiles-unordered": {"tile_order": 0},
        "tiles-ascending": {"tile_order": 1},
        "tiles-descending": {"tile_order": 2},
        # the ELL rows built in cell chunks (two passes) and in chunks of at most 2
        "ell-chunked": {"ell_chunks": 0},
        "ell-chunks2": {"ell_chunks": 2},
        # every jp row through k_sum_partials (gene blocks write their genes' rows themselves by default)
        "gene-direct-off": {"gene_direct": 0},
        "unique-exact": {"unique_fixed": 0},
        # the two group posteriors fused into one (option fuse_groups) against the two-posterior paths
        "fused": {"fuse_groups": 1},
        "one-lane": {"lanes": 1, "fuse_groups": 0},
        "rest-inline": {"rest_thread": 0, "fuse_groups": 0},
        "fused-pipelined": {"pipeline_mb": 0, "pieces": 3, "fuse_groups": 1},
        "fused-pipelined-staged": {"pipeline_mb": 0, "pieces": 2, "upload_staged": 1, "fuse_groups": 1},
        "pipelined-pieces": {"pipeline_mb": 0, "pieces": 3, "fuse_groups": 0},
        "pipelined-one-lane": {"pipeline_mb": 0, "pieces": 1, "lanes": 1, "fuse_groups": 0},
        "pipelined-deferred": {"pipeline_mb": 0, "pieces": 3, "defer_boot": 1, "fuse_groups": 0},
        "pipelined-staged": {"pipeline_mb": 0, "pieces": 3, "upload_staged": 1, "fuse_groups": 0},
        # both groups in alternating pieces
        "pipelined-thread": {"pipeline_mb": 0, "pieces": 3, "lane_thread": 1, "fuse_groups": 0},
        "pipelined-thread-seq": {"pipeline_mb": 0, "pieces": 3, "lane_thread": 1, "interleave": 0, "fuse_groups": 0},
        "tiles-pairs": {"pair_cells": 1, "gene_blocks": 0},
        "tiles-pairs-redo": {"pair_cells": 1, "tile_groups": 2, "gene_blocks": 0},
        "tiles-mult-fallback": {"tile_max_mult": 1},
        "stretch": {"boot_tiles": 0},
        "stretch-forced-redo": {"boot_tiles": 0, "skip_slack": -45.0},
        # the stretch path on tile rows (k_boot2t, option boot2_rows), with forced redo slabs too
        "stretch-k_boot2t": {"boot_tiles": 0, "boot2_rows": 1},
        "stretch-k_boot2t-redo": {"boot_tiles": 0, "boot2_rows": 1, "skip_slack": -45.0},
        # the tables one column per wave, and in 64- and 16-column tasks
        "tables-single": {"tables_pair": 0},
        # the table rows as non-temporal stores (the default only above 256 MB of rows)
        "tables-nt": {"tables_nt": 1},
        "tables-nt-single": {"tables_nt": 1, "tables_pair": 0},
        # the peer lane at the highest stream priority, always and per call (these calls are small)
        "lane-prio-on": {"lane_prio": 1},
        "lane-prio-auto": {"lane_prio": 2},
        "tables-tasks64": {"task_cols": 64},
        "tables-tasks16": {"task_cols": 16},
    }
    got = {}
    for name, opts in runs.items():
        got[name], stats = _run(api, opts, models, counts, prior, groups, nrand, ncores)
        if name == "noskip":
            assert stats["skip_slabs"] == 0 and stats["boot_path"] == 0, stats
        elif name == "tiles-mult-fallback":  # plain k_boot2 on the tile path's columns, no skipping
            assert stats["boot_path"] == 0 and stats["skip_slabs"] == 0, stats
        elif name in ("tiles-forced-redo", "tiles-slab-waves-redo"):
            # 2 bound tiles (64 points): slabs needing more go to k_boot2 (gene blocks: through the
            # four-tile list pass, itself limited to 2)
            assert stats["boot_path"] == 1 and stats["skip_redo"] > 0, stats
        elif name == "gene-forced-list":  # gene blocks with one row per slab: the list pass finishes the rest
            assert stats["boot_path"] == 1 and stats["pair_redo"] > 0 and stats["skip_slabs"] > 0, stats
        elif name in ("gene-list-overflow", "gene-list-overflow-odd"):  # past 40 slabs: k_boot2 directly
            assert stats["boot_path"] == 1 and 0 < stats["pair_redo"] <= 80 and stats["skip_redo"] > 0, stats  # 40 per lane
        elif name == "tiles-pairs":
            # two slabs per wave, two bound tiles each: at these cell counts many slabs need more and
            # take the four-tile list pass
            assert stats["boot_path"] == 1 and stats["skip_slabs"] > 0 and stats["pair_redo"] > 0, stats
        elif name == "tiles-pairs-redo":  # the list pass limited to two tiles too: k_boot2 takes the rest
            assert stats["boot_path"] == 1 and stats["pair_redo"] > 0 and stats["skip_redo"] > 0, stats
        else:
            assert stats["skip_slabs"] > 0 and stats["skip_kept"] < stats["skip_stretches"], (name, stats)
            assert stats["boot_path"] == (0 if name.startswith("stretch") else 1), (name, stats)
        if name.endswith("forced-redo") or name == "stretch-k_boot2t-redo":
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
    for base, others in (("tiles", ("noskip", "tiles-forced-redo", "tiles-slab-waves", "tiles-slab-waves-redo",
                                    "gene-forced-list", "gene-list-overflow", "gene-list-overflow-odd", "gene-3waves", "gene-4waves", "gene-chunks",
                                    "tiles-unordered", "unique-exact", "fused", "one-lane", "rest-inline",
                                    "fused-pipelined", "fused-pipelined-staged", "pipelined-pieces",
                                    "pipelined-one-lane", "pipelined-deferred", "pipelined-staged", "pipelined-thread",
                                    "pipelined-thread-seq",
                                    "tiles-pairs",
                                    "tiles-pairs-redo", "tiles-mult-fallback", "stretch", "stretch-forced-redo",
                                    "stretch-k_boot2t", "stretch-k_boot2t-redo", "tables-single", "tables-tasks64",
                                    "tables-tasks16")),):
        for name in others:
            for i in range(2):
                np.testing.assert_array_equal(got[name]["joint.posteriors"][i], got[base]["joint.posteriors"][i])
            np.testing.assert_array_equal(got[name]["difference.posterior"].values,
                                          got[base]["difference.posterior"].values)
            for k in ("Z", "cZ"):
                np.testing.assert_array_equal(got[name]["results"][k].to_numpy(), got[base]["results"][k].to_numpy())


@pytest.mark.parametrize("layout", ["reversed", "mixed"])
def test_threaded_lane_group_layouts(api, layout):
    """The host-count pipeline with the second lane on its own thread (options lane_thread,
    interleave): with the groups' cells reversed (the second group's range first: both groups go up
    in alternating pieces) and with the groups' cells mixed (no separable ranges: the sequential
    upload), the table equals the unpipelined one bit for bit."""
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
    runs = {"lane-thread": {"pipeline_mb": 0, "pieces": 3, "lane_thread": 1},
            # fused groups: reversed = the second group's cells first (its rows lead the fused list);
            # mixed = no separable ranges (one upload range before the unique sets)
            "fused-pipelined": {"pipeline_mb": 0, "pieces": 3, "fuse_groups": 1},
            "fused": {"fuse_groups": 1}}
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
