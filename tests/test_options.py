"""The context options (include/scde_hip.h): at most 20, and the documented set is exactly the set
scde_ctx_set_option accepts (the measured-and-lost paths were removed with
their kernels and branches).  Source-level check, no GPU."""
import os
import re

from conftest import ROOT


def _implemented():
    src = open(os.path.join(ROOT, "scde_amd", "csrc", "engine.hip")).read()
    body = src[src.index("int scde_ctx_set_option("):src.index("int scde_ctx_get_stat(")]
    return set(re.findall(r'n == "([a-z0-9_]+)"', body))


def _documented():
    hdr = open(os.path.join(ROOT, "include", "scde_hip.h")).read()
    block = hdr[hdr.index("/* Options of a context"):hdr.index("(Removed in round 6")]
    return set(re.findall(r'^ \*   "([a-z0-9_]+)"', block, re.M))


def test_at_most_twenty_options():
    assert len(_implemented()) <= 20, sorted(_implemented())


def test_documented_options_are_the_implemented_ones():
    assert _documented() == _implemented()


def test_removed_options_are_gone():
    removed = {"fuse_groups", "boot2_rows", "piece_taper", "boot_chunks", "ell_chunks", "gene_waves", "gene3_cells",
               "lane_prio", "lane_thread", "interleave", "defer_boot", "upload_staged", "upload_threads", "pair_cells",
               "gene_blocks", "gene_direct", "rest_thread", "tables_pair", "task_cols", "ratio_window", "ratio_block"}
    assert not (removed & _implemented())
    kern = open(os.path.join(ROOT, "scde_amd", "csrc", "kernels.hip")).read()
    for k in ("k_boot2t", "k_tables_reg", "tables_cols_lean"):
        assert k + "<" not in kern and k + "(" not in kern, k
