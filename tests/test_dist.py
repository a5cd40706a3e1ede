"""Gene sharding across ranks: CPU tests under gloo with the oracle as
the per-shard checker, and a GPU test of the device path's global-offset seeding.

The property: sharding is invisible -- for any world size, the gathered table (including
cZ, a global BH over all genes) equals the single-process result, with n.cores chunks
(and so bootstrap seeds) that straddle shard boundaries."""
import os
import socket

import numpy as np
import pytest

from conftest import assert_cz_close, assert_z_close, golden

NRAND = 12
NCORES = 7
NGENES = 90


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    g = golden("esmef500.npz")
    from oracle import oracle as O
    models = {c: g["models"][:, j] for j, c in enumerate(O.MODEL_COLUMNS) if not np.all(np.isnan(g["models"][:, j]))}
    counts = np.asfortranarray(g["counts"][:NGENES])
    prior = {"x": g["prior_x"], "y": g["prior_y"]}
    return models, counts, prior, g["groups"]


def oracle_shard(models, counts_shard, prior, codes, nrand, n_cores, expectation, lo, N, ctx=None):
    """Per-shard compute for the CPU tests: the oracle restatement on rows [lo, lo+n)."""
    from oracle import oracle as O
    r = O.scde_expression_difference(models, counts_shard, prior["x"], prior["y"], codes, n_randomizations=nrand,
                                     n_cores=n_cores, expectation=expectation, gene_offset=lo, ngenes_total=N)
    return np.column_stack([r[k] for k in ("lb", "mle", "ub", "ce", "Z")])


def _worker(rank, world, port, out_path, hip=False, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if hip and backend == "gloo":
        os.environ["SCDE_SAME_DEVICE"] = "1"  # every rank on the one GPU of the box
    import torch.distributed as dist
    if backend == "nccl":
        import torch
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from scde_amd import api, sharded
        models, counts, prior, groups = _inputs()
        if hip:
            api.set_rand("glibc")
        tab = sharded.expression_difference(models, counts, prior, list(groups), n_randomizations=NRAND,
                                            n_cores=NCORES, compute=None if hip else oracle_shard)
        if rank == 0:
            np.save(out_path, tab[["lb", "mle", "ub", "ce", "Z", "cZ"]].to_numpy())
        else:
            assert tab is None
    finally:
        dist.destroy_process_group()


def test_rank_device(monkeypatch):
    from scde_amd.sharded import rank_device
    monkeypatch.delenv("SCDE_SAME_DEVICE", raising=False)
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert rank_device(13) == 5
    monkeypatch.delenv("LOCAL_RANK")
    assert rank_device(3) == 3
    monkeypatch.setenv("SCDE_SAME_DEVICE", "1")
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert rank_device(13) == 0


def test_shard_range_partition():
    from scde_amd.sharded import shard_range
    for N in (0, 1, 7, 90, 20000, 20001):
        for world in (1, 2, 3, 8):
            rs = [shard_range(N, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def test_oracle_shards_compose(oracle):
    """Row ranges computed with global offsets concatenate to the unsharded oracle."""
    models, counts, prior, groups = _inputs()
    full = oracle_shard(models, counts, prior, groups, NRAND, NCORES, 0.0, 0, NGENES)
    parts = [oracle_shard(models, counts[lo:hi], prior, groups, NRAND, NCORES, 0.0, lo, NGENES)
             for lo, hi in ((0, 31), (31, 32), (32, NGENES))]
    np.testing.assert_array_equal(np.vstack(parts), full)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_matches_single_process(world, tmp_path, oracle):
    import torch.multiprocessing as mp
    out = str(tmp_path / "tab.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    from oracle import oracle as O
    models, counts, prior, groups = _inputs()
    ref = O.scde_expression_difference(models, counts, prior["x"], prior["y"], groups, n_randomizations=NRAND,
                                       n_cores=NCORES)
    want = np.column_stack([ref[k] for k in ("lb", "mle", "ub", "ce", "Z", "cZ")])
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_device_shards_match_unsharded():
    """The HIP path with gene_offset/ngenes_total: shards of one call reproduce it (lb/mle/ub/ce
    exactly, Z to the parity tolerance: a shard's unique-count set can differ from the whole
    call's, e.g. no zero count for a cell, which changes the bootstrap's summation order by
    ulps -- the reference's own chunking does the same)."""
    from scde_amd import api, sharded
    models, counts, prior, groups = _inputs()
    api.set_rand("glibc")
    codes = np.asarray(groups, np.int32)
    full = sharded.device_shard(models, counts, prior, codes, NRAND, NCORES, 0.0, 0, NGENES)
    parts = [sharded.device_shard(models, counts[lo:hi], prior, codes, NRAND, NCORES, 0.0, lo, NGENES)
             for lo, hi in ((0, 31), (31, 32), (32, NGENES))]
    sh = np.vstack(parts)
    np.testing.assert_array_equal(sh[:, :4], full[:, :4])
    assert_z_close(sh[:, 4], full[:, 4], what="shards Z vs unsharded")
    want = oracle_shard(models, counts, prior, codes, NRAND, NCORES, 0.0, 0, NGENES)
    for j in range(4):
        np.testing.assert_array_equal(full[:, j], want[:, j])
    assert_z_close(full[:, 4], want[:, 4], what="device shard Z vs oracle")


@pytest.mark.gpu
def test_gloo_hip_shards_match_single_process(tmp_path):
    """Two ranks, each running the HIP path on its shard (both on the box's one GPU), gather
    to rank 0 with cZ there: the table equals the single-process HIP call."""
    import torch.multiprocessing as mp
    from scde_amd import api
    out = str(tmp_path / "tab.npy")
    mp.spawn(_worker, args=(2, _free_port(), out, True), nprocs=2, join=True)
    got = np.load(out)
    models, counts, prior, groups = _inputs()
    api.set_rand("glibc")
    ref = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=NRAND,
                                         n_cores=NCORES)
    want = ref[["lb", "mle", "ub", "ce", "Z", "cZ"]].to_numpy()
    np.testing.assert_array_equal(got[:, :4], want[:, :4])
    assert_z_close(got[:, 4], want[:, 4], what="gloo HIP shards Z")
    assert_cz_close(got[:, 5], want[:, 5], got[:, 4], want[:, 4], what="gloo HIP shards cZ")


@pytest.mark.gpu
def test_nccl_single_rank_device_gather(tmp_path):
    """The RCCL branch of the sharded call (device tensors gathered under the nccl backend, cZ by
    the device BH on rank 0's GPU), run with one rank on the box's one GPU -- RCCL does not
    allow two ranks on one device, so the multi-rank RCCL gather runs only on an 8-GPU node.
    The table equals the single-process HIP call."""
    import torch.multiprocessing as mp
    from scde_amd import api
    out = str(tmp_path / "tab.npy")
    mp.spawn(_worker, args=(1, _free_port(), out, True, "nccl"), nprocs=1, join=True)
    got = np.load(out)
    models, counts, prior, groups = _inputs()
    api.set_rand("glibc")
    ref = api.scde_expression_difference(models, counts, prior, groups=list(groups), n_randomizations=NRAND,
                                         n_cores=NCORES)
    want = ref[["lb", "mle", "ub", "ce", "Z", "cZ"]].to_numpy()
    np.testing.assert_array_equal(got[:, :4], want[:, :4])
    assert_z_close(got[:, 4], want[:, 4], what="RCCL single-rank Z")
    assert_cz_close(got[:, 5], want[:, 5], got[:, 4], want[:, 4], what="RCCL single-rank cZ")
