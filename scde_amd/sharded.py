"""Gene-sharded scde.expression.difference: one process per GPU.

Genes are independent once the draw lists are fixed, so each rank takes a contiguous,
balanced gene range and runs the whole per-gene pipeline (unique tables, both groups'
bootstrap posteriors, ratio posterior, lb/mle/ub/ce/Z) on its own GPU with the seeding
of the *whole* call: with n.cores > 1 the reference splits the N genes into chunks whose
seeds are the chunk starts (R/functions.R:606-617); a shard carries its global offset so
every gene keeps its chunk's draw list (engine.hip ``seeding``).

The single exchange is a gather of the per-gene rows (lb, mle, ub, ce, Z) to rank 0,
where cZ = BH over all genes is computed (R/functions.R:5051).  Over RCCL this is one
``gather`` of a padded (ceil(N/world) x 5) fp64 tensor per rank -- 800 KB at 20k genes.

``compute`` is the per-shard function; the default is the HIP path.  Tests substitute a
CPU checker to run the distributed logic under ``gloo`` without a GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import api
from ._lib import DEParams, check, lib
from .models import model_matrix


def shard_range(ngenes: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced range [lo, hi) of rank ``rank`` among ``world``."""
    base, extra = divmod(ngenes, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def rank_device(rank: int | None = None) -> int:
    """The GPU this rank drives: LOCAL_RANK (one process per GPU of the node), or 0 for
    every rank when SCDE_SAME_DEVICE=1 (rehearsing the multi-rank path on a one-GPU box)."""
    import os
    if os.environ.get("SCDE_SAME_DEVICE") == "1":
        return 0
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    return int(rank or 0)


def device_shard(models, counts_shard, prior, codes, n_randomizations, n_cores, expectation, gene_offset,
                 ngenes_total, ctx=None):
    """Rows (lb, mle, ub, ce, Z) for one shard, computed on ``ctx``'s GPU (host counts in,
    host rows out: scde_expression_difference_host)."""
    ctx = ctx or api.default_context()
    mat = np.asfortranarray(counts_shard, dtype=np.int32)
    n, C = mat.shape
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    codes = np.ascontiguousarray(codes, np.int32)
    res = np.zeros((n, 5), order="F")
    if n == 0:
        return res
    params = DEParams(C, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, len(px),
                      int(n_randomizations), int(n_cores), int(gene_offset), int(ngenes_total),
                      float(expectation), api.get_rand_kind())
    check(lib().scde_expression_difference_host(ctx.handle, mat.ctypes.data_as(ctypes.c_void_p), n, n,
                                                ctypes.byref(params), res.ctypes.data_as(ctypes.c_void_p), None,
                                                None, None))
    return res


def expression_difference(models, counts, prior, groups, n_randomizations=150, n_cores=10, expectation=0.0,
                          compute=None, process_group=None, ctx=None):
    """Sharded scde.expression.difference over the ranks of ``torch.distributed``.

    Every rank passes the full inputs (or at least the same N and its own rows -- only
    rows [lo, hi) of ``counts`` are read).  Returns the N x 6 result table (lb, mle, ub,
    ce, Z, cZ as a pandas DataFrame) on rank 0 and None on the other ranks.

    With the default ``compute`` (the HIP path) each rank runs on its own GPU
    (``rank_device``: LOCAL_RANK), through ``ctx`` if given; the gather goes through the
    process group's backend (device tensors under nccl = RCCL, host tensors under gloo)
    and rank 0 computes cZ on its GPU.  A custom ``compute`` (the CPU checker in the
    tests) runs without any device.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(process_group)
    rank = dist.get_rank(process_group)
    on_device = dist.get_backend(process_group) == "nccl"
    import os
    if on_device and world > 1 and os.environ.get("SCDE_SAME_DEVICE") == "1":
        raise RuntimeError("SCDE_SAME_DEVICE=1 puts every rank on GPU 0, which RCCL does not allow: "
                           "rehearse the multi-rank path with the gloo backend")
    mat, genes = api._align_counts(models, counts)
    N = mat.shape[0]
    codes = api._groups_vector(models, groups)
    lo, hi = shard_range(N, world, rank)
    if compute is None:
        ctx = ctx or api.Context(rank_device(rank))
        rows = device_shard(models, mat[lo:hi], prior, codes, n_randomizations, n_cores, expectation, lo, N,
                            ctx=ctx)
    else:
        rows = compute(models, mat[lo:hi], prior, codes, n_randomizations, n_cores, expectation, lo, N)
    rows = np.asarray(rows, np.float64).reshape(hi - lo, 5)
    per = -(-N // world)
    buf = torch.zeros((per, 5), dtype=torch.float64)
    buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(rows))
    if on_device:
        buf = buf.to(torch.device("cuda", ctx.device if ctx is not None else rank_device(rank)))
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0, group=process_group)
    if rank != 0:
        return None
    rows_all = torch.cat([parts[r][: (lambda b: b[1] - b[0])(shard_range(N, world, r))] for r in range(world)])
    res = rows_all.cpu().numpy()
    if on_device and ctx is not None and N > 0:
        # the rows are on rank 0's GPU already (RCCL gather): BH over all genes there (scde_bh_cz_dev)
        z = rows_all[:, 4].contiguous().to(torch.device("cuda", ctx.device))
        cz = torch.empty_like(z)
        torch.cuda.current_stream(z.device).synchronize()
        api.bh_cz_device(ctx, z.data_ptr(), N, cz.data_ptr())
        ctx.synchronize()
        czh = cz.cpu().numpy()
    else:
        # gloo (host tensors): the library's host BH, no device tensor needed
        czh = api._bh(res[:, 4])
    return api._result_frame(np.asfortranarray(res), czh, genes)


__all__ = ["shard_range", "rank_device", "device_shard", "expression_difference"]
