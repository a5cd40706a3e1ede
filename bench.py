"""bench.py -- genes/sec for scde.expression.difference (401-pt grid, 100 randomizations).

Default workload (north_star's headline = BASELINE.json configs[2] = SURVEY.md §8(d) config 3):
synthetic 20,000 genes x 1,000 cells (500/500 groups), 400-point prior (G = 401 grid points),
n.randomizations = 100, reference seeding n.cores = 1.  One step = one scde.expression.difference
call as the R shim makes it: the host count matrix is uploaded, then unique-count tables,
per-cell NB/Poisson log-posterior tables, bootstrap joint posteriors for both groups, ratio
posterior + lb/mle/ub/ce/Z summary, BH cZ, and the result table lands in host memory
(SURVEY.md §8(d)'s wall time).  The same pass on counts already resident in HBM is reported
beside it as device_resident_genes_per_s.

--config 2: 20,000 genes x 200 cells (100/100), BASELINE configs[1].
--config 4: scde.posteriors(return.individual.posterior.modes = TRUE) on 30,000 genes x 2,000
cells (one group); one step returns jp (N x 401) and modes (N x 2000) to the host.
--config prior: scde.expression.prior on config 3's 20,000 x 1,000
counts, resident; one step = the whole prior (x, y, lp, grid.weight) to the host.
--config 5: pagoda.pathway.wPCA (BASELINE config 5) on a resident
synthetic varinfo of 20,000 genes x 3,000 cells; one step = every gene set's bwpca (10 starts),
its 10 random gene sets and the orientation / normalisation glue, results to the host.
--config 2b: config 2 with batch correction: two batch levels across
both groups; one step = batch posteriors over all 200 cells with each group's batch
composition, both group posteriors, the batch, group and 1601-column batch-adjusted ratio
posteriors with their summaries and BH (three result tables to the host).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU.  Configs
3 and 4 scale strongly by default (the fixed gene set split into contiguous shards, global
seeding offsets); --scaling weak gives every rank a full gene set.  The one exchange is a gather
of per-gene Z to rank 0 (RCCL) for the global BH adjustment, done there on the device.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

NBOOT = 100
LENGTH_OUT = 400
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TF = 78.6  # FP64 vector spec = FP32 vector 157.3 TF (MI355X_MICROARCH.md) / 2
FP64_FMA_MEASURED_TF = 67.0  # v_fma_f64 rate measured on this part (tools/micro/f64_rates.hip)
METRIC = "genes/sec for scde.expression.difference (400-pt grid, 100 randomizations)"

CONFIGS = {
    "2": dict(genes=20000, cells=200, seed=2002, kind="de", cpu_sample=5000,
            workload="config2: synthetic 20000 genes x 200 cells (100/100), 401-pt grid, 100 bootstraps, "
                     "n.cores=1 seeding"),
    "3": dict(genes=20000, cells=1000, seed=2003, kind="de", cpu_sample=1000,
            workload="config3: synthetic 20000 genes x 1000 cells (500/500), 401-pt grid, 100 bootstraps, "
                     "n.cores=1 seeding"),
    "4": dict(genes=30000, cells=2000, seed=2004, kind="posteriors", cpu_sample=100,
            workload="config4: scde.posteriors, synthetic 30000 genes x 2000 cells (one group), 401-pt grid, "
                     "100 bootstraps, return.individual.posterior.modes, n.cores=1 seeding"),
    "2b": dict(genes=20000, cells=200, seed=2002, kind="de_batch", cpu_sample=1500, nbatch=2,
               workload="config2b: batch-corrected scde.expression.difference, synthetic 20000 genes x 200 cells "
                        "(100/100 groups, 2 batch levels), 401-pt grid, 100 bootstraps, n.cores=1 seeding"),
}
CONFIGS["prior"] = dict(genes=20000, cells=1000, seed=2003, kind="prior", cpu_sample=20000,
                        workload="prior: scde.expression.prior, synthetic 20000 genes x 1000 cells (config 3 counts), "
                                 "length.out 400, max.quantile 1")
CONFIGS["5"] = dict(genes=20000, cells=3000, seed=2005, kind="wpca", nsets=200, cpu_sample=4,
                    workload="config5: pagoda.pathway.wPCA on a synthetic varinfo of 20000 genes x 3000 cells, "
                             "200 gene sets (10-500 genes, log-uniform), n.components 2, n.randomizations 10, "
                             "n.starts 10, em.tol 1e-6, em.maxiter 25")
METRIC_PRIOR = "genes/sec for scde.expression.prior (length.out 400, 1000 cells)"
METRIC_WPCA = "gene sets/sec for pagoda.pathway.wPCA (n.components 2, 10 randomizations, 10 starts, 3000 cells)"
METRIC_BATCH = ("genes/sec for batch-corrected scde.expression.difference (400-pt grid, 100 randomizations, "
                "2 batches)")


def synthetic_batch(seed: int, ncells: int, nbatch: int):
    """Batch labels for the batch config: PCG64(seed + 7), uniform over nbatch levels, so
    each group spans every batch."""
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    return np.array(["b%d" % k for k in rng.integers(0, nbatch, ncells)])


def synthetic(seed: int, ngenes: int, ncells: int, two_groups: bool = True):
    """SURVEY.md §8(d) generator: o.ifm-resampled models, log-FPM ~ N(2.5, 2), 10% DE genes,
    NB/Poisson-mixture counts with the models' own dropout curve."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "esmef500.npz"), allow_pickle=False)
    from scde_amd.models import MODEL_COLUMNS
    base = g["models"]
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = rng.integers(0, base.shape[0], ncells)
    mm = base[rows]
    models = {c: mm[:, j] for j, c in enumerate(MODEL_COLUMNS) if not np.all(np.isnan(mm[:, j]))}
    groups = np.repeat([0, 1], ncells // 2).astype(np.int32) if two_groups else np.zeros(ncells, np.int32)
    m = rng.normal(2.5, 2.0, ngenes)
    shift = np.where(rng.random(ngenes) < 0.1, rng.normal(0, 1.5, ngenes), 0.0)
    M = m[:, None] + shift[:, None] * groups[None, :]
    pfail = 1.0 / (1.0 + np.exp(models["conc.b"][None, :] + models["conc.a"][None, :] * M))
    mu = np.exp(models["corr.b"][None, :] + models["corr.a"][None, :] * M)
    theta = models["corr.theta"][None, :]
    nb = rng.negative_binomial(theta, theta / (theta + mu))
    pois = rng.poisson(np.exp(models["fail.r"])[None, :], size=M.shape)
    counts = np.where(rng.random(M.shape) < pfail, pois, nb).astype(np.int32)
    return models, np.asfortranarray(counts), groups


def dominant_kernel_bytes(ngenes, cells_per_group):
    """SURVEY.md §8(d) algorithmic bytes for one bootstrap launch (one group): each gene reads
    each cell's posterior column once (8G B) + its count index (4 B) and writes one jp row."""
    G = LENGTH_OUT + 1
    return ngenes * (cells_per_group * (4 + 8 * G) + 8 * G)


BOOT_STAGES = {0: "bootstrap stage (k_stretch_mask + k_boot2 + redo pass + k_sum_partials)",
               1: "bootstrap stage (k_boot_gene gene blocks + k_boot_tiles list pass + k_boot2_list fallback + "
                  "k_sum_partials)",
               3: "bootstrap stage (general k_boot)"}


def profiled_traffic(config: str, member=None, last=None):
    """HBM-side bytes per stage of the measured kernels from the newest committed rocprofv3
    summary of this config (profiles/rNN_config<C>_summary.json, written by tools/profile.sh +
    tools/pmc_summary.py from separate --pmc passes of this same command; FETCH_SIZE x2 per
    MI355X_MICROARCH.md).  `member(name)` picks the stage's kernels (default: the bootstrap
    stage), `last(name)` the kernel that ends one stage (one launch per stage); bytes and
    durations are summed over the stage's kernels and divided by the number of stages."""
    member = member or stage_kernel
    last = last or stage_last
    d = os.path.join(ROOT, "profiles")
    if not os.path.isdir(d):
        return None
    tag = f"_config{config}_summary.json"
    cands = sorted(f for f in os.listdir(d) if f.endswith(tag))
    if not cands:
        return None
    with open(os.path.join(d, cands[-1])) as f:
        ks = json.load(f)["kernels"]
    stage = {k: v for k, v in ks.items() if member(k)}
    n = max((v.get("calls") or 0 for k, v in ks.items() if last(k)), default=0)
    if not stage or not n:
        return None
    if any(v.get("traffic_bytes") is None for v in stage.values()):
        return None
    out = {"file": "profiles/" + cands[-1], "kernel": " + ".join(sorted(stage)),
           "avg_ms": sum(v["avg_ms"] * v["calls"] for v in stage.values()) / n,
           "traffic_bytes": sum(v["traffic_bytes"] * v["calls"] for v in stage.values()) / n}
    if all(v.get("fp64_flops") is not None for v in stage.values()):
        # FP64 VALU flops per stage from the gfx950 instruction counters (tools/pmc_summary.py)
        out["fp64_flops"] = sum(v["fp64_flops"] * v["calls"] for v in stage.values()) / n
        out["fma_f64_insts"] = sum(v["SQ_INSTS_VALU_FMA_F64"] * v["calls"] for v in stage.values()) / n
    cyc = sum(v.get("SQ_WAVE_CYCLES", 0) * v["calls"] for v in stage.values())
    if cyc > 0:  # share of the stage's wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)
        out["wait_frac"] = sum(v.get("SQ_WAIT_ANY", 0) * v["calls"] for v in stage.values()) / cyc
    return out


def add_profile_fields(roof: dict, prof, stage_s=None):
    """traffic / counter-bytes fraction / wait share from a profiled_traffic() record, on the
    profile's own rocprofv3 stage time (the time base of `frac` too, so every fraction in the line
    can be recomputed from the committed profile); stage_s (seconds per stage, HIP events in this
    run), when given, adds the same bytes over that live time beside it."""
    if not prof:
        return
    roof["traffic"] = prof["traffic_bytes"]
    roof["traffic_source"] = f"{prof['file']} ({prof['kernel']}, rocprofv3 avg {prof['avg_ms']:.3f} ms per stage)"
    roof["rocprof_stage_ms"] = prof["avg_ms"]
    roof["counter_bytes_frac"] = prof["traffic_bytes"] / (prof["avg_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
    roof["time_base"] = "rocprofv3 kernel durations of the committed profile (stage = its kernels per stage)"
    if stage_s:
        roof["counter_bytes_frac_live"] = prof["traffic_bytes"] / stage_s / 1e9 / HBM_PEAK_GBS
    if prof.get("wait_frac") is not None:
        roof["wait_frac"] = prof["wait_frac"]


def stage_kernel(name: str) -> bool:
    """Kernels of the bootstrap stage (bench's 'boot' slot)."""
    return ((name.startswith("k_boot") and "exact" not in name) or name.startswith("k_stretch_mask")
            or name == "k_sum_partials")


def stage_last(name: str) -> bool:
    """The kernel that ends one stage (one per bootstrap launch)."""
    return name == "k_sum_partials"


def _cpu_chunk(job):
    """One mclapply-style worker: the oracle on a contiguous gene chunk with the global
    n.cores chunk seeds (gene_offset / ngenes_total), as scde.posteriors' forked workers.
    Returns (genes, start, end) wall-clock stamps of the compute."""
    cfg, models, sub, groups, prior, lo, hi, ncores, ntotal = job
    from oracle import oracle as O
    O.lib()
    t0 = time.time()
    sub = np.ascontiguousarray(sub)
    if cfg["kind"] == "de":
        O.scde_expression_difference(models, sub, prior["x"], prior["y"], groups, n_randomizations=NBOOT,
                                     n_cores=ncores, gene_offset=lo, ngenes_total=ntotal)
    elif cfg["kind"] == "de_batch":
        O.scde_expression_difference_batch(models, sub, prior["x"], prior["y"], groups, cfg["batch"],
                                           n_randomizations=NBOOT, n_cores=ncores, gene_offset=lo,
                                           ngenes_total=ntotal)
    else:
        O.scde_posteriors(models, sub, prior["x"], n_randomizations=NBOOT, return_individual_posterior_modes=True,
                          n_cores=ncores, gene_offset=lo, ngenes_total=ntotal)
    return hi - lo, t0, time.time()


def cpu_baseline_parallel(cfg, models, counts, groups, prior, sample_genes, workers):
    """The reference's CPU path is fork-parallel (mclapply over n.cores gene chunks): the oracle
    in `workers` worker processes on the first sample_genes genes.  The workers are spawned
    (fresh interpreters, no GPU state), so this runs after the GPU work; the wall time is from
    the first chunk's start to the last chunk's end (interpreter start-up excluded)."""
    import multiprocessing as mp
    n = min(sample_genes, counts.shape[0])
    bounds = np.linspace(0, n, workers + 1).astype(int)
    prior_h = {"x": np.asarray(prior["x"]), "y": np.asarray(prior["y"])}
    jobs = [(cfg, models, counts[int(bounds[i]):int(bounds[i + 1])], groups, prior_h, int(bounds[i]),
             int(bounds[i + 1]), workers, n) for i in range(workers) if bounds[i + 1] > bounds[i]]
    with mp.get_context("spawn").Pool(len(jobs)) as pool:
        res = pool.map(_cpu_chunk, jobs)
    done = sum(r[0] for r in res)
    dt = max(r[2] for r in res) - min(r[1] for r in res)
    return done / dt, dt


def cpu_baseline(cfg, models, counts, groups, prior, sample_genes):
    """The oracle (C restatement of the reference loops, 1 core) on a bounded gene sample."""
    from oracle import oracle as O
    sub = np.ascontiguousarray(counts[:sample_genes])
    t0 = time.perf_counter()
    if cfg["kind"] == "de":
        O.scde_expression_difference(models, sub, prior["x"], prior["y"], groups, n_randomizations=NBOOT, n_cores=1)
    elif cfg["kind"] == "de_batch":
        O.scde_expression_difference_batch(models, sub, prior["x"], prior["y"], groups, cfg["batch"],
                                           n_randomizations=NBOOT, n_cores=1)
    else:
        O.scde_posteriors(models, sub, prior["x"], n_randomizations=NBOOT, return_individual_posterior_modes=True,
                          n_cores=1)
    dt = time.perf_counter() - t0
    return sample_genes / dt, dt


def bench_prior(args, cfg, rank, world, device):
    """--config prior: scde.expression.prior on resident counts.  Roofline of the element
    pass that bins (k_prior_bin): it must read each count once (4 B per gene x cell)."""
    from scde_amd import api
    from scde_amd.prior import expression_prior
    NG, NC = cfg["genes"], cfg["cells"]
    models, counts, _ = synthetic(cfg["seed"] + rank, NG, NC)
    ctx = api.Context(device)
    dc = api.DeviceCounts(ctx, counts)
    for _ in range(args.warmup):
        prior = expression_prior(models, dc, length_out=LENGTH_OUT, ctx=ctx)
    ctx.set_profiling(True)
    ctx.reset_kernel_times()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        prior = expression_prior(models, dc, length_out=LENGTH_OUT, ctx=ctx)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    kt = ctx.kernel_times()
    bin_ms, bin_n = kt["prior_bin"]
    bin_s = bin_ms / max(bin_n, 1) / 1e3
    per_launch = 4 * NG * NC
    achieved = per_launch / bin_s / 1e9 if bin_n else None
    out = {"metric": METRIC_PRIOR, "value": NG * args.steps / dt, "unit": "genes/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": f"synthetic (PCG64 seed {cfg['seed']}; o.ifm-resampled models)",
           "config": {"workload": cfg["workload"], "genes_per_gpu": NG, "cells": NC, "length_out": LENGTH_OUT,
                      "parallelism": "single GPU"},
           "roofline": {"bound": "hbm", "kernel": "k_prior_bin (magnitudes, weights, binning)",
                        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": None,
                        "avg_launch_ms": bin_s * 1e3, "launches": bin_n, "algorithmic_bytes_per_launch": per_launch},
           "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]}}
    add_profile_fields(out["roofline"], profiled_traffic("prior", lambda k: "k_prior_bin" in k,
                                                         lambda k: "k_prior_bin" in k))
    cpu_sample = cfg["cpu_sample"] if args.cpu_sample is None else args.cpu_sample
    if rank == 0 and cpu_sample > 0:
        from oracle import prior as OP
        n = min(cpu_sample, NG)
        t1 = time.perf_counter()
        OP.expression_prior(models, counts[:n], LENGTH_OUT)
        secs = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": n / secs, "unit": "genes/s", "cores": 1, "kind": "port",
                               "sample": f"oracle numpy restatement (oracle/prior.py) on the first {n} genes, "
                                         f"{secs:.1f}s"}
    if rank == 0:
        print(json.dumps(out))
    dc.free()
    ctx.close()


def synthetic_varinfo(seed: int, ngenes: int, ncells: int, nsets: int):
    """A pagoda varinfo stand-in: low-rank structure in gene blocks plus noise, weights in
    (0, 1] with 15% near-zero (dropout-like); gene sets of log-uniform size 10..500, half
    of them drawn from one structured block."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nf = 8
    L = rng.normal(size=(ngenes, nf)) * (rng.uniform(size=(ngenes, 1)) < 0.3)
    R = rng.normal(size=(nf, ncells)) * np.linspace(2.0, 0.5, nf)[:, None]
    mat = L @ R
    mat += rng.normal(size=(ngenes, ncells))
    matw = rng.uniform(0.05, 1.0, size=(ngenes, ncells))
    matw[rng.uniform(size=(ngenes, ncells)) < 0.15] = 1e-3
    genes = [f"g{i}" for i in range(ngenes)]
    block = np.nonzero(L[:, 0] != 0)[0]
    sets = {}
    for k in range(nsets):
        size = int(round(10 * 50 ** rng.uniform()))
        pool = block if (k % 2 == 0 and len(block) >= size) else np.arange(ngenes)
        sets[f"SET:{k:05d}"] = [genes[i] for i in rng.choice(pool, size=size, replace=False)]
    return {"mat": mat, "matw": matw, "genes": genes, "batch": None}, sets


def bench_wpca(args, cfg, rank, world, device):
    """--config 5: pagoda.pathway.wPCA, every bwpca call batched on the device (wpca.hip).
    Roofline: FP64 VALU.  The starts of a problem share each loaded element on chip (5 per
    workgroup for npcs = 1), so the EM kernels are compute-bound; achieved = the reference
    formulation's flops (_wpca_work) / the EM launches' time."""
    from scde_amd import api
    from scde_amd import pagoda as PG
    NG, NC = cfg["genes"], cfg["cells"]
    vinfo, sets = synthetic_varinfo(cfg["seed"] + rank, NG, NC, cfg["nsets"])
    ctx = api.Context(device)
    pdev = PG.PagodaDevice(vinfo, ctx)
    kw = dict(n_components=2, n_randomizations=10, n_starts=10, seed=1, device=pdev)
    for _ in range(args.warmup):
        PG.pagoda_pathway_wPCA(None, sets, **kw)
    ctx.set_profiling(True)
    ctx.reset_kernel_times()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = PG.pagoda_pathway_wPCA(None, sets, **kw)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    kt = ctx.kernel_times()
    nsets = len(out)
    em_ms, em_n = kt["wpca_em"]
    # algorithmic work of one step's EM launches: replay the step's problems with iteration counts
    ctx.set_profiling(False)
    step_bytes, step_flops = _wpca_work(PG, pdev, sets)
    em_s_step = em_ms / args.steps / 1e3
    achieved = step_flops / em_s_step / 1e12 if em_n else None
    res = {"metric": METRIC_WPCA, "value": nsets * args.steps / dt, "unit": "gene sets/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": f"synthetic varinfo (PCG64 seed {cfg['seed']}): rank-8 gene-block structure + N(0,1) noise, "
                   f"uniform weights with 15% at 1e-3",
           "config": {"workload": cfg["workload"], "genes": NG, "cells": NC, "gene_sets": nsets,
                      "parallelism": "single GPU"},
           "roofline": {"bound": "fp64-valu", "kernel": "k_wpca_ms1 + k_wpca_em (EM iterations)",
                        "achieved": achieved, "peak": FP64_VALU_PEAK_TF, "unit": "TFLOP/s",
                        "frac": achieved / FP64_VALU_PEAK_TF if achieved else None, "traffic": None,
                        "em_ms_per_step": em_s_step * 1e3, "launches_per_step": em_n / args.steps,
                        "algorithmic_flops_per_step": step_flops,
                        "pass_bytes_per_step": step_bytes,
                        "pass_bytes_note": "16 B x cells x genes per EM pass per start (the reference's reads); "
                                           "starts share their columns on chip, so HBM sees a fraction"},
           "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]}}
    # per step: the step's EM launches (one k_wpca_final<1> closes each step's npcs = 1 batch)
    prof = profiled_traffic("5", lambda k: k.startswith("k_wpca_ms1") or k.startswith("k_wpca_em"),
                            lambda k: k.startswith("k_wpca_final<1"))
    add_profile_fields(res["roofline"], prof)
    cpu_sample = cfg["cpu_sample"] if args.cpu_sample is None else args.cpu_sample
    if rank == 0 and cpu_sample > 0:
        from oracle import wpca as W
        # sets near 40 genes keep the sample to ~10-30 s on one core
        names = sorted(sorted(sets), key=lambda k: abs(len(sets[k]) - 40))[:cpu_sample]
        sub = {k: sets[k] for k in names}
        mat, matw = _prepared_host(vinfo)
        t1 = time.perf_counter()
        W.pagoda_pathway_wPCA(mat, matw, vinfo["genes"], sub, n_components=2, n_randomizations=10, n_starts=10,
                              center=False, seed=1)
        secs = time.perf_counter() - t1
        sizes = [len(sets[k]) for k in names]
        # scale to the whole workload's mix by gene count (EM work grows with set size)
        mean_all = float(np.mean([len(v) for v in sets.values()]))
        rate = cpu_sample / secs * (np.mean(sizes) / mean_all)
        res["cpu_baseline"] = {"value": rate, "unit": "gene sets/s", "cores": 1, "kind": "port",
                               "sample": f"oracle C restatement (oracle/bwpca_oracle.c) + R glue on {cpu_sample} "
                                         f"gene sets of {sizes} genes ({secs:.1f}s), scaled by mean set size "
                                         f"{mean_all:.0f}"}
    if rank == 0:
        print(json.dumps(res))
    pdev.free()
    ctx.close()


def _prepared_host(vinfo):
    from scde_amd.pagoda import weighted_mat_center
    mat = weighted_mat_center(vinfo["mat"], vinfo["matw"], None)
    return mat, np.asarray(vinfo["matw"], dtype=np.float64)


def _wpca_work(PG, pdev, sets):
    """Replays one step's batch with iteration counts.  Per (problem, start) with d genes,
    n cells, npcs K and `it` EM iterations, the reference's loops (src/bwpca.cpp:221-294) do
    per element: the start's coefficient step (1 + 2K + 3K^2 flops), then per iteration the
    coefficient step, the eigenvector step (5K + 2(K-1)) and the fit (2K + 4):
    3K^2 + 11K + 3 flops.  Each pass reads the value and weight columns: 16 B per element."""
    orig = PG.WpcaBatch.run
    tot = [0.0, 0.0]

    def run(self, dev, **kw):
        kw["want_iterations"] = True
        res = orig(self, dev, **kw)
        for p, r in enumerate(res):
            K = min(self.npcs[p], self.d[p])
            el = float(dev.ncells) * self.d[p]
            its = r["iterations"].astype(np.float64)
            tot[0] += float(np.sum(1 + 2 * its)) * 16.0 * el
            tot[1] += float(np.sum((1 + 2 * K + 3 * K * K) + its * (3 * K * K + 11 * K + 3))) * el
        return res
    PG.WpcaBatch.run = run
    try:
        PG.pagoda_pathway_wPCA(None, sets, n_components=2, n_randomizations=10, n_starts=10, seed=1, device=pdev)
    finally:
        PG.WpcaBatch.run = orig
    return tot[0], tot[1]


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="3", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default=None, choices=["strong", "weak"],
                    help="multi-GPU: strong = one fixed gene set split over the ranks (configs 3/4 default), "
                         "weak = a full gene set per rank")
    ap.add_argument("--cpu-sample", type=int, default=None, help="genes timed on the CPU baseline (0 = skip)")
    ap.add_argument("--no-profile", action="store_true",
                    help="no HIP-event stage times and no counter step (rocprofv3 runs: tools/profile.sh)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the real path) or gloo (CPU gather; rehearsal with ranks sharing one GPU)")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="oracle worker processes for the parallel CPU baseline (0 = skip; the GPU box's share is 16)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="readiness study, one process: time rank 0's shard of a strong split over this many "
                         "ranks (no collective; not the metric)")
    ap.add_argument("--trace-host", action="store_true",
                    help="end with a second host-count pass (tools/tl_shard.sh: the traced last step is a host step)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="context option for a study run (scde_ctx_set_option); the defaults are the product")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    cpu_sample = cfg["cpu_sample"] if args.cpu_sample is None else args.cpu_sample

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # SCDE_SAME_DEVICE=1 puts every rank on GPU 0 (rehearsing the multi-rank path on a one-GPU box)
    device = 0 if os.environ.get("SCDE_SAME_DEVICE") == "1" else local_rank
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")

    from scde_amd import api
    from scde_amd.models import model_matrix
    from scde_amd.prior import expression_prior
    from scde_amd.sharded import shard_range

    if cfg["kind"] == "prior":
        return bench_prior(args, cfg, rank, world, device)
    if cfg["kind"] == "wpca":
        return bench_wpca(args, cfg, rank, world, device)
    de = cfg["kind"] in ("de", "de_batch")
    batched = cfg["kind"] == "de_batch"
    scaling = args.scaling or ("strong" if args.config in ("3", "4") else "weak")
    if scaling == "strong":
        # one data set of cfg genes, split by shard_range; global gene offsets keep the seeding
        NTOT = cfg["genes"]
        models, counts_all, groups = synthetic(cfg["seed"], NTOT, cfg["cells"], two_groups=de)
        g0, g1 = shard_range(NTOT, world, rank) if args.shard_of <= 1 else shard_range(NTOT, args.shard_of, 0)
        counts = np.asfortranarray(counts_all[g0:g1])
    else:
        NTOT = cfg["genes"] * world
        models, counts, groups = synthetic(cfg["seed"] + rank, cfg["genes"], cfg["cells"], two_groups=de)
        counts_all = counts
        g0 = rank * cfg["genes"]
    NG, NC = counts.shape
    if batched:
        cfg["batch"] = synthetic_batch(cfg["seed"], NC, cfg["nbatch"])
    zero_frac = float(np.mean(counts == 0))
    ctx = api.Context(device)
    for o in args.opt:
        k, v = o.split("=", 1)
        ctx.set_option(k, float(v))
    # the prior is an input of the measured path: computed once, on the GPU,
    # from the whole data set (so every rank of a strong-scaling run holds the same grid)
    dcp = api.DeviceCounts(ctx, counts_all)
    prior = expression_prior(models, dcp, length_out=LENGTH_OUT, ctx=ctx)
    dcp.free()
    del counts_all
    mm, lt, sq = model_matrix(models)
    px = np.ascontiguousarray(prior["x"], np.float64)
    py = np.ascontiguousarray(prior["y"], np.float64)
    codes = np.ascontiguousarray(groups, np.int32)
    G = len(px)
    L = api.lib()
    P = api._p
    counts_p = P(counts)
    if de:
        # one rank: cZ (BH) in the same call on device; several: Z gathered to rank 0, BH there
        params = api.DEParams(NC, mm.ctypes.data, lt, sq, codes.ctypes.data, px.ctypes.data, py.ctypes.data, G,
                              NBOOT, 1, g0, NTOT, 0.0, api.get_rand_kind(), int(world == 1))
        res = np.zeros((NG, 6 if world == 1 else 5), order="F")
        if batched:
            blevels = sorted(set(cfg["batch"].tolist()))
            bcodes = np.ascontiguousarray([blevels.index(x) for x in cfg["batch"].tolist()], np.int32)
            res = np.zeros((NG, 18), order="F")  # batch.adjusted, results, batch.effect
    else:
        cellidx = np.arange(NC, dtype=np.int32)
        jp = np.zeros((NG, G), order="F")
        modes = np.zeros((NG, NC), order="F")

    def run(dev_counts=None):
        """One pass of the path.  dev_counts None: from the host count matrix (the timed
        value: counts uploaded, every kernel, table back on the host); else the counts
        already resident in HBM (the device-resident rate, reported beside it)."""
        if not de:
            if dev_counts is None:
                api.check(L.scde_posteriors_host(ctx.handle, counts_p, NG, NG, NC, P(cellidx), NC, P(mm), lt, sq,
                                                 P(px), G, NBOOT, 1, g0, NTOT, 1, 0, None, None, None, 0, P(jp),
                                                 P(modes), None))
            else:
                api.check(L.scde_posteriors_dev(ctx.handle, dev_counts, NG, NG, P(cellidx), NC, P(mm), lt, sq, P(px),
                                                G, NBOOT, 1, g0, NTOT, 1, 0, None, None, None, 0, P(jp), P(modes),
                                                None))
            return
        if batched:
            if dev_counts is None:
                api.check(L.scde_expression_difference_batch_host(ctx.handle, counts_p, NG, NG, ctypes.byref(params),
                                                                  P(mm), P(bcodes), len(blevels), P(res), None, None,
                                                                  None, None, None))
            else:
                api.check(L.scde_expression_difference_batch_dev(ctx.handle, dev_counts, NG, NG,
                                                                 ctypes.byref(params), P(mm), P(bcodes), len(blevels),
                                                                 P(res), None, None, None, None, None))
        elif dev_counts is None:
            api.check(L.scde_expression_difference_host(ctx.handle, counts_p, NG, NG, ctypes.byref(params), P(res),
                                                        None, None, None))
        else:
            api.check(L.scde_expression_difference_dev(ctx.handle, dev_counts, NG, NG, ctypes.byref(params), P(res),
                                                       None, None, None))
        if dist is not None:
            import torch
            # Z of every table (1 or 3) to rank 0; BH over all genes there, cZ to the host
            zcols = [4, 10, 16] if batched else [4]
            per = -(-NTOT // world) if scaling == "strong" else NG
            zt = torch.zeros((len(zcols), per), dtype=torch.float64)
            zt[:, :NG] = torch.from_numpy(np.ascontiguousarray(res[:, zcols].T))
            zt = zt.reshape(-1)
            if args.dist_backend == "nccl":
                zt = zt.cuda()
            gathered = [torch.empty_like(zt) for _ in range(world)] if rank == 0 else None
            dist.gather(zt, gathered, dst=0)
            if rank == 0:
                sizes = [(lambda b: b[1] - b[0])(shard_range(NTOT, world, r)) if scaling == "strong" else NG
                         for r in range(world)]
                zall = torch.cat([t.view(len(zcols), per)[:, :n] for t, n in zip(gathered, sizes)], 1).cuda()
                cz = torch.empty_like(zall)
                torch.cuda.current_stream().synchronize()
                for k in range(len(zcols)):
                    api.bh_cz_device(ctx, zall[k].data_ptr(), zall.shape[1], cz[k].data_ptr())
                ctx.synchronize()
                cz_host = cz.cpu()  # noqa: F841  (the tables' last columns, on the host)

    def barrier():
        ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def timed(dev_counts=None, steps=args.steps, profile=False, on_start=None):
        for _ in range(args.warmup):
            run(dev_counts)
        if on_start is not None:
            on_start()
        if profile:
            ctx.set_profiling(True)
        ctx.reset_kernel_times()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            run(dev_counts)
        barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            import torch
            tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        return dt

    # the CPU baselines run first (the reference's fork-parallel path and one core),
    # so the GPU passes come last in the run and a coarse external GPU-busy sampler sees them
    cpu_fields = {}
    par = None
    if rank == 0 and world == 1 and cpu_sample > 0 and args.cpu_workers > 0:
        par = cpu_baseline_parallel(cfg, models, counts, groups, prior, cpu_sample * args.cpu_workers,
                                    args.cpu_workers)
    if rank == 0 and world == 1 and cpu_sample > 0:
        what = ("batch + group posteriors, 3 ratio posteriors + summaries + BH" if batched else
                "both groups + ratio + summary + BH" if de else "posteriors + modes")
        gps, secs = cpu_baseline(cfg, models, counts, groups, prior, cpu_sample)
        cpu = cpu_model()
        single = {"value": gps, "unit": "genes/s", "cores": 1, "kind": "port", "cpu": cpu,
                  "sample": f"oracle C restatement, first {cpu_sample} genes of the same batch, {what}, {secs:.1f}s"}
        if par is not None:
            n = min(cpu_sample * args.cpu_workers, NG)
            cpu_fields["cpu_baseline"] = {"value": par[0], "unit": "genes/s", "cores": args.cpu_workers, "kind": "port",
                                   "cpu": cpu,
                                   "sample": f"oracle C restatement in {args.cpu_workers} worker processes "
                                             f"(mclapply-style gene chunks, n.cores={args.cpu_workers} seeding), "
                                             f"first {n} genes of the same batch, {what}, {par[1]:.1f}s wall"}
            cpu_fields["cpu_baseline_1core"] = single
        else:
            cpu_fields["cpu_baseline"] = single

    reallocs0 = [0.0]

    def count_from_here():  # after the warm-up calls (grow-only buffers reach their sizes there)
        ctx.reset_stats()
        reallocs0[0] = ctx.stat("buf_reallocs")

    # the metric: host-resident counts -> host-resident result table
    dt = timed(on_start=count_from_here)
    sync_stats = {"stream_syncs_per_step": ctx.stat("stream_syncs") / args.steps,
                  "arena_syncs_per_step": ctx.stat("arena_syncs") / args.steps,
                  "buf_reallocs_per_step": (ctx.stat("buf_reallocs") - reallocs0[0]) / args.steps,
                  "device_syncs_per_step": 0.0,
                  # host-count pieces: host ms per step waiting for uploads / building and launching
                  "piece_wait_ms_per_step": ctx.stat("piece_wait_ms") / args.steps,
                  "piece_host_ms_per_step": ctx.stat("piece_host_ms") / args.steps,
                  # host wall time of the call's phases (set-up, unique sets, posteriors enqueued,
                  # ratio + read-back incl. the final wait), ms per step
                  "host_phase_ms_per_step": {k: ctx.stat(f"host_{k}_ms") / args.steps
                                             for k in ("setup", "unique", "post", "tail")},
                  "upload_wake_ms_per_step": ctx.stat("upload_wake_ms") / args.steps,
                  "upload_first_ms_per_step": ctx.stat("upload_first_ms") / args.steps,
                  # 16-bit uploads: the issuing thread's ms per step waiting for the narrowing
                  # threads, issuing copies + widening kernels, waiting for ring slots to free
                  "u16_ms_per_step": {k: ctx.stat(f"u16_{k}_ms") / args.steps for k in ("wait", "issue", "free")}}
    # device-resident rate (counts already in HBM), product settings
    dc = api.DeviceCounts(ctx, counts)
    dt_dev = timed(dc.ptr)
    # per-stage HIP-event times from a separate pass with the two groups' posteriors one after
    # the other (option lanes = 1): concurrent lanes share the CUs, and a stage's time would then
    # include the other group's kernels.  tools/profile.sh's rocprof runs pass --opt lanes=1 too,
    # so its per-kernel averages describe the same launches.
    if not args.no_profile:
        ctx.set_option("lanes", 1)
        timed(dc.ptr, profile=True)
    kt = ctx.kernel_times()
    ctx.set_profiling(False)
    for o in args.opt:  # back to the run's settings
        k, v = o.split("=", 1)
        ctx.set_option(k, float(v))
    if not any(o.startswith("lanes=") for o in args.opt):
        ctx.set_option("lanes", 2)

    # arithmetic the bootstrap kernels issue in one step (one extra untimed step with the
    # context's counters on): FP64 lane FMAs of k_boot_tiles / k_boot2.  Not in --no-profile
    # runs (tools/profile.sh's rocprofv3 passes): the counters' atomics slow that step's
    # kernels 2x, which would skew rocprof's per-kernel averages
    step_fma = None
    stage_name = "bootstrap stage"
    if not args.no_profile:
        ctx.set_option("skip_stats", 1)
        ctx.reset_stats()
        run(dc.ptr)
        ctx.synchronize()
        step_fma = ctx.stat("boot_f64_fma")
        stage_name = BOOT_STAGES.get(int(ctx.stat("boot_path")), "bootstrap stage")
        ctx.set_option("skip_stats", 0)

    if args.trace_host:
        timed()
    total_genes = NTOT * args.steps
    value = total_genes / dt
    boot_ms, boot_n = kt["boot"]
    boot_avg_s = (boot_ms / max(boot_n, 1)) / 1e3
    boot_step_s = boot_ms / 1e3 / args.steps
    launches_per_step = boot_n / args.steps if boot_n else 0
    cpg = NC // 2 if de else NC
    # bootstrap launches of one step and their cells: (per group) + (all cells, per group) if batched
    launch_cells = ([cpg, cpg] if de else [NC]) + ([NC, NC] if batched else [])
    step_bytes = sum(dominant_kernel_bytes(NG, c) for c in launch_cells)
    per_launch_bytes = step_bytes / len(launch_cells)
    # the committed rocprofv3 profile of this config (N = 1 only: a shard's stage is another workload)
    prof = profiled_traffic(args.config) if args.shard_of <= 1 and world == 1 else None
    # live: the FMAs the FP64 bootstrap kernels issue (self-counted in one extra step) over the stage's
    # HIP-event time in this run's lanes = 1 pass
    live_tf = 2 * step_fma / boot_step_s / 1e12 if boot_n and step_fma else None
    live = {"stage_ms": boot_avg_s * 1e3 if boot_n else None, "launches_per_step": launches_per_step,
            "achieved": live_tf, "frac": live_tf / FP64_VALU_PEAK_TF if live_tf else None,
            "f64_fma_per_step": step_fma,
            "basis": "lane FMAs the FP64 bootstrap kernels issue (self-counted: computed grid points x slab boots x "
                     "entries, x2 flops) / the stage's HIP-event time in this run (lanes = 1 pass)"}
    if prof and prof.get("fp64_flops"):
        # One time base, the committed profile's: FP64 flops per stage from the gfx950 instruction
        # counters (SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64 x 64 lanes, FMA x2) over its rocprofv3 stage time
        achieved = prof["fp64_flops"] / (prof["avg_ms"] / 1e3) / 1e12
        basis = (f"FP64 VALU flops per stage from {prof['file']} (SQ_INSTS_VALU_{{FMA,ADD,MUL,TRANS}}_F64 x 64, "
                 f"FMA x2) / its rocprofv3 stage time (sum of the stage's kernel durations per stage)")
    else:
        achieved = live_tf or 0.0
        basis = live["basis"]
    roof = {"bound": "fp64-valu", "kernel": stage_name, "achieved": achieved, "peak": FP64_VALU_PEAK_TF,
            "unit": "TFLOP/s", "frac": achieved / FP64_VALU_PEAK_TF,
            "frac_of_measured_fma_rate": achieved / FP64_FMA_MEASURED_TF, "achieved_basis": basis,
            "traffic": None, "live": live}
    if prof:
        add_profile_fields(roof, prof)
        if prof.get("fp64_flops"):
            roof["fp64_flops_per_stage"] = prof["fp64_flops"]
            roof["fma_f64_wave_insts_per_stage"] = prof["fma_f64_insts"]
            if step_fma and launches_per_step:
                # the self-counted row FMAs against the counter's FMA lanes (rows are most of them)
                roof["self_counted_over_counter_fma"] = (step_fma / launches_per_step) / (64.0 * prof["fma_f64_insts"])
    # SURVEY.md §8(d)'s byte model describes the reference formulation (every cell's column read per
    # gene and boot); the kernels skip the baseline cells and the tiles the post-check proves
    # irrelevant, so this is work avoided, not a roofline (its "fraction" can exceed 1): reported
    # outside `roofline`
    ref_model = {"algorithmic_bytes_per_launch": per_launch_bytes,
                 "bytes_per_s_over_live_stage": step_bytes * args.steps / (boot_ms / 1e3) if boot_n else None,
                 "reference_fp64_adds_per_launch": NBOOT * sum(launch_cells) / len(launch_cells) * G * NG,
                 "note": "SURVEY.md 8(d)'s reference-formulation work per bootstrap launch; the kernels do not "
                         "perform it (sparse deltas over a shared baseline, post-checked tile skipping), so it "
                         "bounds nothing and is not a roofline fraction"}
    out = {
        "metric": (METRIC_BATCH if batched else METRIC) if de else "genes/sec for scde.posteriors with posterior modes "
                                                                   "(400-pt grid, 100 randomizations)",
        "value": value,
        "unit": "genes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (PCG64 seed {cfg['seed']}{'+rank' if scaling == 'weak' else ''}; o.ifm-resampled models; "
                f"zero fraction {zero_frac:.3f})",
        "config": {"workload": cfg["workload"], "genes_total": NTOT, "genes_per_gpu": NG, "cells": NC, "grid": G,
                   "n_randomizations": NBOOT, "parallelism": f"gene-shard x{world} ({scaling})",
                   "timed_region": "host counts -> upload -> unique tables, posteriors, ratio, summary, BH -> "
                                   "host result table"},
        **({"shard_of": args.shard_of,
            "shard_note": "one process timing rank 0's shard of a strong split; value = all genes / that time "
                          "(a projection, no collective, not the metric)"} if args.shard_of > 1 else {}),
        "device_resident_genes_per_s": NTOT * args.steps / dt_dev,
        "device_resident_ms_per_step": dt_dev / args.steps * 1e3,
        "roofline": roof,
        "reference_formulation": ref_model,
        "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kt.items() if v[1]},
        # in-library synchronisation over the timed steps: context-scoped
        # stream drains by grow-only buffer regrowth and pinned-arena wraps, and reallocations
        # (hipFree waits for the device); 0 in steady state
        "host_syncs": sync_stats,
        **cpu_fields,
    }
    dc.free()
    if rank == 0:
        print(json.dumps(out))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
