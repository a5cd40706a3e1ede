/*
 * scde_hip.h -- C ABI of the MI355X-native scde differential-expression path.
 *
 * Two layers:
 *
 *  1. Drop-in replacements for the five native entry points the reference
 *     resolves by name through `.Call(..., PACKAGE = "scde")`
 *     (NAMESPACE:29 useDynLib(scde); no R_registerRoutines).  Arguments are
 *     the R objects the R glue passes, flattened to plain pointers:
 *     matrices are R column-major, list-of-int-vectors become (values,
 *     offsets[n+1]).  Host pointers in, host pointers out; the GPU work is
 *     internal.  The `.Call` shim a maintainer would add is in INTEGRATION.md.
 *
 *  2. The device-resident pipeline (what bench.py times): counts stay in HBM,
 *     one call runs scde.expression.difference for one batch of genes.
 *
 * Every function returns 0 on success or a nonzero SCDE_E* code; the message
 * is available from scde_last_error() (thread-local).  Errors are never
 * silently replaced by a CPU fallback: there is none.
 */
#ifndef SCDE_HIP_H
#define SCDE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCDE_OK 0
#define SCDE_EARG 1   /* invalid argument / shape */
#define SCDE_EHIP 2   /* HIP runtime error (no device, launch failure, OOM) */
#define SCDE_EINTERNAL 3
#define SCDE_EFORK 4  /* a GPU entry in a process forked after this library initialised HIP
                         in its parent (R's mclapply after an n.cores = 1 call): the child
                         cannot use the inherited runtime; nothing was run */

const char* scde_last_error(void);
int scde_version(void); /* 100 * major + minor */

/* Which C-library rand() the bootstrap draws reproduce (the reference calls the
 * platform's srand()/rand(), src/jpmatLogBoot.cpp:221,256):
 *   SCDE_RAND_GLIBC  glibc TYPE_3 (Linux; the default)
 *   SCDE_RAND_DARWIN Darwin/BSD libc Park-Miller (macOS; reproduces the vignette)
 * Process-wide default for layer 1 and scde_posteriors_dev; also read once from
 * the environment variable SCDE_RAND=glibc|darwin. */
#define SCDE_RAND_GLIBC 0
#define SCDE_RAND_DARWIN 2
int scde_set_rand_kind(int kind);
int scde_get_rand_kind(void);

/* ---------------------------------------------------------------- layer 1 */

/* Replaces logBootPosterior  (src/jpmatLogBoot.cpp:100, decl src/jpmatLogBoot.h:8).
 *  models     ncells x 12 col-major (R `mm`, NaN where a column is absent)
 *  ucl_vals   concatenated Ucl list (unique counts per cell), ucl_off[ncells+1]
 *  counti     ngenes x ncells col-major, 0-based index into the cell's Ucl
 *  magnitudes ngrid natural-log magnitudes (marginals)
 *  outputs    jp    ngenes x ngrid col-major                   (always)
 *             modes ngenes x ncells col-major       (return_post in {1,3})
 *             post  ncells consecutive ngenes x ngrid col-major blocks (return_post in {2,3})
 */
int scde_logBootPosterior(const double* models, int ncells, const int* ucl_vals, const int64_t* ucl_off,
                          const int* counti, int ngenes, const double* magnitudes, int ngrid, int nboot, int seed,
                          int return_post, int local_theta, int square_logit_conc, int ensemble, double* jp,
                          double* modes, double* post);

/* Replaces logBootBatchPosterior  (src/jpmatLogBoot.cpp:343, decl .h:9).
 *  batch_vals/batch_off: BatchIL (0-based cell indices per batch level), nbatch levels
 *  composition: nbatch draws-per-boot counts (R `table(batch[ii])`).
 *  return_post 3 is not handled by the reference (falls through to jp only); same here. */
int scde_logBootBatchPosterior(const double* models, int ncells, const int* ucl_vals, const int64_t* ucl_off,
                               const int* counti, int ngenes, const double* magnitudes, int ngrid,
                               const int* batch_vals, const int64_t* batch_off, const int* composition, int nbatch,
                               int nboot, int seed, int return_post, int local_theta, int square_logit_conc,
                               double* jp, double* modes, double* post);

/* Replaces jpmatLogBoot  (src/jpmatLogBoot.cpp:11, decl .h:6).  mats: nmat pointers
 * to nrows x ncols col-major log-posterior matrices.  out: nrows x ncols col-major. */
int scde_jpmatLogBoot(const double* const* mats, int nmat, int nrows, int ncols, int nboot, int seed, double* out);

/* Replaces jpmatLogBatchBoot  (src/jpmatLogBoot.cpp:48, decl .h:7).  Matll flattened:
 * type k owns mats[type_off[k] .. type_off[k+1]); comp[k] draws per boot. */
int scde_jpmatLogBatchBoot(const double* const* mats, const int* type_off, const int* comp, int ntypes, int nrows,
                           int ncols, int nboot, int seed, double* out);

/* Replaces matSlideMult  (src/matSlideMult.cpp:5, decl src/matSlideMult.h:6).
 * m1, m2: nrows x ncols col-major; out: nrows x (2*ncols-1) col-major. */
int scde_matSlideMult(const double* m1, const double* m2, int nrows, int ncols, double* out);

/* calculate.ratio.posterior + quick.distribution.summary (R/functions.R:3491-3510,
 * 5039-5050) on host buffers.  prior_y may be NULL (skip.prior.adjustment).
 * diffv: 2n-1 column values (as.numeric(colnames)), zi: 0-based index of the
 * expectation column.  ratio (nrows x (2n-1) col-major) and res (nrows x 5
 * col-major: lb, mle, ub, ce, Z) may each be NULL. */
int scde_ratio_summary(const double* pmat1, const double* pmat2, int nrows, int n, const double* prior_y,
                       const double* diffv, int zi, double* ratio, double* res);

/* quick.distribution.summary of an existing ratio posterior (R/functions.R:5039-5050):
 * rpost nrows x m col-major (m odd, rows already normalised), diffv m values, zi the
 * expectation column.  res: nrows x 5 col-major (lb, mle, ub, ce, Z). */
int scde_distribution_summary(const double* rpost, int nrows, int m, const double* diffv, int zi, double* res);

/* BH-adjusted cZ = sign(Z) qnorm(p.adjust(pnorm(|Z|, lower=F), "BH"), lower=F)
 * (R/functions.R:5051).  Host-only. */
int scde_bh_cz(const double* z, int64_t n, double* cz);

/* ---------------------------------------------------------------- layer 2 */

typedef struct scde_ctx scde_ctx;

int scde_ctx_create(int device, scde_ctx** out);
void scde_ctx_destroy(scde_ctx* ctx);
int scde_ctx_synchronize(scde_ctx* ctx);
/* Per-kernel HIP-event timing on the context's stream (0 = off). */
int scde_ctx_set_profiling(scde_ctx* ctx, int on);
/* slot names: 0 tables, 1 boot, 2 ratio_summary, 3 unique, 4 other, 5 prior_stats,
 * 6 prior_bin, 7 prior_tail; ms totals and launch counts */
int scde_ctx_kernel_times(scde_ctx* ctx, double* ms, int64_t* launches, int nslots);
int scde_ctx_reset_kernel_times(scde_ctx* ctx);
/* Options of a context: 20, each the switch of a default path or a documented operating / test mode
 * (defaults are the product settings; the environment is read once, at context creation, for
 * SCDE_OPTIONS -- see scde_ctx_set_option).  Every one leaves the results unchanged unless noted.
 * Bootstrap paths:
 *   "boot_tiles"    1/0  the FP64 bootstrap on bounded 32-point tiles (k_boot_gene gene blocks, their
 *                   four-tile list pass k_boot_tiles; default 1) or k_boot2's 64-point stretches (0)
 *   "boot_tiles_cells"  the cell count from which the tile path is used (default 400; below: k_boot2's
 *                   64-point stretch mask -- config 2b's 200-cell batch posteriors: 8.2 ms of
 *                   bootstrap per step with it against 12.0 with gene blocks)
 *   "boot_skip"     1/0  grid-stretch / tile skipping in the bootstrap (default 1)
 *   "boot_nb"       boots per bootstrap slab (0 = automatic; a multiple of 4 in [4, 32])
 *   "tile_order"    0..3  the tile bootstrap takes the genes in order of their count sums,
 *                   so waves in flight share columns and tiles in L2: 1 ascending, 2 descending
 *                   (heaviest genes first: a shorter tail), 3 (default) descending in
 *                   scde.posteriors calls and in DE launches of at most 8,192 genes, ascending in
 *                   larger DE launches, 0 gene order
 * Test modes forcing the bootstrap's second-chance paths (each must still give the same bits):
 *   "skip_slack"    mask heuristic slack (NaN = default 20 + 0.15 C; negative: redo slabs)
 *   "tile_groups"   32-point tiles the list pass computes per slab, 1..4 (default 4; with 2, slabs
 *                   needing more go to k_boot2 whole)
 *   "tile_max_mult" the largest draw multiplicity the tile path takes (default 127, the int8 bound
 *                   operand; a call with a larger one runs plain k_boot2 on the same columns)
 *   "gene_rows"     1..4 rows per slab a gene block gives each slab at most (default 4; fewer:
 *                   the four-tile list pass takes the rest)
 *   "gene_list_cap" slabs the list pass takes at most (0 = 16384; beyond: k_boot2)
 *   "skip_stats"    1/0  count kept stretches and redo slabs (one host sync per launch)
 * Host pipeline:
 *   "lanes"         2/1  a DE call's second group runs on a peer context (its own streams and
 *                   workspace, same device) beside the first (default 2), or after it (1; bench's
 *                   per-stage timing pass and the rocprof runs use 1).  Memory: the peer holds a
 *                   second grow-only workspace (tables, deltas, slab partials, joint posterior:
 *                   about 2.3 GB at 20k genes x 500 cells per group), so two
 *                   lanes roughly double a DE call's device footprint; setting 1 releases the peer
 *   "pipeline_mb"   host-count DE / scde.posteriors calls whose matrix has at least this many MB
 *                   upload on a copy stream in column pieces that the kernels follow (default 32)
 *   "pieces"        pieces of that upload (the DE call's first group; the posteriors call's
 *                   selected cells), 1..8 (default 5)
 *   "upload_u16"    0..2  host-count ranges of 8 MB or more go up as 16-bit counts: narrowed by 4
 *                   host threads into a pinned ring, widened on the device, counts outside
 *                   [0, 65535] listed and patched in (half the PCIe bytes): 1 (default) in
 *                   scde_posteriors_host calls, 2 in every host entry, 0 none
 *   "modes_overlap" 1/0  scde.posteriors' read-backs run on a read-back thread beside the device
 *                   work (default 1): the modes piece by piece as each piece's tables finish, the
 *                   joint posterior in gene chunks of the bootstrap; 0: both after the bootstrap on
 *                   the main stream (rocprofv3 runs)
 *   "jp_chunks"     1..64 gene chunks of scde.posteriors' gene-block bootstrap (default 4, at most
 *                   one per 256 genes; with or without modes_overlap): each chunk finishes before
 *                   the next starts (chunks of <= 8192 genes run heaviest genes first, which shares
 *                   more columns in L2) and, with modes_overlap, its joint posterior rows are read
 *                   back while the next runs
 * Tables and other kernels:
 *   "unique_fixed"  1/0  build each call's unique count tables with one host sync (fixed
 *                   1024-word bitmaps per cell, counts below 65,536; a set with another count is
 *                   rebuilt with exact widths); default 1, 0 = the exact three-phase build
 *   "tables_nt"     0..2 the posterior-table rows as non-temporal stores: 0 never, 1 always, 2 when
 *                   the call's rows exceed 256 MB (default)
 *   "wpca_ms"       1/0  the multi-start npcs = 1 weighted-PCA kernel (default 1)
 * (Removed in round 6, each measured slower or equal and deleted with its kernels and branches:
 * fuse_groups, boot2_rows / k_boot2t, piece_taper, boot_chunks, ell_chunks, gene_waves /
 * gene3_cells, lane_prio, lane_thread, interleave, defer_boot, upload_staged, upload_threads,
 * pair_cells / gene_blocks (pair mode), gene_direct, rest_thread, tables_pair, task_cols,
 * ratio_window / ratio_block: fixed at their defaults.)
 * Statistics: "skip_slabs", "skip_stretches", "skip_kept", "skip_redo", "degen", "tiles_<i>"
 * (k_boot_tiles slabs computing i tiles), "pair_redo" (slabs the gene blocks left to the four-tile
 * list pass) (with skip_stats); "boot_f64_fma" (FP64 lane FMAs the
 * bootstrap kernels issued), also with skip_stats; "boot_path": the bootstrap kernel of the last
 * posterior (0 k_boot2, 1 k_boot_tiles / k_boot_gene, 3 the general k_boot); "stream_syncs",
 * "arena_syncs" (this context's and its peer's streams drained by a buffer regrowth / a pinned
 * arena wrap) and "buf_reallocs" (process-wide workspace reallocations, each a hipFree): 0 in
 * steady state. */
/* Options can also come from the environment: SCDE_OPTIONS="name=value,..." is applied to every
 * context as it is created (an unknown name fails the creation). */
int scde_ctx_set_option(scde_ctx* ctx, const char* name, double value);
int scde_ctx_get_stat(scde_ctx* ctx, const char* name, double* value);
/* Test hook: make the next `count` failures happen at fault point `where` ("u16_slot": the second
 * slot of a 16-bit host-count upload fails as if its copy had) -- the error paths' recovery is
 * tested through it (tests/test_gpu_fullsize.py).  "handoff_spin" (count = shader clocks, 0 off):
 * every later call queues a one-wave spin kernel of that length on a stream after each of its
 * cross-stream waits (so the work it produces next starts late) and before each event another
 * stream or thread waits on (each piece's tables and unique sets, the pieces' uploads, the 16-bit
 * ring, the aux set-up, the peer lane's start and finish, the read-back thread's events): a
 * consumer that misses its wait reads unwritten data every time (tests/test_gpu_ordering.py; stat
 * "handoff_spins" counts them).  "skip_lane_join": the next `count` DE calls leave out the main
 * stream's wait for the peer lane -- the ordering tests' negative control.  Not for production
 * use. */
int scde_ctx_inject_fault(scde_ctx* ctx, const char* where, int count);
int scde_ctx_reset_stats(scde_ctx* ctx);

/* device buffers owned by the context's allocator */
int scde_dev_alloc(scde_ctx* ctx, int64_t bytes, void** dptr);
int scde_dev_free(scde_ctx* ctx, void* dptr);
int scde_h2d(scde_ctx* ctx, void* dst, const void* src, int64_t bytes);
int scde_d2h(scde_ctx* ctx, void* dst, const void* src, int64_t bytes);

/* The same BH cZ on device buffers (z_dev, cz_dev: n doubles in HBM), on the context's
 * stream: pnorm, stable descending radix sort, cummin scan, qnorm.  For the gathered Z
 * of a sharded call (R/functions.R:5051). */
int scde_bh_cz_dev(scde_ctx* ctx, const double* z_dev, int64_t n, double* cz_dev);

typedef struct scde_de_params {
  int ncells;              /* cells (columns of counts) */
  const double* models;    /* host, ncells x 12 col-major (NaN where absent; corr.a clamp applied inside) */
  int local_theta;         /* "corr.ltheta.b" present */
  int square_logit_conc;   /* "conc.a2" present */
  const int* groups;       /* host, per cell: 0 / 1 (level order), -1 = NA */
  const double* prior_x;   /* host, ngrid */
  const double* prior_y;   /* host, ngrid */
  int ngrid;
  int nboot;               /* n.randomizations */
  int n_cores;             /* reference seeding mode: chunk seeds as R's n.cores */
  int64_t gene_offset;     /* first global gene index of this shard */
  int64_t ngenes_total;    /* global number of genes (for chunk seeds) */
  double expectation;      /* R `expectation` (log2 scale) */
  int rand_kind;           /* SCDE_RAND_GLIBC / SCDE_RAND_DARWIN */
  int compute_cz;          /* 1: this call covers every gene; results gain a 6th column cZ (device BH) */
} scde_de_params;

/* scde.expression.difference (R/functions.R:304-407, no batch) on device-resident
 * counts (int32, column-major, leading dimension ld, rows gene_offset.. of the shard
 * start at counts_dev).  results: host ngenes x 5 col-major (lb, mle, ub, ce, Z), or
 * x 6 with cZ when p->compute_cz (whole call = all genes); for shards cZ is left to
 * scde_bh_cz / scde_bh_cz_dev over the gathered Z.  jp1/jp2 (ngenes x ngrid) and
 * ratio (ngenes x (2*ngrid-1)) are optional host outputs, col-major. */
int scde_expression_difference_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes,
                                   const scde_de_params* p, double* results, double* jp1, double* jp2,
                                   double* ratio);

/* Batch-corrected scde.expression.difference (R/functions.R:321-399) on device-resident
 * counts: p as for scde_expression_difference_dev (compute_cz is implied), batch_models
 * ncells x 12 col-major (NULL = p->models), batch_codes[ncells] in [0, nbatch) (level
 * order).  results: host, three consecutive ngenes x 6 col-major blocks (lb, mle, ub, ce,
 * Z, cZ) for batch.adjusted, results, batch.effect.  Optional host outputs, col-major:
 * jp1/jp2 (the groups' joint posteriors, ngenes x ngrid), ratio (the group difference posterior, ngenes x (2*ngrid-1)), adj_ratio (the
 * batch-adjusted posterior, ngenes x (4*ngrid-3)), batch_ratio (ngenes x (2*ngrid-1)). */
int scde_expression_difference_batch_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes,
                                         const scde_de_params* p, const double* batch_models,
                                         const int* batch_codes, int nbatch, double* results, double* jp1,
                                         double* jp2, double* ratio, double* adj_ratio, double* batch_ratio);

/* The same three calls on the caller's HOST count matrix, as the R shim makes them
 * (R/functions.R:304 scde.expression.difference, :566 scde.posteriors; the R glue hands
 * the count matrix to the native side once per call): counts int32 column-major with
 * leading dimension ld >= ngenes and p->ncells (scde_posteriors_host: ncells_total)
 * columns, staged into the context's device buffer on its stream, then the resident
 * pipeline above.  ctx may be NULL: the process-wide default context (device
 * $SCDE_DEVICE, created lazily on first use, i.e. after any fork). */
int scde_expression_difference_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes,
                                    const scde_de_params* p, double* results, double* jp1, double* jp2,
                                    double* ratio);
int scde_expression_difference_batch_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes,
                                          const scde_de_params* p, const double* batch_models,
                                          const int* batch_codes, int nbatch, double* results, double* jp1,
                                          double* jp2, double* ratio, double* adj_ratio, double* batch_ratio);
int scde_posteriors_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes, int ncells_total,
                         const int* cellidx, int ncells_sel, const double* models_sel, int local_theta,
                         int square_logit_conc, const double* prior_x, int ngrid, int nboot, int n_cores,
                         int64_t gene_offset, int64_t ngenes_total, int return_post, int ensemble,
                         const int* batch_vals, const int64_t* batch_off, const int* composition, int nbatch,
                         double* jp, double* modes, double* post);

/* pagoda.varnorm's posterior-mode consumer (R/functions.R:1414-1507; SURVEY.md section 8(f)
 * row 4).  Runs scde.posteriors (n.cores seeding, nboot randomizations) over all cells and,
 * with a batch (batch_codes[ncells] in [0, nbatch), nbatch > 1), over each level's cells; the
 * modes are jp %*% as.numeric(colnames(jp)) (use_expected_value) or the magnitude of each row's
 * maximum.  Outputs (host): modes (1 [+ nbatch]) x ngenes (dataset-wide, then per level);
 * matw ngenes x ncells = 1 - mfp * sfp with mfp = scde.failure.probability at log(dataset
 * modes) and sfp = ppois(count - 1, exp(fail.r), lower.tail = FALSE) (1466-1474); bmatw (with
 * a batch) the same with each cell's level modes (1485-1506).  models: ncells x 12 col-major. */
int scde_pagoda_varnorm_weights_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, int ncells,
                                    const double* models, int local_theta, int square_logit_conc,
                                    const double* prior_x, int ngrid, int nboot, int n_cores, const int* batch_codes,
                                    int nbatch, int use_expected_value, double* modes, double* matw, double* bmatw);
int scde_pagoda_varnorm_weights_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes, int ncells,
                                     const double* models, int local_theta, int square_logit_conc,
                                     const double* prior_x, int ngrid, int nboot, int n_cores,
                                     const int* batch_codes, int nbatch, int use_expected_value, double* modes,
                                     double* matw, double* bmatw);

/* scde.expression.prior (R/functions.R:225-254; replaces the R-level function, which has
 * no .Call) on device-resident counts (ngenes x ncells int32, column stride ld).  models:
 * ncells x 12 col-major (conc.b, conc.a, ..., corr.b, corr.a, ..., conc.a2 at column 11 when
 * square_logit_conc).  max_value NULL = quantile(x[x < Inf], max_quantile) of the
 * log10(FPM + 1) magnitudes (type 7).  Outputs (host, length_out + 1 each): x, y, lp,
 * grid_weight (lp / grid_weight may be NULL); max_value_out (nullable) receives the
 * max.value used.  length_out in [1, 2047]. */
int scde_expression_prior_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, int ncells,
                              const double* models, int square_logit_conc, int length_out, double pseudo_count,
                              double bw, double max_quantile, const double* max_value, double* x, double* y,
                              double* lp, double* grid_weight, double* max_value_out);

/* scde.posteriors (R/functions.R:566-669) on device-resident counts for the cells
 * listed in cellidx (host, ncells_sel entries).  Outputs are host, col-major.
 * batch_* may be NULL (no batch).  return_post: R postflag (0..3). */
int scde_posteriors_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const int* cellidx,
                        int ncells_sel, const double* models_sel, int local_theta, int square_logit_conc,
                        const double* prior_x, int ngrid, int nboot, int n_cores, int64_t gene_offset,
                        int64_t ngenes_total, int return_post, int ensemble, const int* batch_vals,
                        const int64_t* batch_off, const int* composition, int nbatch, double* jp, double* modes,
                        double* post);

/* ---------------------------------------------------------------- weighted PCA
 * Bailey's EM weighted PCA behind bwpca() / pagoda.pathway.wPCA() (BASELINE config 5;
 * SURVEY.md section 8(f) row 3).
 *
 * .Call("baileyWPCA", Mat, Matw, Npcs, Nstarts, Smooth, EMtol, EMmaxiter, Seed, Nshuffles)
 * (src/bwpca.cpp:59-182; declared src/bwpca.h:8) on host buffers.  mat, matw: n (cells)
 * x d (genes) col-major.  The reference's random inputs are arguments, produced by the
 * caller exactly as the reference draws them (the .Call shim in INTEGRATION.md):
 *   starts: (1 + nshuffles) x nstarts x (d x K) uniforms, K = min(npcs, d), in draw order
 *           (arma::randu<arma::mat>(d, npcs) per start = R's unif_rand() stream;
 *           src/bwpca.cpp:197-198; Seed is a no-op there);
 *   perms:  nshuffles x d x n row indices (set_random_matrices' std::random_shuffle over
 *           rand(); src/bwpca.cpp:41-57), see scde_shuffle_perms.
 * Outputs: rotation d x K, scores n x K, scoreweights n x K (nullable), var K, totvar,
 * randvar nshuffles (src/bwpca.cpp:164-180).  npcs <= 8. */
int scde_baileyWPCA(const double* mat, const double* matw, int n, int d, int npcs, int nstarts, int smooth,
                    double em_tol, int em_maxiter, const double* starts, int nshuffles, const int* perms,
                    double* rotation, double* scores, double* scoreweights, double* var, double* totvar,
                    double* randvar);

/* A batch of baileyWPCA problems on one device-resident matrix pair: M_dev / W_dev are
 * ncells x mcols col-major (column stride ld), i.e. pagoda's t(varinfo$mat) / t(matw).
 * Problem p: d[p] columns cols[col_off[p] ..], npcs[p] (K = min(npcs, d) <= 8), nstarts[p]
 * starts from starts[start_off[p] ..] (nstarts x d x K uniforms), rows permuted per column
 * by perms[perm_off[p] ..] (d x ncells) when perm_off (nullable) is >= 0.  Outputs (host),
 * concatenated in problem order: rotation d x K, scores / scoreweights / colmeans ncells x K
 * (colmeans[j, k] = mean_g M[j, g] |rotation[g, k]|, pagoda's orientation statistic;
 * scoreweights / colmeans nullable), stats K + 2 per problem (var[K], totvar, the residual
 * of component 1 alone), iterations (nullable) per (problem, start). */
int scde_bwpca_batch_dev(scde_ctx* ctx, const double* M_dev, const double* W_dev, int64_t ld, int ncells,
                         int64_t mcols, int nprob, const int* d, const int* npcs, const int* nstarts,
                         const int64_t* col_off, const int* cols, int64_t ncols, const int64_t* perm_off,
                         const int* perms, int64_t nperms, const int64_t* start_off, const double* starts,
                         int64_t nstart_vals, int smooth, double em_tol, int em_maxiter, double* rotation,
                         double* scores, double* scoreweights, double* colmeans, double* stats, int* iterations);

/* R's RNG (src/main/RNG.c), host side, for the mirror of the R glue: set.seed(seed) into
 * a 625-word Mersenne-Twister state (word 0 = mti), unif_rand() draws, and R >= 3.6
 * sample.int(n, k) without replacement (1-based, rejection sampling). */
int scde_r_set_seed(uint32_t seed, uint32_t* state);
int scde_r_unif_rand(uint32_t* state, int64_t n, double* out);
int scde_r_sample(uint32_t* state, int n, int k, int* out);
/* set_random_matrices' permutations (src/bwpca.cpp:41-57) after srand(seed) with the
 * platform rand() (scde_set_rand_kind): nshuffles x d x n. */
int scde_shuffle_perms(unsigned int seed, int nshuffles, int d, int n, int* perms);

/* ---------------------------------------------------------------- PAGODA helpers
 * The remaining .Call symbols of the package (src/pagoda.cpp; declared src/pagoda.h:5-8),
 * SURVEY.md section 8(f) row 4.  Host buffers, R column-major. */

/* .Call("winsorizeMatrix", Mat, Trim) (src/pagoda.cpp:6-31): per row, the round(ncol * trim)
 * smallest values become the next smallest, the largest the next largest.  ncol <= 8192,
 * or round(ncol * trim) <= 32. */
int scde_winsorizeMatrix(const double* mat, int nrow, int ncol, double trim, double* out);

/* .Call("matWCorr", Mat, Matw) (src/pagoda.cpp:41-65): weighted correlation of columns i < j
 * with weights sqrt(w_i w_j) / sum; out ncol x ncol: 1 on the diagonal, c(j, i) below it,
 * 0 above (as the reference fills it). */
int scde_matWCorr(const double* mat, const double* matw, int nrow, int ncol, double* out);

/* .Call("matCorr", X, Y) = arma::cor(x, y) (src/pagoda.cpp:33-38): x nrow x nx, y nrow x ny,
 * out nx x ny. */
int scde_matCorr(const double* x, int nrow, int nx, const double* y, int ny, double* out);

/* .Call("plSemicompleteCor2", Pl) (src/pagoda.cpp:67-117): np sparse vectors (list element p
 * = gene indices idx[off[p] .. off[p+1]) increasing, values val[...]); r = correlation over
 * the shared genes (np x np, 1 on the diagonal), n = union sizes (np x np, 0 on it). */
int scde_plSemicompleteCor2(int np, const int64_t* off, const int* idx, const double* val, double* r, int* n);

#ifdef __cplusplus
}
#endif
#endif /* SCDE_HIP_H */
