// kernels.h -- argument blocks and launchers for kernels.hip (internal).
#pragma once

#ifndef SCDE_BOOT_WPE
#define SCDE_BOOT_WPE 8  // k_boot2 (NB <= 20) occupancy target: 8 waves per SIMD = 64 VGPRs
#endif
#ifndef SCDE_BOOT_ASMLD
#define SCDE_BOOT_ASMLD 1  // k_boot2 column look-ahead issued from asm with explicit vmcnt waits
#endif
#ifndef SCDE_NB_CLOSED
#define SCDE_NB_CLOSED 1  // the tables' NB log-pmf in closed form (0: nmath's saddle-point form)
#endif
#ifndef SCDE_TAB_WPE
#define SCDE_TAB_WPE 4  // k_tables_cell occupancy target (waves per SIMD)
#endif
#ifndef SCDE_BOOT_EB
#define SCDE_BOOT_EB 4  // ELL entries per k_boot2 batch (rows are padded to a multiple of 8, plus 8)
#endif
#ifndef SCDE_BOOT_DIAG
#define SCDE_BOOT_DIAG 0  // bit switches that remove parts of k_boot2 for timing studies
#endif
#ifndef SCDE_RATIO_WPE
#define SCDE_RATIO_WPE 1  // k_ratio_summary occupancy target (waves per SIMD; 1 = compiler's choice)
#endif
#ifndef SCDE_RATIO_DIAG
#define SCDE_RATIO_DIAG 0  // timing-only builds: 1 skips the slide, 2 the summary (results wrong)
#endif
#ifndef SCDE_WPCA_BLOCK
#define SCDE_WPCA_BLOCK 512  // wpca.hip workgroup size (8 waves)
#endif
#include <hip/hip_runtime.h>

namespace scde {

// k_col_consts record per column: [n or -1, n - x, stirlerr sum, 0.5 lf, log(size/(size+x)),
// log X - log n, log(n - X) - log n, dpois_log(x, failure rate), log po, log(1 - po)] with
// po = size / (size + x) (the count's own grid point), padded to 10 doubles
constexpr int kColc = 11;
// columns per task of the cell-staged tables kernels (k_tables_lpc: one lane per column)
#ifndef SCDE_TAB_TASK_COLS
#define SCDE_TAB_TASK_COLS 64
#endif
constexpr int kTabTaskCols = SCDE_TAB_TASK_COLS;

struct TablesArgs {
  const int* ucl;            // flat unique counts, [ncols]
  const long long* ucl_off;  // [ncells + 1]
  long long ncols;
  int ncells;
  int G, GS;
  const double* mu;          // [ncells][GS]
  const double* lcfp;        // [ncells][GS]
  const double* lcfpr;       // [ncells][GS]
  const double* theta;       // [ncells][GS]
  const double* cellscal;    // [ncells][2] = {max log cfp, exp(fail.r)}
  double minlogprob;         // -DBL_MAX / ncells / 1.1
  // k_tables_lpc writes its rows (T, D) as non-temporal stores (the same bits)
  int nt_rows;
  double* T;                 // [ncols][GS] log-posterior columns
  int* maxi;                 // [ncols] argmax (nullable)
  unsigned char* has_clamp;  // [ncols]
  int const_theta;           // theta is the same at every grid point (no local theta fit)
  const double* pq;          // [ncells][4][GS] p, q, log p, log q (const_theta), nullable
  const double* colc;        // [ncols][kColc] k_col_consts output (with pq), nullable
  const double* cfp = nullptr;  // [ncells][GS] exp(lcfp) from k_cell_prep (nullable: computed when staged)
  // Fused baseline-delta output (bootstrap path; the k_delta pass folded into the tables):
  //   phase 0: every column -> T (no D);
  //   phase 1: one wave per cell, its count-0 column -> D (and T if non-null); writes
  //            zcol[c] and base_col[c] (count-0 column when it has no clamp and use_baseline);
  //   phase 2: every other column -> D = T - T[base_col] (T itself where the cell has no
  //            baseline), pad lanes [G, GS) zeroed, column ncols all zero; T if non-null.
  int phase;
  int use_baseline;
  double* D;      // [ncols + 1][GS]
  int* zcol;      // [ncells] count-0 column or -1
  int* base_col;  // [ncells]
  // chunked launches (the host-count pipeline): every column array above (ucl, T, maxi,
  // has_clamp, D, U, UQ, colc) and the per-cell arrays start at the chunk's first column / cell;
  // zcol and base_col hold global column indices, col_base = the chunk's first global column
  int col_base;
  // Cell-staged tables (phases 0 and 2, G <= 448): per block {cell, first column, end
  // column, 0}; one task with cell -1 writes the ELL pad column (phase 2).  Null: the
  // column-per-wave kernel.
  const int4* tasks;
  int ntasks;
  // Stretch bounds for k_boot2's grid-stretch skipping (nullable): per column and 64-point
  // stretch j, max_j T (phase 1) or max_j T - max_j T[baseline column] (phase 2; the
  // maximum itself where the cell has no baseline); 0 for the pad column.  [ncols + 1][8]
  double* U;
  // k_boot_tiles' tile bounds (phase 2; nullable): per 32-point tile the column's maximum in
  // units of 2^-8, rounded up, as four balanced base-256 digits (packu); phase-2 columns
  // store it minus their baseline column's value.  Pad column: 0.  A NaN sets *nanflag.
  unsigned* UQ;            // [ncols + 1][kQTiles]
  int* nanflag;
  // nullable: the launch does nothing unless *gate != 0 (the exact fallback's T tables are
  // built only when some gene needs them)
  const int* gate;
  // k_tables only: take just the columns k_tables_lpc leaves (colc n < 0, flagged by
  // k_col_consts in the int after colc's last column); the launch exits unless that flag is set
  int slow_only;
};

// ---- k_boot_tiles' integer tile bounds
constexpr int kQTiles = 16;  // 32-point bound tiles per column (G <= 448 uses <= 14)
constexpr int kBTile = 32;   // grid points per bound tile
__host__ __device__ inline unsigned packu(int u) { return ((unsigned)u + 0x80808080u) ^ 0x80808080u; }  // |u| < 2^31
__host__ __device__ inline int unpacku(unsigned p) { return (int)((p ^ 0x80808080u) - 0x80808080u); }
// ZUq[set][l][t][Bp]: the baseline cells' part of the tile bounds (four digits l)
hipError_t launch_zuq(const unsigned* UQ, const int* base_col, int ncells, const unsigned char* W8, int Bp, int nsets,
                      int* ZUq, hipStream_t s);

struct BootArgs {
  const double* T;  // [ncols][GS]
  int G, GS;
  const int2* ent;  // [ngenes][ent_stride] (cell, flat column)
  const int* nnz;   // [ngenes]
  int ent_stride;
  const int* base_col;  // [ncells] baseline column (count 0) or -1; nullable
  const double* Wt;     // [nsets][ncells][Bp] draw multiplicities
  int ncells, Bp, nboot;
  const int* wset;   // [ngenes] draw-set id per gene (nullable -> 0)
  const double* Z;   // [nsets][Bp][GS] baseline sums (nullable)
  double norm_mult;  // nboot for logBoot*Posterior, 1 for jpmat*
  double degen_thresh;
  double* out;
  long long out_g, out_k;
  int* degen;  // [ngenes]
  int ngenes;
};

struct Boot2Args {
  const double* D;  // [ncols + 1][GS] baseline-delta columns (k_delta)
  long long ncols_p1;  // columns of D (ncols + 1)
  const int2* ent;  // [ngenes][ent_stride] (cell, column) -- the k_ell list
  const int* nnz;
  int ent_stride;
  const double* Wt;  // [nsets][ncells][Bp], Bp a multiple of nb
  int Bp, ncells;
  const int* wset;
  const double* Z;  // [nsets][Bp][GS]
  int G, GS, nboot, nb;
  double norm_mult, degen_thresh;
  double* part;  // [ceil(nboot/nb)][ngenes][GS] per-slab partial jp rows
  long long part_stride;
  double* out;
  long long out_g, out_k;
  int* degen;
  int ngenes;
  // Grid-stretch skipping (nullable U disables it; needs G <= 448, nb <= 20): stretch
  // bounds of the columns (TablesArgs::U) and their baseline part ZU [nsets][Bp][8]
  const double* U;
  const double* ZU;
  int* mask;     // [ngenes][P] needed-stretch bits (k_stretch_mask output)
  double* ubuf;  // [ngenes][P][8][nb] stretch upper bounds (k_stretch_mask output)
  int* redo;     // [ngenes][P] slabs whose skipped stretches failed the post-check (tile path:
                 // fallback flags, then the fallback list length and [ngenes * P] list)
  double slack;  // heuristic slack of the mask (NaN: the default 20 + 0.15 C)
};

// k_boot_tiles (with Boot2Args; needs G <= 448): multiplicities as bytes and the tables'
// 16-point tile bounds for the exact integer tile bounds of each (gene, slab)
struct TileBootArgs {
  const unsigned char* W8p;  // [nsets][ncells][P][32] draw multiplicities (<= 127): per slab the pairs
                             // (boot r, boot 16 + r) of its boots, r < 16 (0 past the slab's live boots)
  int Bq;                    // ZUq's boot stride: a multiple of 32, >= the last slab's first boot + 32
  const unsigned* UQ;        // [ncols + 1][kQTiles] packed 32-point tile maxima (units of 2^-8, rounded up)
  const int* ZUq;            // [nsets][4][kQTiles][Bq] baseline tile-bound digit sums
  const int* nanflag;        // tables saw a NaN: every slab goes to k_boot2
  int maxgroups;             // 32-point bound tiles computed per slab, 1..4 (4; tests force the fallback with fewer)
  int* stats;                // nullable: [0] slabs, [1] tiles computed, [2] tiles, [3] slabs left to k_boot2,
                             // [4] sum of groups x entries (FMA count / (64 nb)), [5] entries of the slabs left,
                             // [6 + i] slabs that computed i tiles (i <= 28), [35] slabs a pair pass left
  const int* order;          // nullable: genes in this order (launch_gene_order)
  unsigned* pmask;           // [ngenes][P] tiles each slab's partial row holds (k_sum_partials reads those)
  int* wide = nullptr;       // [1 + ngenes * P] the list pass's slabs: [0] length, then g * P + p
  int gene = 0;              // k_boot_gene: a 4-wave block per (gene, group of SG slabs), 16 rows shared
                             // by the group's slabs; failures take the list pass over `wide`
  int SG = 0;                // slabs per group (<= 8, SG x nb <= 128)
  int kcap = 4;              // rows per slab at most (tests force the list pass with fewer)
  int list_cap = 0;          // slabs the list pass takes at most (0: 16384; tests force the overflow to k_boot2)
  const unsigned char* W8g = nullptr;  // [nsets][ncells][groups][4 windows][32] the group's boots 32 w + j
                                       // as pair slots (boot 32 w + j, 32 w + 16 + j), 0 past its boots
  // gene blocks only: this launch takes genes [g_lo, g_hi) (g_hi < 0: all) -- a posterior's bootstrap in
  // gene chunks, each finished (list pass, fallback, slab sums) before the next, so its jp rows can
  // be read back while the next chunk runs; `order` then holds each chunk's genes sorted within it
  int g_lo = 0, g_hi = -1;
  // gene blocks holding all of a gene's slabs (SG >= P): [ngenes] flags; a gene whose slabs all pass
  // their post-checks gets its jp row from its block (summed in slab order, as k_sum_partials would)
  // and flag 1, so k_sum_partials skips it (null: every row through k_sum_partials)
  int* gdone = nullptr;
};
hipError_t launch_boot_tiles(const Boot2Args& a, const TileBootArgs& tb, hipStream_t s);
// gene order for the tile bootstrap: the keys launch_ell formed (per-gene count sums), sorted
hipError_t launch_gene_order(const unsigned* key, const int* idx, int n, unsigned* key_out, int* order, void* work,
                             size_t* work_bytes, hipStream_t s, int bits = 16);

struct ExactArgs {
  const double* T;  // log tables; or fused D columns when base_col is set (T = D + D[base])
  const int* base_col;
  int G, GS;
  const int* draws;  // [nsets][nboot][ndraw] cell index per draw, reference order (-1: no draw, the
                     // shorter group's padding when two groups are fused)
  int ndraw, nboot;
  long long gene_mod;  // fused groups: gene g reads uci row g % gene_mod (0: g)
  const int* wset;
  const long long* ucl_off;
  const int* uci;  // [ld_uci x ncells] or null for jpmat (column = cell*ngenes + g)
  long long ld_uci;
  double norm_mult;
  const int* degen;
  double* out;
  long long out_g, out_k;
  int ngenes;
  int g_lo = 0, g_hi = -1;  // the launch's genes [g_lo, g_hi) (g_hi < 0: all): a gene chunk
};

struct NoBootArgs {
  const double* T;  // log tables, or normalised exp tables for ensemble
  int G, GS;
  const long long* ucl_off;
  const int* uci;
  long long ld_uci;
  int ncells, ngenes;
  int ensemble;
  double* out;
  long long out_g, out_k;
};

struct RatioArgs {
  const double* jp1;
  long long j1g, j1k;
  const double* jp2;
  long long j2g, j2k;
  const double* prior_y;  // nullable: skip.prior.adjustment
  int n, ngenes;
  int normalize;  // 1: divide by the (long double) row sum (calculate.ratio.posterior); 0: raw matSlideMult
  const double* xin;  // nullable: summarise this ratio matrix [g*xg + o*xo] (m = 2n-1 columns) instead
  long long xg, xo;
  double* ratio;  // nullable; [g*rg + o*ro]
  long long rg, ro;
  const double* diffv;  // [2n-1]
  int zi;
  double* res;  // nullable; column-major res_ld x 5 (lb, mle, ub, ce, Z)
  long long res_ld;
  int window, block;  // register-window width R (4, 5, 7, 8) and block size (64/128/256); 0 = default
};

hipError_t launch_cell_prep(const double* models, int ncells, int G, int GS, const double* mag, int lt, int sq,
                            double* mu, double* lcfp, double* lcfpr, double* theta, double* cellscal,
                            double* pq, hipStream_t s, double* cfp = nullptr);
hipError_t launch_col_consts(const int* ucl, const long long* ucl_off, long long ncols, int ncells,
                             const double* theta, int GS, const double* cellscal, double* colc, hipStream_t s);
hipError_t launch_tables(const TablesArgs& a, hipStream_t s);
// gsets > 0 (two fused groups): sets from gsets on sum the cells from gsplit on, the others the
// cells before it, each in its group's own order
hipError_t launch_stretch_zu(const double* U, const int* base_col, int ncells, const double* Wt, int Bp, int nsets,
                             double* ZU, hipStream_t s, int gsets = 0, int gsplit = 0);
hipError_t launch_base_cols(const int* ucl, const long long* ucl_off, int ncells, const unsigned char* has_clamp,
                            int use_baseline, int* base_col, hipStream_t s);
// padto 8: rows padded to a multiple of 8 plus one batch of 8 (k_boot2's look-ahead); 64: to a
// multiple of 64 plus 8 (k_boot_tiles' bound MFMAs take 64-entry steps)
// cell_off: added to the cell of every entry (a fused second group's cells follow the first's)
// work: ell_work_bytes(ngenes, ncells) bytes (null allowed when that is 0) -- the per cell-chunk
// entry counts and count sums of the two-pass build.  key (nullable, with ucl and idx): the
// tile bootstrap's 16-bit gene-order keys (log-scaled sums of the entries' counts ucl[col]) and gene indices, the
// launch's genes being genes kg0 .. of kgn split into kch gene chunks (the chunk index in the
// key's top bits; desc: descending within a chunk)
// out[i] = in[i] for n 16-bit counts
hipError_t launch_widen16(const unsigned short* in, int* out, size_t n, hipStream_t s);
// out[exc[i].x] = exc[i].y for n listed counts (indices relative to out)
hipError_t launch_patch32(const int2* exc, size_t n, int* out, hipStream_t s);
// max_chunks: at most this many cell chunks (0: as many as fill the chip twice, at most 64)
size_t ell_work_bytes(int ngenes, int ncells, int max_chunks = 0);
hipError_t launch_ell(const int* uci, long long ld_uci, int ngenes, int ncells, const long long* ucl_off,
                      const int* base_col, int stride, int pad_col, int padto, int2* ent, int* nnz, hipStream_t s,
                      int cell_off, void* work, const int* ucl = nullptr, unsigned* key = nullptr, int* idx = nullptr,
                      int kg0 = 0, int kgn = 0, int kch = 1, int desc = 0, int max_chunks = 0);
hipError_t launch_baseline_z(const double* T, int G, int GS, const int* base_col, int ncells, const double* Wt,
                             int Bp, int nsets, double* Z, hipStream_t s, int gsets = 0, int gsplit = 0);
// Draw multiplicities on the device from the draw lists draws[nsets][nboot][ndraw] (cell index, -1
// = no draw): Wt[set][c][Bp] (doubles), and for the tile path (nullable) W8[set][c][Bt],
// W8p[set][c][P][32] (per slab of nb boots the pairs (j, 16 + j) in slots 2j, 2j + 1) and
// W8g[set][c][NGR][128] (per group of SG slabs four 32-boot windows as pair slots).  The arrays are
// zeroed here first.  ncells <= kMultMaxCells.
constexpr int kMultMaxCells = 16384;
hipError_t launch_mult(const int* draws, int nsets, int nboot, int ndraw, int ncells, int Bp, double* Wt, int Bt,
                       unsigned char* W8, int nb, int P, unsigned char* W8p, int SG, int NGR, unsigned char* W8g,
                       hipStream_t s);
// test hook: one wave spinning `cycles` shader clocks on stream s (handoff_spin)
hipError_t launch_spin(hipStream_t s, long long cycles);
hipError_t launch_boot(const BootArgs& a, hipStream_t s);
hipError_t launch_boot_exact(const ExactArgs& a, hipStream_t s);
int boot2_nb(int nboot);
hipError_t launch_boot2(const Boot2Args& a, hipStream_t s);
hipError_t launch_delta(const double* T, const long long* ucl_off, int ncells, long long ncols, const int* base_col,
                        int G, int GS, double* D, hipStream_t s);
hipError_t launch_noboot(const NoBootArgs& a, hipStream_t s);
hipError_t launch_ensemble_cols(const double* T, long long ncols, int G, int GS, double* E, hipStream_t s);
hipError_t launch_modes(const int* uci, long long ld_uci, int ngenes, int ncells, const long long* ucl_off,
                        const int* maxi, const double* mag, double* modes, long long mg, long long mc,
                        hipStream_t s);
hipError_t launch_post(const int* uci, long long ld_uci, int ngenes, int c, const long long* ucl_off,
                       const double* T, int G, int GS, double* post, long long pg, long long pk, hipStream_t s);
hipError_t launch_cell_minmax(const int* counts, long long ld, long long g0, int ngenes, int ncells,
                              const int* cellidx, int* cmax, int* cmin, hipStream_t s);
hipError_t launch_mark(const int* counts, long long ld, long long g0, int ngenes, int ncells, const int* cellidx,
                       const long long* woff, unsigned long long* bits, hipStream_t s,
                       int* flags = nullptr);
hipError_t launch_rank(const unsigned long long* bits, const long long* woff, int ncells, int* rank, int* nuniq,
                       hipStream_t s,
                       const int* flags_in = nullptr, int* flags_out = nullptr);
hipError_t launch_fill_ucl(const unsigned long long* bits, const long long* woff, int ncells, const int* rank,
                           const long long* ucl_off, int* ucl, hipStream_t s);
hipError_t launch_uci(const int* counts, long long ld, long long g0, int ngenes, int ncells, const int* cellidx,
                      const long long* woff, const unsigned long long* bits, const int* rank, int* uci,
                      hipStream_t s);
hipError_t launch_colmajor_to_rows(const double* src, int nrows, int ncols, int GS, double* dst, hipStream_t s);
// device BH cZ (bh.hip); work == nullptr -> *work_bytes = required size
hipError_t launch_bh_cz(const double* z, int n, double* cz, void* work, size_t* work_bytes, hipStream_t s);

// scde.expression.prior (prior.hip).  cellp: 5 x C (corr.b, corr.a, conc.b, conc.a, conc.a2).
// Stats: out[0..3] = sum w, sum w over finite v, max finite v, count of finite v; occ:
// prior_items(N, C) x 256 count multiplicities (read back by launch_prior_bin); vout (nullable)
// = v per element in R order.
hipError_t launch_prior_stats(const int* counts, long long ld, int N, int C, const double* cellp, int sq,
                              double* vout, int* occ, double* partials, int nb, double* out, hipStream_t s);
long long prior_items(int N, int C);
int prior_blocks(int N, int C, int cap);
int prior_grid_n(int L);
// hist: prior_grid_n(L) u64 (zeroed here); work: 3 x prior_grid_n(L) doubles; out: 4 x (L+1)
// (x, y, lp, grid.weight)
hipError_t launch_prior_bin(const int* counts, long long ld, int N, int C, const double* cellp, int sq,
                            const int* occ, double wsum, double max_value, double bw, int L,
                            unsigned long long* hist, int nb, hipStream_t s);
hipError_t launch_prior_tail(double tot_mass, double max_value, double bw, int L, double pc,
                             const unsigned long long* hist, double* work, double* out, hipStream_t s);
hipError_t launch_sort_doubles(const double* in, double* out, long long n, void* work, size_t* work_bytes,
                               hipStream_t s);
hipError_t launch_ratio_summary(const RatioArgs& a, hipStream_t s);


// ---- weighted PCA (wpca.hip; src/bwpca.cpp).  One problem = a column subset of the
// resident cells x genes value/weight matrices (column g at M + col*ld), optionally
// row-permuted per column (internal shuffles).  All offsets in elements.
constexpr int kWpcaMaxK = 8;
struct WpcaProb {
  int d, K, nstarts, pad;
  long long col_off;    // cols[col_off .. +d)
  long long perm_off;   // perms[perm_off .. + d*n) or -1
  long long start_off;  // starts[start_off .. + nstarts*d*K): randu(d, K) per start
  long long sE_off;     // scratch: best eigenvectors, nstarts x d x K
  long long sC_off;     // scratch: coefficient slots, nstarts x 2 x n x K
  long long sW_off;     // scratch: working coefficients (when not in LDS), nstarts x n x K
  long long mom_off;    // scratch: moments + smoothing row, nstarts x d x (NM + 1)
  long long stat_off;   // stat rows (pres, bpres, iterations, best slot), one per start
  long long out_rot, out_sc, out_pcw, out_cm, out_var;  // outputs (var: K + 2 doubles)
};
struct WpcaLaunch {
  const double* M;
  const double* W;
  long long ld;
  int n, dmax;
  const WpcaProb* probs;
  const int2* blocks;
  const int* cols;
  const int* perms;
  const double* starts;
  int maxiter;
  double tol;
  const double* smoothc;
  int L;
  double* scratch;
  double* stat;
  double* out;
  int lds_cap;
};
int wpca_max_k();
int wpca_ms_group();
bool wpca_ms_ok(int n, int dmax);
// npcs = 1, em without smoothing: blocks = (problem, first start of a group of wpca_ms_group())
hipError_t launch_wpca_ms(const WpcaLaunch& a, int nblocks, hipStream_t s);
hipError_t launch_wpca_em(int K, const WpcaLaunch& a, int nblocks, hipStream_t s);
hipError_t launch_wpca_final(int K, const WpcaLaunch& a, const int* kidx, int nprob, hipStream_t s);

// ---- PAGODA helpers (pagoda.hip; src/pagoda.cpp).  Matrices column-major.
// winsorize: m k x n, ntr per side; n <= 8192, or ntr <= 32
hipError_t launch_winsorize(const double* m, int k, int n, int ntr, double* out, hipStream_t s);
// matWCorr: m, w k x n -> out n x n
hipError_t launch_matwcorr(const double* m, const double* w, int k, int n, double* out, hipStream_t s);
// matCorr: x k x nx, y k x ny -> out nx x ny; stats: 2 (nx + ny) doubles of scratch
hipError_t launch_matcorr(const double* x, int k, int nx, const double* y, int ny, double* stats, double* out,
                          hipStream_t s);
// plSemicompleteCor2: np lists (off[np + 1], idx, val) -> r, cnt np x np
hipError_t launch_plcor(int np, const long long* off, const int* idx, const double* val, double* r, int* cnt,
                        hipStream_t s);
// pagoda.varnorm's mode consumer: modes from jp (expected value or row-maximum magnitude);
// the weight matrix 1 - mfp * sfp for cells cellidx (matw: ngenes x ncells col-major)
hipError_t launch_vn_modes(const double* jp, long long jg, long long jk, int ngenes, int G, const double* mag,
                           int expected, double* modes, hipStream_t s);
hipError_t launch_vn_matw(const int* counts, long long ld, int ngenes, const int* cellidx, int ncells,
                          const double* models, int mld, int sq, const double* modes, const long long* mode_off,
                          double* matw, hipStream_t s);

}  // namespace scde
