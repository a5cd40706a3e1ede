// engine.hip -- host orchestration and the C ABI (include/scde_hip.h).
//
// Restates the R glue of the path on the host side (R/functions.R:566-669
// scde.posteriors, 3491-3531 ratio posterior / Z, 5039-5051 summary / BH) and
// drives the gfx950 kernels in kernels.hip on one HIP stream per context.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <functional>
#include <thread>
#include <atomic>
#include <memory>
#include <unistd.h>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "kernels.h"
#include "scde_hip.h"

using namespace scde;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// Fork guard (SURVEY.md §8(b) threading row).  The reference's R glue forks mclapply
// workers that each make their own .Call (R/functions.R:606-617), and with n.cores = 1 (or
// N <= n.cores) it calls in the R parent itself (629-637), so a session can initialise HIP
// in the parent and fork later.  A HIP runtime is not fork-safe: a child must not touch the
// state it inherited.  g_hip_pid records the process that made this library's first HIP
// call; any GPU entry in another process (a fork child of it) fails with SCDE_EFORK before
// any HIP call.  A process forked *before* that first call (mclapply from a fresh session)
// sees 0 and initialises its own runtime, as tests/test_fork.py checks.
std::atomic<pid_t> g_hip_pid{0};

int fork_guard() {
  const pid_t me = getpid();
  pid_t p = g_hip_pid.load(std::memory_order_acquire);
  if (p == me) return SCDE_OK;
  if (p == 0 && g_hip_pid.compare_exchange_strong(p, me)) return SCDE_OK;
  if (p == me) return SCDE_OK;
  return fail(SCDE_EFORK,
              "HIP was initialised by process %d before this process (%d) was forked from it; a forked child "
              "cannot use the inherited GPU runtime. Run scde with n.cores = 1 in the parent (the fused entries "
              "honour n.cores for seeding only), or make the first GPU call in the child",
              (int)p, (int)me);
}

#define FORK_GUARD()                      \
  do {                                    \
    if (int fg_ = fork_guard()) return fg_; \
  } while (0)

#define HCHK(expr)                                                                     \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(SCDE_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define RCHK(expr)            \
  do {                        \
    int r_ = (expr);          \
    if (r_ != SCDE_OK) return r_; \
  } while (0)

inline long long round_up(long long a, long long b) { return (a + b - 1) / b * b; }

// The C library rand() the reference calls (srand(Seed), then
// `rj = rand()/(RAND_MAX/n)` with rejection; src/jpmatLogBoot.cpp:220-221,255-257),
// with private state.  Its output depends on the platform libc:
//   SCDE_RAND_GLIBC  (0) glibc TYPE_3 additive feedback generator (Linux);
//   SCDE_RAND_DARWIN (2) Darwin/BSD libc: Park-Miller "minimal standard"
//                        x = 16807 x mod (2^31-1), srand(s) keeps s, returns x --
//                        the generator behind the package vignette's printed
//                        results (vignettes/diffexp.md:113-139).
int g_rand_kind = 0;

struct PlatformRand {
  int kind;
  int32_t t[31];
  int f = 3, r = 0;
  PlatformRand(unsigned int seed, int k) : kind(k) {
    if (kind == 2) {
      t[0] = (int32_t)seed;
      return;
    }
    if (seed == 0) seed = 1;
    t[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
      const long hi = word / 127773, lo = word % 127773;
      word = (int32_t)(16807 * lo - 2836 * hi);
      if (word < 0) word += 2147483647;
      t[i] = word;
    }
    for (int i = 0; i < 310; ++i) next();
  }
  int next() {
    if (kind == 2) {
      const long hi = t[0] / 127773, lo = t[0] % 127773;
      long x = 16807 * lo - 2836 * hi;
      if (x < 0) x += 0x7fffffff;
      t[0] = (int32_t)x;
      return (int)x;
    }
    const uint32_t v = (uint32_t)t[f] + (uint32_t)t[r];
    t[f] = (int32_t)v;
    if (++f >= 31) f = 0;
    if (++r >= 31) r = 0;
    return (int)(v >> 1);
  }
  int draw(int n) {
    int rj;
    while (n <= (rj = next() / (2147483647 / n))) {
    }
    return rj;
  }
};

// Reallocations of an existing workspace buffer (grow-only, so early calls only): each one is
// a hipFree, which waits for the device, plus -- for grow(keep) -- a copy after the owning
// context's streams are synchronised.  Counted process-wide (stat "buf_reallocs") so a
// regression that reallocates in steady state shows.
std::atomic<long long> g_buf_reallocs{0};

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    if (p) {
      g_buf_reallocs.fetch_add(1, std::memory_order_relaxed);
      hipError_t e = hipFree(p);
      p = nullptr;
      cap = 0;
      if (e != hipSuccess) return e;
    }
    size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  // ensure(bytes), or with keep: grown (25% headroom) keeping the contents, after
  // sync_streams() has drained every stream of the owning context that may still write or
  // read the old allocation (scoped to that context: the peer lane, other contexts and torch
  // streams keep running)
  template <class SyncStreams>
  hipError_t grow(bool keep, size_t bytes, SyncStreams&& sync_streams) {
    if (!keep || !p) return ensure(bytes);
    if (bytes <= cap) return hipSuccess;
    const size_t want = bytes + bytes / 4;
    void* q = nullptr;
    g_buf_reallocs.fetch_add(1, std::memory_order_relaxed);
    hipError_t e = sync_streams();
    if (e == hipSuccess) e = hipMalloc(&q, want);
    if (e == hipSuccess) e = hipMemcpy(q, p, cap, hipMemcpyDeviceToDevice);
    if (e != hipSuccess) {
      if (q) (void)hipFree(q);
      return e;
    }
    (void)hipFree(p);
    p = q;
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// R's chunk(seq_len(N), n) = split(x, sort(rank(x) %% n)) (R/functions.R:606):
// label r in 0..n-1 has #{i in 1..N : i %% n == r} genes, chunks in label order.
std::vector<long long> r_chunk_starts(long long N, int n) {
  std::vector<long long> starts;
  long long pos = 0;
  for (int r = 0; r < n; ++r) {
    long long cnt = (r == 0) ? N / n : (N >= r ? (N - r) / n + 1 : 0);
    if (cnt > 0) starts.push_back(pos);
    pos += cnt;
  }
  starts.push_back(N);
  return starts;
}

}  // namespace

enum {
  SLOT_TABLES = 0,
  SLOT_BOOT = 1,
  SLOT_RATIO = 2,
  SLOT_UNIQUE = 3,
  SLOT_OTHER = 4,
  SLOT_PRIOR_STATS = 5,
  SLOT_PRIOR_BIN = 6,
  SLOT_PRIOR_TAIL = 7,
  SLOT_WPCA_EM = 8,
  SLOT_WPCA_FINAL = 9,
  NSLOTS = 10
};

struct scde_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t home_stream = nullptr;  // `stream` as created (unique builds swap `stream` for a while)
  // host-count entry points: the count upload runs on its own stream, in column chunks, so
  // the first group's kernels start before the second group's columns have arrived
  hipStream_t copy_stream = nullptr;
  hipEvent_t up_ev[2] = {nullptr, nullptr};
  hipEvent_t uq_ev = nullptr;  // the second group's unique sets (built on copy_stream) are ready
  hipEvent_t modes_ev = nullptr;  // run_posterior's posterior modes are computed (they need the tables only)
  // run_posterior's bootstrap set-up (draw uploads, ELL rows, baseline bound sums, Z, gene
  // order) needs only the count-0 columns: it runs on aux_stream after p1_ev (phase 1 of the
  // tables), beside phase 2, and the bootstrap waits for aux_ev
  hipStream_t aux_stream = nullptr;
  hipEvent_t p1_ev = nullptr, aux_ev = nullptr;
  // Pinned staging arena for the small per-call transfers (cell lists, offsets, draws,
  // multiplicities, tasks; the unique builder's size read-backs).  A pageable copy is staged
  // by the runtime and costs 20-40 us of host latency each; from pinned memory it is a plain
  // asynchronous DMA.  Bump-allocated; when full, the device is synchronised (every staged
  // copy has landed) and allocation restarts at 0.
  char* pin = nullptr;
  size_t pin_off = 0;
  // workspace
  Buf models, mag, mu, lcfp, cfp, lcfpr, theta, cellscal, pq, colc, T, E, maxi, has_clamp, base_col, zcol, ent, nnz, Wt, Z, draws,
      ubound, zubound, smask, subuf, sredo,
      degen, wset, prior_y, diffv, jpA, jpB, res, ratio, in1, in2, outbuf, part, bhw;
  // scde.expression.prior
  Buf pr_cell, pr_part, pr_occ, pr_stats, pr_hist, pr_work, pr_out, pr_v, pr_sorted, pr_sortw;
  // weighted PCA (bwpca)
  Buf wp_probs, wp_blocks, wp_kidx, wp_cols, wp_perms, wp_starts, wp_scratch, wp_stat, wp_out, wp_smooth, wp_M, wp_W;
  // PAGODA helpers
  Buf pg_a, pg_b, pg_c, pg_d, pg_e;
  // host-count entry points: the call's counts staged here (grow-only, reused across calls)
  Buf counts_in;
  // fixed-point bootstrap: byte multiplicities, flags/counters
  Buf w8, w8t, w8g, qflags;
  // tile bootstrap gene order: keys, sorted keys, indices, order, sort workspace
  Buf gkey, gkey2, gidx, gorder, gwork, pmask, pwide, ellw, excd, gdone;
  // options (scde_ctx_set_option; include/scde_hip.h lists them): each a default path's switch or a
  // documented operating / test mode; read from the environment only at creation (SCDE_OPTIONS)
  int opt_boot_skip = 1;         // "boot_skip": grid-stretch / tile skipping in the bootstrap (same bits either way)
  double opt_skip_slack = NAN;   // "skip_slack": mask slack (NaN = 20 + 0.15 C); tests force redo slabs
  int opt_boot_nb = 0;           // "boot_nb": boots per slab (0 = automatic; a multiple of 4 in [4, 32])
  int opt_skip_stats = 0;        // "skip_stats": count kept stretches / redo slabs (a host sync per launch)
  int opt_wpca_ms = 1;           // "wpca_ms": the multi-start npcs = 1 kernel (k_wpca_ms1)
  int opt_boot_tiles = 1;        // "boot_tiles": the FP64 bootstrap on bounded 32-point tiles (k_boot_gene)
  int opt_boot_tiles_cells = 400;  // "boot_tiles_cells": cells per call from which it is used (fewer: the
                                   // rows are wide, most slabs need > 8 tiles, k_boot2's stretches win)
  int opt_tile_groups = 4;       // "tile_groups": 32-point bound tiles the list pass computes per slab (1..4; tests)
  int opt_tile_max_mult = 127;   // "tile_max_mult": largest multiplicity the tile path takes (int8; tests lower it
                                 // to force the fallback onto plain k_boot2 after the tables were set up for tiles)
  int opt_tile_order = 3;        // "tile_order": the tile bootstrap takes genes by count sum (cache sharing):
                                 // 1 ascending, 2 descending (heaviest first), 3 (default: descending in
                                 // scde.posteriors and in DE launches of at most kDescGenes genes, where the
                                 // last, heaviest blocks would set the launch's tail), 0 in gene order
  int opt_unique_fixed = 1;      // "unique_fixed": one host sync per unique build (fixed 1024-word bitmaps)
  int opt_upload_u16 = 1;        // "upload_u16": host-count ranges of >= 8 MB go up as 16-bit counts (U16Ring): 1
                                 // scde.posteriors' host entry, 2 every host entry, 0 none
  int opt_modes_overlap = 1;     // "modes_overlap": scde.posteriors' read-backs (modes piece by piece, jp in gene
                                 // chunks) overlap the tables and the bootstrap from a read-back thread (0: after
                                 // the bootstrap, on the main stream -- rocprofv3 runs, where the pageable
                                 // read-back becomes blit kernels that would share the CUs)
  int opt_jp_chunks = 4;         // "jp_chunks": gene chunks of scde.posteriors' gene-block bootstrap (host entry: each
                                 // chunk's jp rows read back while the next runs; 1: one launch, jp after it)
  int opt_gene_list_cap = 0;     // "gene_list_cap": slabs k_boot_gene's list pass takes at most (0: 16384; tests)
  int opt_gene_rows = 4;         // "gene_rows": rows per slab k_boot_gene gives each slab at most (tests force its
                                 // four-tile list pass with fewer)
  double opt_pipeline_mb = 32;  // "pipeline_mb": host-count DE calls from this many MB of counts upload in two
                                // column ranges, each group starting once its cells are in HBM
  int opt_pieces = 5;           // "pieces": the first group's columns of a pipelined host-count DE call upload
                                // in this many pieces, each piece's unique sets and tables starting as it lands
                                // (round 6, config 3, 5 alternating runs each: 4 pieces 6.49-6.78 ms host ->
                                // host, 5 pieces 6.38-6.48, 6 pieces 6.41-6.58)
  int opt_tables_nt = 2;        // "tables_nt": table rows as non-temporal stores (0 no, 1 yes, 2 when the call's
                                // rows exceed 256 MB)
  int fault_u16 = 0;            // test hook (scde_ctx_inject_fault): 16-bit upload slots to fail
  long long spin_cycles = 0;    // test hook: a spin kernel before every cross-stream handoff (handoff_spin)
  int fault_skip_join = 0;      // test hook: DE calls whose main stream skips its wait for the peer lane
  std::atomic<long long> st_spins{0};  // handoff spins launched (any thread; the peer counts its own)
  int opt_lanes = 2;            // "lanes": a DE call's two group posteriors run concurrently (2: the second
                                // group on `peer`, its own streams and workspace) or one after the other (1)
  // fixed settings that were options until round 5 (the alternatives measured slower or equal and were
  // removed)
  static constexpr int opt_ratio_window = 4;   // k_ratio_summary register window
  static constexpr int opt_ratio_block = 128;  // k_ratio_summary block size
  static constexpr int opt_upload_threads = 4; // the 16-bit narrowing pool
  static constexpr int opt_gene_direct = 1;    // gene blocks holding all of a gene's slabs write its jp row
  static constexpr int opt_ell_chunks = 1;     // the ELL rows in one pass
  static constexpr int opt_gene_blocks = 1;    // the tile path as k_boot_gene gene blocks
  // the second lane of a DE call: a context on the same device, created on first use; its
  // options are copied from this one per call and its timings/statistics merged back
  scde_ctx* peer = nullptr;
  hipEvent_t lane_ev[2] = {nullptr, nullptr};  // [0] this stream -> peer, [1] peer -> this stream
  hipEvent_t piece_ev[8] = {nullptr};           // run_posterior's pieces: unique sets built
  hipEvent_t piece_up_ev[8] = {nullptr};        // the pieces' uploads landed (upload worker)
  hipStream_t uq_stream = nullptr;              // the pieces' and the second group's unique builds
  // host-count upload thread (created on first use, lives with the context): a pageable copy
  // blocks its calling thread for the whole transfer, so the pieces go up from here, back to
  // back, while the caller builds unique sets and queues kernels
  struct Uploader {
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    bool stop = false, busy = false;
    long long job = 0;
    std::function<int(int)> issue;  // issue(j): upload range j and record its event
    int nranges = 0, issued = 0, err = 0;
    std::string err_msg;  // the worker thread's error text (its g_err is its own)
    std::chrono::steady_clock::time_point t_start;  // the job's start (stat upload_wake_ms)
    double wake_ms = 0, first_ms = 0;  // summed: start -> worker awake, start -> first range issued
  } upl;
  // Device -> host read-backs from a worker thread (a pageable hipMemcpy blocks its calling thread
  // for the whole transfer): scde.posteriors' modes columns piece by piece and its jp rows chunk by
  // chunk, each after the event recorded when its kernels were queued, so the read-back streams
  // out while later pieces' tables and chunks' bootstraps run.  Jobs of one call; dnl_wait drains.
  struct Downloader {
    struct Job {
      int ev;  // index into evs
      void* dst;
      const void* src;
      size_t dpitch, spitch, width, height;
    };
    std::thread th;
    std::mutex m;
    std::condition_variable cv, cvd;
    std::deque<Job> q;
    std::vector<hipEvent_t> evs;
    hipStream_t stream = nullptr;
    int pending = 0, err = 0, nev = 0;
    std::string err_msg;
    bool stop = false;
    bool hold = false;  // jobs queue but wait (dnl_hold): pageable read-backs slow the host-count uploads
  } dnl;
  // 16-bit host-count uploads (option "upload_u16"): a pool of T threads narrows each 4M-count
  // slot of the caller's int32 matrix to uint16 into a pinned ring slot, listing the counts
  // outside [0, 65535] (index, value) as they go; the upload worker sends the slot up, a widening
  // kernel writes the int32 counts behind it on the copy stream and a patch kernel the listed
  // ones (real matrices hold a few: config 4's synthetic 60M counts hold 10) -- half the PCIe bytes (tools/micro/h2d_u16.hip, 240 MB of counts: 2.9 ms
  // against 4.5 ms pageable).  Slots carry a global sequence number q (ring slot q % kRing); the
  // threads may write slot q once q < free_upto, i.e. once slot q - kRing's DMA has completed.
  // Every wait blocks (condition variables, blocking-sync events): spinning threads would eat the
  // process's CPU share that the caller's thread and the lanes' threads need.
  struct U16Ring {
    static constexpr int kRing = 4;
    static constexpr size_t kSlotCounts = size_t(4) << 20;
    unsigned short* pin = nullptr;  // kRing slots
    unsigned short* dev = nullptr;  // kRing device slots (widened from)
    hipEvent_t ev[kRing] = {};
    long long seq = 0;     // next sequence number
    long long issued = 0;  // slots whose DMA is queued
    long long free_upto = kRing;  // (under m, as fin and abort)
    int fin[kRing] = {};
    static constexpr int kMaxT = 32;
    std::vector<int2> exc[kRing][kMaxT];  // per ring slot and thread: (index in the slot, count)
    std::vector<int2> exc_all;            // one slot's list, uploaded
    bool abort = false;
    std::vector<std::thread> th;
    int T = 0;
    std::mutex m;
    std::condition_variable cv, cvd, cvf;  // job / job done, slot freed / slot narrowed
    long long job = 0;
    int busy = 0;
    bool stop = false;
    const int* src = nullptr;
    size_t n = 0;
    long long q0 = 0;
    int nslots = 0;
    double st_wait_ms = 0, st_issue_ms = 0, st_free_ms = 0;  // issuer: narrowing waits, copy issue, slot frees
  } u16;
  // statistics (scde_ctx_get_stat)
  double st_skip_slabs = 0, st_skip_kept = 0, st_skip_stretches = 0, st_skip_redo = 0, st_degen = 0;
  // host wall time of scde_expression_difference_{dev,host} phases (ms, summed over calls):
  // setup, unique tables (incl. their syncs), posteriors enqueued, ratio + results read back
  double st_host_ms[4] = {0, 0, 0, 0};
  // arithmetic the bootstrap kernels issued (skip_stats runs): FP64 lane FMAs of k_boot2 (kept
  // stretches x 64 lanes x slab boots x entries)
  double st_boot_f64_fma = 0;
  double st_stream_syncs = 0;  // grow(keep) drains of this context's streams (scoped, never the device)
  double st_arena_syncs = 0;   // pinned-arena wraps (this context's streams drained)
  // run_posterior's pieces (host ms): waiting for a piece's upload, then its unique build and tables launch
  double st_piece_wait_ms = 0, st_piece_host_ms = 0;
  double st_pair_redo = 0;  // slabs a pair pass of k_boot_tiles left to the four-tile list pass
  double st_boot_path = -1;  // the bootstrap kernel of the last posterior: 0 k_boot2, 1 k_boot_tiles, 3 general
  static constexpr int kQMaxTilesHost = 28;
  double st_tile_hist[kQMaxTilesHost + 1] = {0};
  // ucl/uci of a cell subset (R/functions.R:609-610); one set per group so both groups'
  // unique tables can be built up front, with their host syncs, before the heavy kernels
  struct UniqueSet {
    Buf cellidx, cmax, cmin, woff, bits, rank, nuniq, ucl, ucl_off, uci, flags;
    std::vector<int> cmax_h, cmin_h, nuniq_h;
    std::vector<long long> woff_h, ucl_off_h;
    // pinned landing area of the phases' device -> host size read-backs: the set's own (not
    // the shared staging arena), so no later staging can recycle it before the host reads it
    int fixed_flags = 0;  // unique_phase12_fixed's flags when no pinned landing area exists
    int woff_fixed = 0;   // entries of woff holding the fixed offsets c * fixed_words (0: other contents)
    // bitmap words per cell of the fixed-width build: 1024 (counts below 65,536), widened to the
    // power of two an exact rebuild needed (so a data set with larger counts pays the rebuild's two
    // extra host syncs once, not on every call), at most kUniqueFixedWordsMax
    long long fixed_words = 1024;
    long long woff_fixed_w = 0;  // the width woff_fixed's offsets were uploaded for
    int* pin_land = nullptr;
    size_t pin_land_cap = 0;  // ints
    const int* pin_in = nullptr;  // this phase's read-back (pin_land, or null: pageable fallback)
    std::vector<int4> tasks_h;  // cell-staged tables tasks (k_tables_cell)
    Buf tasks;
    bool ready = false;
    // a piece of a larger set (run_posterior's pieces): phase 3 writes the unique counts into
    // into->ucl from column into_col0 on (grown to an estimate of the whole set's columns,
    // into_cap_hint) and the count indices into into->uci from cell into_c0 on; its own ucl_off
    // (from 0) serves the piece's tables launch
    UniqueSet* into = nullptr;
    long long into_col0 = 0, into_cap_hint = 0;
    int into_c0 = 0;
    int* landing(size_t n) {
      if (n > pin_land_cap) {
        if (pin_land) (void)hipHostFree(pin_land);
        pin_land = nullptr;
        pin_land_cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&pin_land), sizeof(int) * n, hipHostMallocDefault) != hipSuccess) {
          pin_land = nullptr;
          (void)hipGetLastError();
          return nullptr;
        }
        pin_land_cap = n;
      }
      return pin_land;
    }
    void release() {
      Buf* b[] = {&cellidx, &cmax, &cmin, &woff, &bits, &rank, &nuniq, &ucl, &ucl_off, &uci, &flags, &tasks};
      for (Buf* x : b) x->release();
      woff_fixed = 0;
      if (pin_land) (void)hipHostFree(pin_land);
      pin_land = nullptr;
      pin_land_cap = 0;
    }
  } us[3];
  static constexpr int kMaxPieces = 8;
  UniqueSet upc[kMaxPieces];  // run_posterior's pieces
  UniqueSet task_us;          // run_posterior's tables tasks (unpieced): per context, so lanes sharing a
                              // unique set never write one tasks buffer
  // profiling
  bool profile = false;
  struct Pending {
    int slot;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> evpool;
  double ms[NSLOTS] = {0};
  long long launches[NSLOTS] = {0};
  std::vector<void*> user_allocs;

  hipEvent_t get_event() {
    if (!evpool.empty()) {
      hipEvent_t e = evpool.back();
      evpool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  hipEvent_t mark_begin(int slot) {
    if (!profile) return nullptr;
    hipEvent_t a = get_event();
    (void)hipEventRecord(a, stream);
    (void)slot;
    return a;
  }
  void mark_end(int slot, hipEvent_t a) {
    if (!profile || !a) return;
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, stream);
    pending.push_back({slot, a, b});
  }
  int sync() {
    HCHK(hipStreamSynchronize(stream));
    if (peer) {  // the peer lane's timings count as this context's
      RCHK(peer->sync());
      for (int i = 0; i < NSLOTS; ++i) {
        ms[i] += peer->ms[i];
        launches[i] += peer->launches[i];
        peer->ms[i] = 0;
        peer->launches[i] = 0;
      }
    }
    for (auto& p : pending) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
        ms[p.slot] += t;
        launches[p.slot] += 1;
      }
      evpool.push_back(p.a);
      evpool.push_back(p.b);
    }
    pending.clear();
    return SCDE_OK;
  }
  ~scde_ctx() {
    if (dnl.th.joinable()) {
      {
        std::lock_guard<std::mutex> lk(dnl.m);
        dnl.stop = true;
      }
      dnl.cv.notify_all();
      dnl.th.join();
    }
    for (auto e : dnl.evs) (void)hipEventDestroy(e);
    if (dnl.stream) (void)hipStreamDestroy(dnl.stream);
    if (upl.th.joinable()) {
      {
        std::lock_guard<std::mutex> lk(upl.m);
        upl.stop = true;
      }
      upl.cv.notify_all();
      upl.th.join();
    }
    if (!u16.th.empty()) {  // (after the upload worker, its only user)
      {
        std::lock_guard<std::mutex> lk(u16.m);
        u16.stop = true;
      }
      u16.cv.notify_all();
      for (auto& t : u16.th) t.join();
    }
    if (u16.pin) (void)hipHostFree(u16.pin);
    if (u16.dev) (void)hipFree(u16.dev);
    for (auto& e : u16.ev)
      if (e) (void)hipEventDestroy(e);
    if (peer) {
      (void)hipStreamSynchronize(peer->stream);
      delete peer;
    }
    for (auto& e : lane_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : piece_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : piece_up_ev)
      if (e) (void)hipEventDestroy(e);
    if (uq_stream) (void)hipStreamDestroy(uq_stream);
    Buf* all[] = {&models, &mag, &mu,  &lcfp, &cfp, &lcfpr, &theta,  &cellscal, &pq, &colc, &T,      &E,      &maxi,
                  &has_clamp, &base_col, &zcol, &ent, &nnz, &Wt, &Z, &draws, &degen, &wset, &prior_y, &diffv,
                  &jpA,    &jpB, &res,   &ratio, &in1, &in2, &outbuf, &part, &bhw, &ubound, &zubound, &smask, &subuf, &sredo};
    for (Buf* b : all) b->release();
    Buf* wp[] = {&wp_probs, &wp_blocks,  &wp_kidx, &wp_cols,   &wp_perms, &wp_starts, &wp_scratch,
                 &wp_stat,  &wp_out,     &wp_smooth, &wp_M,    &wp_W,     &pr_cell,   &pr_part,
                 &pr_occ,   &pr_stats,   &pr_hist, &pr_work,   &pr_out,   &pr_v,      &pr_sorted, &pr_sortw,
                 &pg_a,     &pg_b,       &pg_c,    &pg_d,      &pg_e,      &counts_in, &w8,
                 &w8t,      &w8g,      &qflags,  &gkey,     &gkey2,    &gidx,     &gorder,  &gwork,   &pmask,  &pwide,  &ellw,  &excd, &gdone};
    for (Buf* b : wp) b->release();
    for (auto& u : us) u.release();
    for (auto& u : upc) u.release();
    task_us.release();
    for (void* p : user_allocs) (void)hipFree(p);
    for (auto& p : pending) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (auto e : evpool) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    if (uq_ev) (void)hipEventDestroy(uq_ev);
    if (modes_ev) (void)hipEventDestroy(modes_ev);
    if (p1_ev) (void)hipEventDestroy(p1_ev);
    if (aux_ev) (void)hipEventDestroy(aux_ev);
    if (aux_stream) (void)hipStreamDestroy(aux_stream);
    if (pin) (void)hipHostFree(pin);
    for (auto& e : up_ev)
      if (e) (void)hipEventDestroy(e);
  }
};

// test hook (scde_ctx_inject_fault "handoff_spin"): a spin kernel on the producing stream before every
// event another stream or host thread waits on -- a missing wait then shows as wrong results every time
static hipError_t handoff_spin(scde_ctx* cx, hipStream_t s) {
  if (cx->spin_cycles <= 0) return hipSuccess;
  ++cx->st_spins;
  return launch_spin(s, cx->spin_cycles);
}
// Every cross-stream wait: stream s waits for ev, then (handoff_spin hook) spins -- the work s
// queues next, the producer side of later handoffs, starts late, so a consumer elsewhere that
// misses its wait on that work reads it before it is written every time.  (The spin before each
// event record delays the signal as well.)
static hipError_t handoff_wait(scde_ctx* cx, hipStream_t s, hipEvent_t ev) {
  hipError_t e = hipStreamWaitEvent(s, ev, 0);
  if (e == hipSuccess) e = handoff_spin(cx, s);
  return e;
}
// The main stream's wait for the peer lane's posterior (lane_ev[1]) before the ratio.  Test hook
// "skip_lane_join": the next `count` DE calls leave it out -- the negative control of the ordering
// tests (with the spins, the ratio then reads the second group's joint posterior unwritten).
static hipError_t lane_join(scde_ctx* ctx) {
  if (ctx->fault_skip_join > 0) {
    --ctx->fault_skip_join;
    return hipSuccess;
  }
  return handoff_wait(ctx, ctx->stream, ctx->lane_ev[1]);
}

// Downloader: queue a read-back of `height` rows of `width` bytes (pitches in bytes) after the work
// queued so far on `after`; dnl_wait returns once every queued read-back has landed (or failed).
int dnl_push(scde_ctx* cx, hipStream_t after, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
             size_t height) {
  auto& d = cx->dnl;
  if (!d.th.joinable()) {
    HCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    d.th = std::thread([cx] {
      auto& q = cx->dnl;
      (void)hipSetDevice(cx->device);
      std::unique_lock<std::mutex> lk(q.m);
      for (;;) {
        q.cv.wait(lk, [&] { return q.stop || (!q.q.empty() && !q.hold); });
        if (q.stop) return;
        const scde_ctx::Downloader::Job j = q.q.front();
        q.q.pop_front();
        const hipEvent_t ev = q.evs[j.ev];
        lk.unlock();
        hipError_t e = hipEventSynchronize(ev);
        if (e == hipSuccess)
          e = hipMemcpy2DAsync(j.dst, j.dpitch, j.src, j.spitch, j.width, j.height, hipMemcpyDeviceToHost, q.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(q.stream);
        lk.lock();
        if (e != hipSuccess && !q.err) {
          q.err = SCDE_EHIP;
          q.err_msg = hipGetErrorString(e);
        }
        if (--q.pending == 0) q.cvd.notify_all();
      }
    });
  }
  std::lock_guard<std::mutex> lk(d.m);
  if (d.nev == (int)d.evs.size()) {  // one event per job of a call (reused once dnl_wait drained them)
    hipEvent_t e = nullptr;
    // blocking sync: the read-back thread's hipEventSynchronize sleeps instead of spinning through
    // the tables and the bootstrap (the lanes' threads need the CPU share)
    HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync));
    d.evs.push_back(e);
  }
  const int ei = d.nev++;
  HCHK(handoff_spin(cx, after));
  HCHK(hipEventRecord(d.evs[ei], after));
  d.q.push_back({ei, dst, src, dpitch, spitch, width, height});
  ++d.pending;
  d.cv.notify_all();
  return SCDE_OK;
}

// hold queued read-backs back (on) or let them run (off)
void dnl_hold(scde_ctx* cx, bool on) {
  auto& d = cx->dnl;
  {
    std::lock_guard<std::mutex> lk(d.m);
    d.hold = on;
  }
  d.cv.notify_all();
}

int dnl_wait(scde_ctx* cx) {
  auto& d = cx->dnl;
  dnl_hold(cx, false);
  std::unique_lock<std::mutex> lk(d.m);
  d.cvd.wait(lk, [&] { return d.pending == 0; });
  d.nev = 0;
  const int err = d.err;
  const std::string msg = d.err_msg;
  d.err = 0;
  d.err_msg.clear();
  lk.unlock();
  return err ? fail(err, "read-back failed: %s", msg.c_str()) : SCDE_OK;
}

// every stream of the context that touches its workspace (grow(keep) drains these, not the device)
hipError_t ctx_streams_sync(scde_ctx* cx) {
  for (hipStream_t st : {cx->stream, cx->home_stream, cx->copy_stream, cx->aux_stream, cx->uq_stream}) {
    if (!st) continue;
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
  }
  cx->st_stream_syncs += 1;
  return hipSuccess;
}

namespace {

// ------------------------------------------------------------------ posterior spec
struct PostSpec {
  int ncells = 0;
  const double* models = nullptr;  // host ncells x 12 col-major
  int localtheta = 0, squarelogit = 0;
  const double* mag = nullptr;  // host G
  int G = 0;
  int nboot = 0;
  int postflag = 0;
  int ensemble = 0;
  bool batch_call = false;  // logBootBatchPosterior semantics
  // source A: host ucl/uci
  const int* ucl_host = nullptr;
  const int64_t* ucl_off_host = nullptr;
  const int* uci_host = nullptr;
  // source B: device counts
  const int* counts_dev = nullptr;
  long long ld = 0;
  const int* cellidx_host = nullptr;
  int ngenes = 0;
  // seeding: per set seed, per gene set (empty -> all set 0)
  std::vector<int> seeds;
  std::vector<int> wset;
  // batch
  const int* batch_vals = nullptr;
  const int64_t* batch_off = nullptr;
  const int* comp = nullptr;
  int nbatch = 0;
  // outputs (device)
  double* jp = nullptr;
  long long jp_g = 0, jp_k = 0;
  double* modes = nullptr;  // ngenes x ncells col-major
  bool modes_early = false;  // modes right after the tables, with cx->modes_ev recorded (copy_modes_out)
  double* post = nullptr;   // ncells blocks of ngenes x G col-major
  bool use_baseline = true;
  int rand_kind = 0;
  // counts arriving in pieces (de_run's host-count pipeline): piece j holds this spec's cells
  // [piece_c[j], piece_c[j + 1]) and is in HBM once piece_ready(j) returned and piece_stream
  // reached the point it recorded; run_posterior builds each piece's unique sets on
  // piece_stream and launches its tables as it arrives (piece_ev: one event per piece)
  int npieces = 0;
  const int* piece_c = nullptr;
  std::function<int(int)> piece_ready;
  hipStream_t piece_stream = nullptr;
  hipEvent_t* piece_ev = nullptr;
  // host destinations read back by the context's Downloader while later work runs (the caller then
  // copies neither and drains the Downloader before returning): modes_host, the modes matrix
  // (pieces: each piece's columns once its tables are done); jp_host, the joint posterior in R's
  // layout (jp_g = 1, jp_k = ngenes) -- with the gene-block bootstrap in jp_chunks gene chunks, each
  // chunk's rows read back while the next chunk's bootstrap runs
  double* modes_host = nullptr;
  double* jp_host = nullptr;
  int jp_chunks = 1;
};

constexpr size_t kPinCap = size_t(16) << 20;  // the arena
constexpr size_t kPinMax = size_t(2) << 20;   // larger transfers go direct

// `bytes` of the context's pinned arena (nullptr: too large, or the pinned allocation failed)
char* pin_alloc(scde_ctx* cx, size_t bytes) {
  if (bytes > kPinMax) return nullptr;
  if (!cx->pin) {
    if (hipHostMalloc(reinterpret_cast<void**>(&cx->pin), kPinCap, hipHostMallocDefault) != hipSuccess) {
      cx->pin = nullptr;
      (void)hipGetLastError();
      return nullptr;
    }
    cx->pin_off = 0;
  }
  size_t off = (cx->pin_off + 255) & ~size_t(255);
  if (off + bytes > kPinCap) {
    // reuse from the start: every host -> device copy staged so far must have been read out of
    // the arena first; they are issued on the context's own streams only (device -> host
    // read-backs land in each unique set's own area, never here)
    if (hipStreamSynchronize(cx->stream) != hipSuccess) return nullptr;
    if (cx->home_stream && hipStreamSynchronize(cx->home_stream) != hipSuccess) return nullptr;
    if (cx->copy_stream && hipStreamSynchronize(cx->copy_stream) != hipSuccess) return nullptr;
    if (cx->aux_stream && hipStreamSynchronize(cx->aux_stream) != hipSuccess) return nullptr;
    if (cx->uq_stream && hipStreamSynchronize(cx->uq_stream) != hipSuccess) return nullptr;
    cx->st_arena_syncs += 1;
    off = 0;
  }
  cx->pin_off = off + bytes;
  return cx->pin + off;
}

int upload_on(scde_ctx* cx, Buf& b, const void* src, size_t bytes, hipStream_t st) {
  HCHK(b.ensure(bytes));
  if (!bytes) return SCDE_OK;
  if (char* h = pin_alloc(cx, bytes)) {
    std::memcpy(h, src, bytes);
    src = h;
  }
  HCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, st));
  return SCDE_OK;
}
int upload(scde_ctx* cx, Buf& b, const void* src, size_t bytes) { return upload_on(cx, b, src, bytes, cx->stream); }

// Build ucl/uci for the selected cells on device (R/functions.R:609-610).  Unique
// counts come out sorted ascending rather than in first-appearance order; the order
// only permutes table columns, never values.  Three phases separated by host syncs
// (bitmap sizes need the per-cell maxima; column offsets need the unique counts);
// build_unique_pair interleaves two groups' phases so a DE call syncs twice, not four
// times, and before any heavy kernel is queued.
using UniqueSet = scde_ctx::UniqueSet;
constexpr long long kUniqueFixedWordsMax = 1 << 16;           // counts below 2^22
constexpr double kUniqueFixedBytesMax = double(256 << 20);    // a set's fixed-width bitmaps

int unique_phase1(scde_ctx* cx, const PostSpec& s, UniqueSet& u) {
  const int C = s.ncells, N = s.ngenes;
  hipStream_t st = cx->stream;
  RCHK(upload(cx, u.cellidx, s.cellidx_host, sizeof(int) * C));
  HCHK(u.cmax.ensure(sizeof(int) * C));
  HCHK(u.cmin.ensure(sizeof(int) * C));
  HCHK(launch_cell_minmax(s.counts_dev, s.ld, 0, N, C, u.cellidx.as<int>(), u.cmax.as<int>(), u.cmin.as<int>(), st));
  u.cmax_h.assign(C, 0);
  u.cmin_h.assign(C, 0);
  int* h = u.landing(2 * (size_t)C);
  u.pin_in = h;
  HCHK(hipMemcpyAsync(h ? h : u.cmax_h.data(), u.cmax.p, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  HCHK(hipMemcpyAsync(h ? h + C : u.cmin_h.data(), u.cmin.p, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  return SCDE_OK;
}

int unique_phase2(scde_ctx* cx, const PostSpec& s, UniqueSet& u) {
  const int C = s.ncells, N = s.ngenes;
  hipStream_t st = cx->stream;
  if (u.pin_in) {  // landed (the caller synchronised)
    std::copy(u.pin_in, u.pin_in + C, u.cmax_h.begin());
    std::copy(u.pin_in + C, u.pin_in + 2 * (size_t)C, u.cmin_h.begin());
  }
  u.woff_h.assign(C + 1, 0);
  long long wmax = 1;
  for (int c = 0; c < C; ++c) {
    if (N > 0 && u.cmin_h[c] < 0) return fail(SCDE_EARG, "negative count in cell %d", c);
    u.woff_h[c + 1] = u.woff_h[c] + ((long long)u.cmax_h[c] >> 6) + 1;
    wmax = std::max(wmax, ((long long)u.cmax_h[c] >> 6) + 1);
  }
  // the next fixed-width build of this set: wide enough for these counts (bounded bitmap memory)
  long long fw = u.fixed_words;
  while (fw < wmax && fw < kUniqueFixedWordsMax) fw *= 2;
  if (fw >= wmax && fw != u.fixed_words && (double)C * fw * 8.0 <= kUniqueFixedBytesMax) u.fixed_words = fw;
  RCHK(upload(cx, u.woff, u.woff_h.data(), sizeof(long long) * (C + 1)));
  u.woff_fixed = 0;
  HCHK(u.bits.ensure(sizeof(unsigned long long) * u.woff_h[C]));
  HCHK(hipMemsetAsync(u.bits.p, 0, sizeof(unsigned long long) * u.woff_h[C], st));
  HCHK(launch_mark(s.counts_dev, s.ld, 0, N, C, u.cellidx.as<int>(), u.woff.as<long long>(),
                   u.bits.as<unsigned long long>(), st));
  HCHK(u.rank.ensure(sizeof(int) * u.woff_h[C]));
  HCHK(u.nuniq.ensure(sizeof(int) * C));
  HCHK(launch_rank(u.bits.as<unsigned long long>(), u.woff.as<long long>(), C, u.rank.as<int>(),
                   u.nuniq.as<int>(), st));
  u.nuniq_h.assign(C, 0);
  int* h = u.landing(2 * (size_t)C);  // phase 1's values were copied out by now
  u.pin_in = h;
  HCHK(hipMemcpyAsync(h ? h : u.nuniq_h.data(), u.nuniq.p, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  return SCDE_OK;
}

int unique_phase3(scde_ctx* cx, const PostSpec& s, UniqueSet& u) {
  const int C = s.ncells, N = s.ngenes;
  hipStream_t st = cx->stream;
  if (u.pin_in) std::copy(u.pin_in, u.pin_in + C, u.nuniq_h.begin());
  u.ucl_off_h.assign(C + 1, 0);
  for (int c = 0; c < C; ++c) u.ucl_off_h[c + 1] = u.ucl_off_h[c] + u.nuniq_h[c];
  RCHK(upload(cx, u.ucl_off, u.ucl_off_h.data(), sizeof(long long) * (C + 1)));
  int* ucl = nullptr;
  int* uci = nullptr;
  if (u.into) {  // a piece: into the whole set's arrays (uci sized by the caller)
    const long long need = std::max(u.into_col0 + u.ucl_off_h[C], u.into_cap_hint);
    auto cx_sync = [cx] { return ctx_streams_sync(cx); };
    HCHK(u.into->ucl.grow(u.into_col0 > 0, sizeof(int) * std::max<long long>(1, need), cx_sync));
    ucl = u.into->ucl.as<int>() + u.into_col0;
    uci = u.into->uci.as<int>() + (size_t)N * u.into_c0;
  } else {
    HCHK(u.ucl.ensure(sizeof(int) * std::max<long long>(1, u.ucl_off_h[C])));
    HCHK(u.uci.ensure(sizeof(int) * std::max<long long>(1, (long long)N * C)));
    ucl = u.ucl.as<int>();
    uci = u.uci.as<int>();
  }
  HCHK(launch_fill_ucl(u.bits.as<unsigned long long>(), u.woff.as<long long>(), C, u.rank.as<int>(),
                       u.ucl_off.as<long long>(), ucl, st));
  HCHK(launch_uci(s.counts_dev, s.ld, 0, N, C, u.cellidx.as<int>(), u.woff.as<long long>(),
                  u.bits.as<unsigned long long>(), u.rank.as<int>(), uci, st));
  u.ready = true;
  return SCDE_OK;
}

// Phases 1 and 2 in one, without the per-cell maxima: every cell gets a bitmap of
// u.fixed_words words (1024 at first: counts below 65,536); k_mark flags a negative count or one
// past the bitmap, and such a set is rebuilt with exact widths (phases 1-2), which also widens
// the set's later fixed builds.  One host sync per build.
int unique_phase12_fixed(scde_ctx* cx, const PostSpec& s, UniqueSet& u) {
  const int C = s.ncells, N = s.ngenes;
  hipStream_t st = cx->stream;
  RCHK(upload(cx, u.cellidx, s.cellidx_host, sizeof(int) * C));
  const long long FW = u.fixed_words;
  u.woff_h.resize(C + 1);
  for (int c = 0; c <= C; ++c) u.woff_h[c] = (long long)c * FW;
  // the fixed offsets c * FW are uploaded once per set and width (grow-only; exact-width builds
  // and a new width reset it)
  if (u.woff_fixed_w != FW) u.woff_fixed = 0;
  u.woff_fixed_w = FW;
  if (u.woff_fixed < C + 1) {
    RCHK(upload(cx, u.woff, u.woff_h.data(), sizeof(long long) * (C + 1)));
    u.woff_fixed = C + 1;
  }
  // one memset for the bitmaps and k_mark's flag word after them
  HCHK(u.bits.ensure(sizeof(unsigned long long) * (u.woff_h[C] + 1)));
  HCHK(hipMemsetAsync(u.bits.p, 0, sizeof(unsigned long long) * (u.woff_h[C] + 1), st));
  int* flags = reinterpret_cast<int*>(u.bits.as<unsigned long long>() + u.woff_h[C]);
  HCHK(launch_mark(s.counts_dev, s.ld, 0, N, C, u.cellidx.as<int>(), u.woff.as<long long>(),
                   u.bits.as<unsigned long long>(), st, flags));
  HCHK(u.rank.ensure(sizeof(int) * u.woff_h[C]));
  HCHK(u.nuniq.ensure(sizeof(int) * (C + 1)));
  HCHK(launch_rank(u.bits.as<unsigned long long>(), u.woff.as<long long>(), C, u.rank.as<int>(),
                   u.nuniq.as<int>(), st, flags, u.nuniq.as<int>() + C));
  u.nuniq_h.assign(C, 0);
  u.fixed_flags = 0;
  int* h = u.landing(2 * (size_t)C + 1);
  u.pin_in = h;
  // the unique counts and the flags (nuniq[C]) in one read-back
  if (h) {
    HCHK(hipMemcpyAsync(h, u.nuniq.p, sizeof(int) * (C + 1), hipMemcpyDeviceToHost, st));
  } else {
    HCHK(hipMemcpyAsync(u.nuniq_h.data(), u.nuniq.p, sizeof(int) * C, hipMemcpyDeviceToHost, st));
    HCHK(hipMemcpyAsync(&u.fixed_flags, u.nuniq.as<int>() + C, sizeof(int), hipMemcpyDeviceToHost, st));
  }
  return SCDE_OK;
}

// ns (1 or 2) cell subsets of the same device counts
int build_unique_sets(scde_ctx* cx, const PostSpec* const* s, UniqueSet* const* u, int ns) {
  hipEvent_t ev = cx->mark_begin(SLOT_UNIQUE);
  if (ns < 1 || ns > 4) return fail(SCDE_EINTERNAL, "unique sets per build: 1..4");
  bool exact[4] = {true, true, true, true};
  if (cx->opt_unique_fixed) {
    for (int i = 0; i < ns; ++i) RCHK(unique_phase12_fixed(cx, *s[i], *u[i]));
    HCHK(hipStreamSynchronize(cx->stream));
    for (int i = 0; i < ns; ++i) {
      const int fl = u[i]->pin_in ? u[i]->pin_in[s[i]->ncells] : u[i]->fixed_flags;
      exact[i] = fl != 0;  // a count outside [0, 65536): the exact build (and its error message)
    }
  }
  bool any_exact = false;
  for (int i = 0; i < ns; ++i) any_exact = any_exact || exact[i];
  if (any_exact) {
    for (int i = 0; i < ns; ++i)
      if (exact[i]) RCHK(unique_phase1(cx, *s[i], *u[i]));
    HCHK(hipStreamSynchronize(cx->stream));
    for (int i = 0; i < ns; ++i)
      if (exact[i]) RCHK(unique_phase2(cx, *s[i], *u[i]));
    HCHK(hipStreamSynchronize(cx->stream));
  }
  for (int i = 0; i < ns; ++i) RCHK(unique_phase3(cx, *s[i], *u[i]));
  cx->mark_end(SLOT_UNIQUE, ev);
  return SCDE_OK;
}

// The draw lists alone (cell per draw) and the largest multiplicity of a cell in one boot.
void make_draws_lists(const PostSpec& s, std::vector<int>& draws, int& ndraw, int* maxw) {
  const int C = s.ncells, B = s.nboot, nsets = (int)s.seeds.size();
  if (s.batch_call) {
    ndraw = 0;
    for (int k = 0; k < s.nbatch; ++k) ndraw += std::max(0, s.comp[k]);
  } else {
    ndraw = C;
  }
  const size_t per = (size_t)B * std::max(ndraw, 1);
  draws.assign((size_t)nsets * per, -1);
  std::vector<int> hist((size_t)std::max(C, 1), 0);
  int mx = 0;
  for (int set = 0; set < nsets; ++set) {
    PlatformRand rng((unsigned int)s.seeds[set], s.rand_kind);
    int* dr = draws.data() + (size_t)set * per;
    const int c0 = 0, n = C;
    for (int b = 0; b < B; ++b) {
      int* row = dr + (size_t)b * ndraw;
      int d = 0;
      if (!s.batch_call) {
        for (int j = 0; j < n; ++j) row[d++] = c0 + rng.draw(n);
      } else {
        for (int k = 0; k < s.nbatch; ++k) {
          const int* bi = s.batch_vals + s.batch_off[k];
          const int nbk = (int)(s.batch_off[k + 1] - s.batch_off[k]);
          for (int j = 0; j < s.comp[k]; ++j) row[d++] = bi[rng.draw(nbk)];
        }
      }
      for (int j = 0; j < d; ++j) mx = std::max(mx, ++hist[row[j]]);
      for (int j = 0; j < d; ++j) hist[row[j]] = 0;
    }
  }
  if (maxw) *maxw = mx;
}

// Draw lists and per-cell multiplicities for each seed set.  want_W false: the multiplicities are
// left to the device (launch_mult); only their maximum is formed here (*maxw), from a per-boot
// count of the cells drawn.
void make_draws(const PostSpec& s, int Bp, std::vector<int>& draws, std::vector<double>& W, int& ndraw,
                int* maxw = nullptr, bool want_W = true) {
  const int C = s.ncells, B = s.nboot, nsets = (int)s.seeds.size();
  if (!want_W) {
    make_draws_lists(s, draws, ndraw, maxw);
    return;
  }
  if (s.batch_call) {
    ndraw = 0;
    for (int k = 0; k < s.nbatch; ++k) ndraw += std::max(0, s.comp[k]);
  } else {
    ndraw = C;
  }
  draws.assign((size_t)nsets * B * std::max(ndraw, 1), 0);
  W.assign((size_t)nsets * C * Bp, 0.0);
  for (int set = 0; set < nsets; ++set) {
    PlatformRand rng((unsigned int)s.seeds[set], s.rand_kind);
    int* dr = draws.data() + (size_t)set * B * std::max(ndraw, 1);
    double* w = W.data() + (size_t)set * C * Bp;
    for (int b = 0; b < B; ++b) {
      int d = 0;
      if (!s.batch_call) {
        for (int j = 0; j < C; ++j) {
          const int rj = rng.draw(C);
          dr[(size_t)b * ndraw + d++] = rj;
          w[(size_t)rj * Bp + b] += 1.0;
        }
      } else {
        for (int k = 0; k < s.nbatch; ++k) {
          const int nsamp = s.comp[k];
          if (nsamp > 0) {
            const int* bi = s.batch_vals + s.batch_off[k];
            const int nb = (int)(s.batch_off[k + 1] - s.batch_off[k]);
            for (int j = 0; j < nsamp; ++j) {
              const int cell = bi[rng.draw(nb)];
              dr[(size_t)b * ndraw + d++] = cell;
              w[(size_t)cell * Bp + b] += 1.0;
            }
          }
        }
      }
    }
  }
}

// rest (nullable): return once the tables are queued, with the remaining work (modes, draws,
// bootstrap, outputs) in *rest, to be run later on the same stream -- de_run queues both groups'
// tables before either bootstrap, so the second lane's tables start at once

int run_posterior(scde_ctx* cx, const PostSpec& s, UniqueSet& u, std::function<int()>* rest = nullptr) {
  const int C = s.ncells, G = s.G, N = s.ngenes;
  // cells per call of the kernel choices, the widest cell list (ELL rows), the bootstrap's genes
  const int Ccall = C, Cmax = C, NBg = N;
  // column stride: >= the k_boot2 block (lanes never read past a column); 512 keeps
  // columns 4 KiB-aligned
  const int GS = G <= 448 ? 512 : (int)round_up(G, 64);
  hipStream_t st = cx->stream;
  if (C <= 0 || G <= 0) return fail(SCDE_EARG, "ncells and ngrid must be positive");
  if (s.nboot < 0) return fail(SCDE_EARG, "nboot must be >= 0");
  if (G > 4096) return fail(SCDE_EARG, "ngrid > 4096 unsupported");
  if (s.seeds.empty()) return fail(SCDE_EINTERNAL, "no seed sets");
  if (s.batch_call) {
    for (int k = 0; k < s.nbatch; ++k) {
      if (s.comp[k] < 0) return fail(SCDE_EARG, "negative composition");
      if (s.comp[k] > 0 && s.batch_off[k + 1] - s.batch_off[k] <= 0)
        return fail(SCDE_EARG, "batch %d has draws but no cells", k);
      for (int64_t i = s.batch_off[k]; i < s.batch_off[k + 1]; ++i)
        if (s.batch_vals[i] < 0 || s.batch_vals[i] >= C) return fail(SCDE_EARG, "BatchIL index out of range");
    }
  }
  // ---- per-cell grid vectors
  RCHK(upload(cx, cx->models, s.models, sizeof(double) * C * 12));
  RCHK(upload(cx, cx->mag, s.mag, sizeof(double) * G));
  const size_t cg = sizeof(double) * (size_t)C * GS;
  HCHK(cx->mu.ensure(cg));
  HCHK(cx->lcfp.ensure(cg));
  HCHK(cx->cfp.ensure(cg));
  HCHK(cx->lcfpr.ensure(cg));
  HCHK(cx->theta.ensure(cg));
  HCHK(cx->cellscal.ensure(sizeof(double) * 2 * C));
  hipEvent_t ev = cx->mark_begin(SLOT_OTHER);
  if (!s.localtheta) HCHK(cx->pq.ensure(4 * cg));
  HCHK(launch_cell_prep(cx->models.as<double>(), C, G, GS, cx->mag.as<double>(), s.localtheta, s.squarelogit,
                        cx->mu.as<double>(), cx->lcfp.as<double>(), cx->lcfpr.as<double>(), cx->theta.as<double>(),
                        cx->cellscal.as<double>(), s.localtheta ? nullptr : cx->pq.as<double>(), st,
                        cx->cfp.as<double>()));
  cx->mark_end(SLOT_OTHER, ev);
  // ---- unique counts (prebuilt by build_unique_sets when u.ready; piece by piece with the
  // tables below when the counts arrive in pieces)
  std::vector<long long>& ucl_off_h = u.ucl_off_h;
  const bool pieces = s.npieces > 0 && !s.ucl_host;
  if (s.ucl_host) {
    ucl_off_h.assign(s.ucl_off_host, s.ucl_off_host + C + 1);
    if (ucl_off_h[0] != 0) return fail(SCDE_EARG, "ucl_off[0] must be 0");
    for (int c = 0; c < C; ++c)
      if (ucl_off_h[c + 1] < ucl_off_h[c]) return fail(SCDE_EARG, "ucl_off must be non-decreasing");
    RCHK(upload(cx, u.ucl_off, ucl_off_h.data(), sizeof(long long) * (C + 1)));
    RCHK(upload(cx, u.ucl, s.ucl_host, sizeof(int) * std::max<long long>(1, ucl_off_h[C])));
    // validate counti against the per-cell list sizes (the reference would read out of bounds)
    for (int c = 0; c < C; ++c) {
      const long long nu = ucl_off_h[c + 1] - ucl_off_h[c];
      const int* col = s.uci_host + (size_t)N * c;
      for (int g = 0; g < N; ++g)
        if (col[g] < 0 || col[g] >= nu) return fail(SCDE_EARG, "counti[%d,%d]=%d out of range [0,%lld)", g, c, col[g], nu);
    }
    RCHK(upload(cx, u.uci, s.uci_host, sizeof(int) * std::max<long long>(1, (long long)N * C)));
  } else if (!u.ready && !pieces) {
    const PostSpec* sp[1] = {&s};
    UniqueSet* up[1] = {&u};
    RCHK(build_unique_sets(cx, sp, up, 1));
  }
  u.ready = false;  // consumed by this call
  // ---- K1 tables
  // Bootstrap path with G <= 1024 (k_boot2): the tables kernel writes the baseline-delta
  // columns D directly (phase 1: count-0 columns and base_col, phase 2: the rest); T itself
  // is kept only when individual posteriors are returned.
  const bool boot_path = s.nboot > 0 && (s.batch_call || !s.ensemble);
  // the launch plan; its column-count conditions are checked again once the count is known
  // (pieces: the tables launch piece by piece before the last piece has arrived)
  struct Plan {
    bool fast, fused, keep_T, tpath, stretch_skip;
    bool operator==(const Plan& o) const {
      return fast == o.fast && fused == o.fused && keep_T == o.keep_T && tpath == o.tpath &&
             stretch_skip == o.stretch_skip;
    }
  };
  const bool want_post = s.batch_call ? (s.postflag == 2) : (s.postflag == 2 || s.postflag == 3);
  // k_boot2 forms column and multiplicity-row offsets in 32 bits: past that, the general kernel
  auto make_plan = [&](long long nc) {
    Plan p{};
    p.fast = ((G + 63) / 64) * 64 <= 1024 && (nc + 1) * (long long)GS < (1LL << 31) &&
             (long long)C * round_up(std::max(s.nboot, 1), 32) < (1LL << 31);
    p.fused = boot_path && p.fast;
    p.keep_T = !p.fused || (want_post && s.post);
    int nbp = p.fast ? boot2_nb(s.nboot) : 16;
    if (p.fast) {
      const int v = cx->opt_boot_nb;  // tuning option: a multiple of 4 in [4, 32]
      if (v >= 4 && v <= 32 && v % 4 == 0) nbp = v;
    }
    // k_boot_tiles: G <= 448, nb <= 20, multiplicities <= 127 (int8), int32 digit sums.  The
    // tables are set up for it before the draws exist; should a multiplicity exceed 127 (a
    // cell drawn 128 times in one boot), plain k_boot2 runs on the same D columns instead.
    p.tpath = p.fused && s.nboot > 0 && G <= 448 && cx->opt_boot_skip && cx->opt_boot_tiles &&
              Ccall >= cx->opt_boot_tiles_cells && nbp <= 20 && C < 100000 && (nc + 1) * (long long)GS < (1LL << 31);
    // k_boot2 grid-stretch skipping (G <= 448: at most 7 stretches of 64 points); the
    // tables kernel emits the per-column stretch maxima
    p.stretch_skip = p.fused && !p.tpath && G <= 448 && cx->opt_boot_skip;
    return p;
  };
  // pieces: planned for the smallest column count (every condition holds for fewer columns)
  const Plan plan0 = make_plan(pieces ? 0 : ucl_off_h[C]);
  const bool want_maxi = s.batch_call ? (s.postflag == 1) : (s.postflag == 1 || s.postflag == 3);
  TablesArgs ta{};
  // buffers for `cap` columns (pieces: grown keeping what earlier pieces wrote) and the
  // launch arguments over the whole column range
  auto cx_sync = [cx] { return ctx_streams_sync(cx); };
  auto setup_tables = [&](const Plan& p, long long cap, bool keep) -> int {
    const size_t ncap = (size_t)std::max<long long>(1, cap);
    if (p.keep_T) HCHK(cx->T.grow(keep, sizeof(double) * ncap * GS, cx_sync));
    HCHK(cx->maxi.grow(keep, sizeof(int) * ncap, cx_sync));
    HCHK(cx->has_clamp.grow(keep, ncap, cx_sync));
    if (p.tpath) HCHK(cx->ubound.grow(keep, sizeof(unsigned) * kQTiles * (ncap + 1), cx_sync));
    if (p.fused) {
      HCHK(cx->E.grow(keep, sizeof(double) * (ncap + 1) * GS, cx_sync));
      if (p.stretch_skip) HCHK(cx->ubound.grow(keep, sizeof(double) * 8 * (ncap + 1), cx_sync));
    }
    if (!s.localtheta) HCHK(cx->colc.grow(keep, sizeof(double) * (kColc * ncap + 1), cx_sync));  // + the slow-column flag
    ta.ucl = u.ucl.as<int>();
    ta.ucl_off = u.ucl_off.as<long long>();
    ta.ncells = C;
    ta.G = G;
    ta.GS = GS;
    ta.mu = cx->mu.as<double>();
    ta.lcfp = cx->lcfp.as<double>();
    ta.lcfpr = cx->lcfpr.as<double>();
    ta.theta = cx->theta.as<double>();
    ta.cellscal = cx->cellscal.as<double>();
    // the reference's clamp, -DBL_MAX / (cells in the call) / 1.1 (src/jpmatLogBoot.cpp:127)
    ta.minlogprob = -1 * DBL_MAX / C / 1.1;
    // rows that fit the 256 MB last-level cache can be read back from it by the bootstrap: plain
    // stores there
    ta.nt_rows = cx->opt_tables_nt == 1 || (cx->opt_tables_nt == 2 && (double)ncap * GS * sizeof(double) > 256.0 * (1 << 20));
    ta.T = p.keep_T ? cx->T.as<double>() : nullptr;
    ta.maxi = want_maxi ? cx->maxi.as<int>() : nullptr;
    ta.has_clamp = cx->has_clamp.as<unsigned char>();
    ta.const_theta = s.localtheta ? 0 : 1;
    ta.pq = s.localtheta ? nullptr : cx->pq.as<double>();
    ta.colc = s.localtheta ? nullptr : cx->colc.as<double>();
    ta.cfp = cx->cfp.as<double>();
    ta.use_baseline = s.use_baseline ? 1 : 0;
    ta.UQ = p.tpath ? cx->ubound.as<unsigned>() : nullptr;
    ta.nanflag = p.tpath ? cx->qflags.as<int>() : nullptr;
    ta.D = p.fused ? cx->E.as<double>() : nullptr;
    ta.zcol = p.fused ? cx->zcol.as<int>() : nullptr;
    ta.base_col = p.fused ? cx->base_col.as<int>() : nullptr;
    ta.U = p.stretch_skip ? cx->ubound.as<double>() : nullptr;
    return SCDE_OK;
  };
  // the tables of cells [c0, c1), whose columns [col0, col0 + nc) are described by the
  // cell-local offsets off_h (device copy off_d, from 0); last: the pad column's task and p1_ev
  auto launch_tables_range = [&](const Plan& p, int c0, int c1, long long col0, const long long* off_d,
                                 const std::vector<long long>& off_h, bool last, UniqueSet& tu) -> int {
    const int Cc = c1 - c0;
    const long long nc = off_h[Cc];
    TablesArgs tc = ta;
    tc.ucl = ta.ucl + col0;
    tc.ucl_off = off_d;
    tc.ncols = nc;
    tc.ncells = Cc;
    const size_t co = (size_t)c0 * GS;
    tc.mu = ta.mu + co;
    tc.lcfp = ta.lcfp + co;
    tc.lcfpr = ta.lcfpr + co;
    if (tc.cfp) tc.cfp = ta.cfp + co;
    tc.theta = ta.theta + co;
    tc.cellscal = ta.cellscal + 2 * (size_t)c0;
    if (tc.pq) tc.pq = ta.pq + 4 * co;
    if (tc.T) tc.T = ta.T + (size_t)col0 * GS;
    if (tc.maxi) tc.maxi = ta.maxi + col0;
    tc.has_clamp = ta.has_clamp + col0;
    if (tc.colc) tc.colc = ta.colc + (size_t)kColc * col0;
    if (tc.UQ) tc.UQ = ta.UQ + (size_t)kQTiles * col0;
    if (tc.U) tc.U = ta.U + (size_t)8 * col0;
    if (tc.D) tc.D = ta.D + (size_t)col0 * GS;
    if (tc.zcol) tc.zcol = ta.zcol + c0;
    if (tc.base_col) tc.base_col = ta.base_col + c0;
    tc.col_base = (int)col0;
    // cell-staged tables (G <= 448): tasks of up to 64 columns of one cell -- one lane per column in
    // k_tables_lpc (constant theta); with local theta (k_tables_cell, 8 columns per wave) a launch that
    // would fill fewer than 4 rounds of the chip's block slots takes 32-column tasks, so its last
    // round is shorter
    if (G <= 448 && nc > 0) {
      const long long kTaskCols =
          (!s.localtheta || nc / kTabTaskCols >= 4096) ? kTabTaskCols : std::min(32, kTabTaskCols);
      tu.tasks_h.clear();
      for (int c = 0; c < Cc; ++c)
        for (long long b = off_h[c]; b < off_h[c + 1]; b += kTaskCols)
          tu.tasks_h.push_back(make_int4(c, (int)b, (int)std::min(b + kTaskCols, off_h[c + 1]), 0));
      if (p.fused && last) tu.tasks_h.push_back(make_int4(-1, 0, 0, 0));  // the ELL pad column
      RCHK(upload(cx, tu.tasks, tu.tasks_h.data(), sizeof(int4) * tu.tasks_h.size()));
      tc.tasks = tu.tasks.as<int4>();
      tc.ntasks = (int)tu.tasks_h.size();
    }
    hipEvent_t evt = cx->mark_begin(SLOT_TABLES);
    if (!s.localtheta && nc > 0)
      HCHK(launch_col_consts(tc.ucl, off_d, nc, Cc, tc.theta, GS, tc.cellscal,
                             cx->colc.as<double>() + (size_t)kColc * col0, st));
    if (p.fused) {
      tc.phase = 1;
      HCHK(launch_tables(tc, st));
      if (last) {
        if (!cx->p1_ev) HCHK(hipEventCreateWithFlags(&cx->p1_ev, hipEventDisableTiming));
        HCHK(handoff_spin(cx, st));
        HCHK(hipEventRecord(cx->p1_ev, st));
      }
      tc.phase = 2;
      HCHK(launch_tables(tc, st));
    } else {
      HCHK(launch_tables(tc, st));
    }
    cx->mark_end(SLOT_TABLES, evt);
    return SCDE_OK;
  };
  if (plan0.tpath) {
    HCHK(cx->qflags.ensure(sizeof(int) * 40));
    HCHK(hipMemsetAsync(cx->qflags.p, 0, sizeof(int) * 40, st));
  }
  if (plan0.fused) {
    HCHK(cx->base_col.ensure(sizeof(int) * std::max(1, C)));
    HCHK(cx->zcol.ensure(sizeof(int) * std::max(1, C)));
  }
  bool tables_done = false;
  const bool want_modes = s.batch_call ? (s.postflag == 1) : (s.postflag == 1 || s.postflag == 3);
  const bool modes_pieces = pieces && want_modes && s.modes && s.modes_host && N > 0;
  if (pieces) {
    // piece j: cells [piece_c[j], piece_c[j+1]) of this spec; its unique sets are built (on
    // the copy stream, beside the previous piece's tables) into u's arrays at the running
    // column offset, then its tables launch
    HCHK(u.uci.ensure(sizeof(int) * std::max<long long>(1, (long long)N * C)));
    ucl_off_h.assign(C + 1, 0);
    long long col0 = 0;
    int jlast = 0;
    for (int j = 0; j < s.npieces; ++j)
      if (s.piece_c[j + 1] > s.piece_c[j]) jlast = j;
    // the pieces' modes read-backs start once every piece's counts are up: run beside the uploads,
    // the pageable read-backs held them back (config 4: ~1 ms per 120 MB read-back)
    if (modes_pieces) dnl_hold(cx, true);
    using pclock = std::chrono::steady_clock;
    auto pms = [](pclock::time_point a, pclock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    for (int j = 0; j < s.npieces; ++j) {
      const int c0 = s.piece_c[j], c1 = s.piece_c[j + 1];
      const auto tw = pclock::now();
      RCHK(s.piece_ready(j));
      if (j == jlast && modes_pieces) dnl_hold(cx, false);  // (every piece's counts are up)
      const auto th = pclock::now();
      cx->st_piece_wait_ms += pms(tw, th);
      struct Lap {
        scde_ctx* cx;
        pclock::time_point t;
        ~Lap() { cx->st_piece_host_ms += std::chrono::duration<double, std::milli>(pclock::now() - t).count(); }
      } lap{cx, th};
      if (c1 == c0) continue;
      UniqueSet& pu = cx->upc[j];
      PostSpec ps;
      ps.ncells = c1 - c0;
      ps.counts_dev = s.counts_dev;
      ps.ld = s.ld;
      ps.cellidx_host = s.cellidx_host + c0;
      ps.ngenes = N;
      pu.into = &u;
      pu.into_col0 = col0;
      pu.into_c0 = c0;
      pu.into_cap_hint = c0 > 0 ? (long long)((double)col0 / c0 * C * 1.1) : 0;  // leading pieces may be empty
      const PostSpec* sp[1] = {&ps};
      UniqueSet* up[1] = {&pu};
      const hipStream_t main = cx->stream;
      cx->stream = s.piece_stream;
      const int rc = build_unique_sets(cx, sp, up, 1);
      cx->stream = main;
      pu.into = nullptr;
      RCHK(rc);
      HCHK(handoff_spin(cx, s.piece_stream));
      HCHK(hipEventRecord(s.piece_ev[j], s.piece_stream));
      HCHK(handoff_wait(cx, st, s.piece_ev[j]));
      for (int c = c0; c < c1; ++c) ucl_off_h[c + 1] = col0 + pu.ucl_off_h[c - c0 + 1];
      const long long nc = pu.ucl_off_h[c1 - c0];
      // The whole set's column offsets go up on this stream BEFORE the last piece's tables: the
      // bootstrap set-up (ELL rows) reads them on the aux stream, which waits only for p1_ev, the
      // event after the last piece's phase-1 tables.  Uploaded after the loop (rounds 3-4), the ELL
      // builder could read the previous call's offsets -- identical when the same data is run again,
      // garbage after a call on other data (the r04 full-size failure).
      if (j == jlast) RCHK(upload(cx, u.ucl_off, ucl_off_h.data(), sizeof(long long) * (C + 1)));
      // capacity for this piece plus an estimate of the rest (grown keeping the columns so far)
      const long long est = std::max<long long>(col0 + nc, (long long)((double)(col0 + nc) / c1 * C * 1.1));
      RCHK(setup_tables(plan0, est, j > 0));
      RCHK(launch_tables_range(plan0, c0, c1, col0, pu.ucl_off.as<long long>(), pu.ucl_off_h, j == jlast, pu));
      if (modes_pieces) {  // the piece's posterior modes, read back while the next pieces' tables run
        HCHK(launch_modes(u.uci.as<int>() + (size_t)N * c0, N, N, c1 - c0, pu.ucl_off.as<long long>(),
                          cx->maxi.as<int>() + col0, cx->mag.as<double>(), s.modes + (size_t)N * c0, 1, N, st));
        const size_t bytes = sizeof(double) * (size_t)N * (c1 - c0);
        RCHK(dnl_push(cx, st, s.modes_host + (size_t)N * c0, bytes, s.modes + (size_t)N * c0, bytes, bytes, 1));
      }
      col0 += nc;
    }
    ta.ucl_off = u.ucl_off.as<long long>();
    tables_done = make_plan(col0) == plan0;  // else: the whole tables again, planned for col0 columns
  }
  const long long ncols = ucl_off_h[C];
  const Plan plan = make_plan(ncols);
  const bool fast = plan.fast, fused = plan.fused, stretch_skip = plan.stretch_skip;
  bool tpath = plan.tpath;
  ta.ncols = ncols;
  if (!tables_done) {
    if (plan.tpath && !plan0.tpath) {
      HCHK(cx->qflags.ensure(sizeof(int) * 40));
      HCHK(hipMemsetAsync(cx->qflags.p, 0, sizeof(int) * 40, st));
    }
    if (plan.fused) {
      HCHK(cx->base_col.ensure(sizeof(int) * std::max(1, C)));
      HCHK(cx->zcol.ensure(sizeof(int) * std::max(1, C)));
    }
    RCHK(setup_tables(plan, ncols, false));
    ta.ncols = ncols;
    RCHK(launch_tables_range(plan, 0, C, 0, u.ucl_off.as<long long>(), ucl_off_h, true, cx->task_us));
  }
  std::vector<int> draws;
  std::vector<double> W;
  int ndraw = 0, maxw = 0;
  const int nsets = (int)s.seeds.size();
  // tile path ELL rows: a multiple of 64 entries (the bound MFMAs' K steps) plus 64
  const int qstride = (int)round_up(std::max(Cmax, 1), 64) + 64;
  // FP64 path: boots per slab; the draws come after the tables launch (the host's RNG work
  // then overlaps the tables kernel instead of leaving the GPU idle in front of it)
  int nb = fast ? boot2_nb(s.nboot) : 16;
  if (fast) {
    const int v = cx->opt_boot_nb;  // tuning option: a multiple of 4 in [4, 32]
    if (v >= 4 && v <= 32 && v % 4 == 0) nb = v;
  }
  const int Bp = (int)round_up(std::max(s.nboot, 1), nb);
  const int Bt = (int)round_up(Bp, 32) + 128;  // byte multiplicity rows: the last gene group reads 128 boots
  auto rest_fn = [=, &s, &u]() mutable -> int {
  // ---- individual posterior modes (src/jpmatLogBoot.cpp:277-296): argmax of each cell's table
  // column, known as soon as the tables are; computed here so the caller's read-back of the
  // (ngenes x ncells) matrix overlaps the bootstrap (pieces with modes_host: done piece by piece)
  if (want_modes && s.modes && s.modes_early && !modes_pieces) {
    HCHK(launch_modes(u.uci.as<int>(), N, N, C, u.ucl_off.as<long long>(), cx->maxi.as<int>(),
                      cx->mag.as<double>(), s.modes, 1, N, st));
    if (s.modes_host) {
      const size_t bytes = sizeof(double) * (size_t)N * C;
      RCHK(dnl_push(cx, st, s.modes_host, bytes, s.modes, bytes, bytes, 1));
    } else {
      if (!cx->modes_ev) HCHK(hipEventCreateWithFlags(&cx->modes_ev, hipEventDisableTiming));
      HCHK(handoff_spin(cx, st));
      HCHK(hipEventRecord(cx->modes_ev, st));
    }
  }
  // jp read back in gene chunks (the gene-block bootstrap below), else once at the end
  bool jp_sent = false;
  // fused (fast) path: the draw lists here, the multiplicity arrays on the device (launch_mult)
  const bool dev_mult = fused && C <= kMultMaxCells;
  if (fused && s.nboot > 0) {
    if (dev_mult) {
      make_draws(s, Bp, draws, W, ndraw, &maxw, false);
    } else {
      make_draws(s, Bp, draws, W, ndraw);
      maxw = 0;
      for (double w : W) maxw = std::max(maxw, (int)w);
    }
    tpath = tpath && maxw <= std::min(127, cx->opt_tile_max_mult);
  }
  // ---- joint posterior
  if (!s.batch_call && s.ensemble) {
    HCHK(cx->E.ensure(sizeof(double) * std::max<long long>(1, ncols) * GS));
    HCHK(launch_ensemble_cols(cx->T.as<double>(), ncols, G, GS, cx->E.as<double>(), st));
    NoBootArgs na{cx->E.as<double>(), G, GS, u.ucl_off.as<long long>(), u.uci.as<int>(), N, C, N, 1,
                  s.jp, s.jp_g, s.jp_k};
    HCHK(launch_noboot(na, st));
  } else if (s.nboot == 0 && !s.batch_call) {
    NoBootArgs na{cx->T.as<double>(), G, GS, u.ucl_off.as<long long>(), u.uci.as<int>(), N, C, N, 0,
                  s.jp, s.jp_g, s.jp_k};
    HCHK(launch_noboot(na, st));
  } else if (s.nboot == 0) {
    // logBootBatchPosterior with Nboot = 0 returns zeros (src/jpmatLogBoot.cpp:469-497)
    HCHK(hipMemsetAsync(s.jp, 0, sizeof(double) * (size_t)N * G, st));
  } else {
    if (!fused) make_draws(s, Bp, draws, W, ndraw);
    // the set-up below reads only phase 1's count-0 columns (fused path): on the aux stream,
    // beside phase 2 of the tables
    hipStream_t sa = st;
    if (fused) {
      if (!cx->aux_stream) HCHK(hipStreamCreateWithFlags(&cx->aux_stream, hipStreamNonBlocking));
      if (!cx->aux_ev) HCHK(hipEventCreateWithFlags(&cx->aux_ev, hipEventDisableTiming));
      sa = cx->aux_stream;
      HCHK(handoff_wait(cx, sa, cx->p1_ev));
    }
    if (!dev_mult) RCHK(upload_on(cx, cx->Wt, W.data(), sizeof(double) * W.size(), sa));
    RCHK(upload_on(cx, cx->draws, draws.data(), sizeof(int) * draws.size(), sa));
    if (!fused) {
      HCHK(cx->base_col.ensure(sizeof(int) * C));
      HCHK(launch_base_cols(u.ucl.as<int>(), u.ucl_off.as<long long>(), C, cx->has_clamp.as<unsigned char>(),
                            s.use_baseline ? 1 : 0, cx->base_col.as<int>(), st));
    }
    // + one look-ahead batch (k_boot2); the tile path's bounds read whole 64-entry steps
    const int stride = tpath ? qstride : (int)round_up(Cmax, 8) + 8;
    HCHK(cx->ent.ensure(sizeof(int2) * std::max<long long>(1, (long long)NBg * stride)));
    HCHK(cx->nnz.ensure(sizeof(int) * std::max(1, NBg)));
    ev = cx->mark_begin(SLOT_OTHER);
    if (!fused) {
      HCHK(cx->E.ensure(sizeof(double) * (size_t)(ncols + 1) * GS));
      HCHK(launch_delta(cx->T.as<double>(), u.ucl_off.as<long long>(), C, ncols, cx->base_col.as<int>(), G, GS,
                        cx->E.as<double>(), st));
    }
    // the baseline columns: T (slow path) or the fused D buffer, which holds T there
    const double* Tbase = fused ? cx->E.as<double>() : cx->T.as<double>();
    // k_boot_gene (not with pair mode): groups of gene_sg slabs per 4-wave block
    // k_boot_gene (gene_blocks, the default at every cell count the tile path runs; measured against
    // pair mode at config 4: bootstrap 11.16 -> 9.94 ms per step) or, without it, k_boot_tiles'
    // wave per slab (pair mode from pair_cells)
    const int gene_sg = (tpath && cx->opt_gene_blocks) ? std::min({(s.nboot + nb - 1) / nb, 8, 128 / nb}) : 0;
    // gene chunks (scde.posteriors, R-layout jp): the bootstrap over genes [gch(k), gch(k + 1))
    // finishes (list pass, fallback, slab sums, exact rows) before chunk k + 1 starts; with jp_host,
    // chunk k's jp rows go back to the host while it runs -- the read-back of the last chunk only is
    // left after the bootstrap.  Calls without the read-back thread (modes_overlap 0, the profiling
    // runs) chunk too, in the descending order below, whose L2 reuse is better (config 4: 29.1 ->
    // 24.1 GB of counter bytes, 10.8 -> 9.85 ms of k_boot_gene per step)
    const int nchunks = (gene_sg > 0 && s.jp_g == 1 && s.jp_k == N)
                            ? std::max(1, std::min(cx->opt_jp_chunks, NBg / 256 + 1)) : 1;
    auto gch = [NBg, nchunks](int k) { return (int)((long long)NBg * k / nchunks); };
    // tile path: genes in order of their count sums (waves in flight share columns in L2), keyed by
    // the ELL builder; with gene chunks each chunk's genes in order among themselves (the chunk
    // index in the keys' top bits: one sort)
    const bool have_order = tpath && fast && cx->opt_tile_order && NBg > 1;
    // descending (heaviest genes first, shorter tail) for small launches; ascending for large ones.
    // Measured (bootstrap ms per step, ascending -> descending): config 4's 7,500-gene chunks 10.59
    // -> 9.77, config 3's shard of 8 (2,500 genes per lane) 0.70 -> 0.63, config 3 (20,000 genes
    // per lane) 3.95 -> 4.09
    // scde.posteriors (R-layout jp) takes descending order at every chunk size (config 4, k_boot_gene
    // per step, ascending -> descending: chunks of 10,000 genes 26.9 -> 23.9 GB of counter bytes,
    // 10.3 -> 9.77 ms; one launch of 30,000 genes 29.1 -> 24.4 GB)
    constexpr int kDescGenes = 8192;
    const bool post_layout = s.jp_g == 1 && s.jp_k == N;
    const int order_desc = cx->opt_tile_order == 2 ||
                           (cx->opt_tile_order == 3 && (post_layout || (NBg + nchunks - 1) / nchunks <= kDescGenes));
    if (have_order) {
      HCHK(cx->gkey.ensure(sizeof(unsigned) * NBg));
      HCHK(cx->gkey2.ensure(sizeof(unsigned) * NBg));
      HCHK(cx->gidx.ensure(sizeof(int) * NBg));
      HCHK(cx->gorder.ensure(sizeof(int) * NBg));
    }
    // ELL rows (and the gene-order keys)
    HCHK(cx->ellw.ensure(std::max<size_t>(1, ell_work_bytes(N, C, cx->opt_ell_chunks))));
    HCHK(launch_ell(u.uci.as<int>(), N, N, C, u.ucl_off.as<long long>(), cx->base_col.as<int>(), stride, (int)ncols,
                    tpath ? 64 : 8, cx->ent.as<int2>(), cx->nnz.as<int>(), sa, 0, cx->ellw.p,
                    have_order ? u.ucl.as<int>() : nullptr, have_order ? cx->gkey.as<unsigned>() : nullptr,
                    have_order ? cx->gidx.as<int>() : nullptr, 0, NBg, nchunks, order_desc, cx->opt_ell_chunks));
    if (have_order) {
      size_t wb = 0;
      HCHK(launch_gene_order(nullptr, nullptr, NBg, nullptr, nullptr, nullptr, &wb, sa));
      HCHK(cx->gwork.ensure(std::max<size_t>(wb, 1)));
      HCHK(launch_gene_order(cx->gkey.as<unsigned>(), cx->gidx.as<int>(), NBg, cx->gkey2.as<unsigned>(),
                             cx->gorder.as<int>(), cx->gwork.p, &wb, sa));
    }
    if (dev_mult) {
      // the multiplicity arrays from the uploaded draw lists, on the device (host loops over
      // sets x cells x boots and their uploads cost ~0.1-0.4 ms of host time per posterior)
      const int P = (s.nboot + nb - 1) / nb;
      const int NGR = gene_sg > 0 ? (P + gene_sg - 1) / gene_sg : 0;
      const size_t sc = (size_t)nsets * C;
      HCHK(cx->Wt.ensure(sizeof(double) * std::max<size_t>(1, sc * Bp)));
      if (tpath) {
        HCHK(cx->w8.ensure(std::max<size_t>(1, sc * Bt)));
        HCHK(cx->w8t.ensure(std::max<size_t>(1, sc * P * 32)));
        if (gene_sg > 0) HCHK(cx->w8g.ensure(std::max<size_t>(1, sc * NGR * 128)));
      }
      HCHK(launch_mult(cx->draws.as<int>(), nsets, s.nboot, ndraw, C, Bp, cx->Wt.as<double>(), Bt,
                       tpath ? cx->w8.as<unsigned char>() : nullptr, nb, P,
                       tpath ? cx->w8t.as<unsigned char>() : nullptr, gene_sg, NGR,
                       (tpath && gene_sg > 0) ? cx->w8g.as<unsigned char>() : nullptr, sa));
    }
    if (tpath && !dev_mult) {
      // byte multiplicities [set][cell][boot] (baseline bound sums and the tile bounds)
      // and, for the tile bounds' A fragments, per slab the pairs (boot r, boot 16 + r) of its nb
      // boots, so one 16-bit load serves both 16-boot MFMA tiles
      const int P = (s.nboot + nb - 1) / nb;
      std::vector<unsigned char> w8((size_t)nsets * C * Bt, 0), w8p((size_t)nsets * C * P * 32, 0);
      for (int set = 0; set < nsets; ++set)
        for (int c = 0; c < C; ++c) {
          const double* wr = W.data() + ((size_t)set * C + c) * Bp;
          for (int b = 0; b < Bp; ++b) w8[((size_t)set * C + c) * Bt + b] = (unsigned char)wr[b];
          for (int p = 0; p < P; ++p)
            for (int j = 0; j < 32 && j < nb; ++j) {
              const int b = p * nb + j;
              if (b >= Bp) continue;
              const size_t slot = (j < 16) ? 2 * j : 2 * (j - 16) + 1;
              w8p[(((size_t)set * C + c) * P + p) * 32 + slot] = (unsigned char)wr[b];
            }
        }
      RCHK(upload_on(cx, cx->w8, w8.data(), w8.size(), sa));
      RCHK(upload_on(cx, cx->w8t, w8p.data(), w8p.size(), sa));
      if (gene_sg > 0) {  // k_boot_gene: per (cell, group of gene_sg slabs) four 32-boot windows as pair slots
        const int NGR = (P + gene_sg - 1) / gene_sg;
        std::vector<unsigned char> w8g((size_t)nsets * C * NGR * 128, 0);
        for (int set = 0; set < nsets; ++set)
          for (int c = 0; c < C; ++c) {
            const double* wr = W.data() + ((size_t)set * C + c) * Bp;
            for (int gr = 0; gr < NGR; ++gr) {
              const int gb0 = gr * gene_sg * nb, gnb = std::min(gene_sg, P - gr * gene_sg) * nb;
              for (int j = 0; j < gnb && j < 128; ++j) {
                const int b = gb0 + j;
                if (b >= Bp) break;
                const int w = j >> 5, jj = j & 31;
                const size_t slot = (jj < 16) ? 2 * jj : 2 * (jj - 16) + 1;
                w8g[(((size_t)set * C + c) * NGR + gr) * 128 + 32 * w + slot] = (unsigned char)wr[b];
              }
            }
          }
        RCHK(upload_on(cx, cx->w8g, w8g.data(), w8g.size(), sa));
      }
    }
    if (tpath) {
      HCHK(cx->zubound.ensure(sizeof(int) * (size_t)nsets * 4 * kQTiles * Bt));
      HCHK(launch_zuq(cx->ubound.as<unsigned>(), cx->base_col.as<int>(), C, cx->w8.as<unsigned char>(), Bt, nsets,
                      cx->zubound.as<int>(), sa));
    }
    HCHK(cx->Z.ensure(sizeof(double) * (size_t)nsets * Bp * GS));
    HCHK(launch_baseline_z(Tbase, G, GS, cx->base_col.as<int>(), C, cx->Wt.as<double>(), Bp, nsets,
                           cx->Z.as<double>(), sa));
    if (stretch_skip) {
      HCHK(cx->zubound.ensure(sizeof(double) * 8 * (size_t)nsets * Bp));
      HCHK(launch_stretch_zu(cx->ubound.as<double>(), cx->base_col.as<int>(), C, cx->Wt.as<double>(), Bp, nsets,
                             cx->zubound.as<double>(), sa));
    }
    cx->mark_end(SLOT_OTHER, ev);
    if (nsets > 1) {
      if ((int)s.wset.size() != NBg) return fail(SCDE_EINTERNAL, "wset size mismatch");
      RCHK(upload_on(cx, cx->wset, s.wset.data(), sizeof(int) * NBg, sa));
    }
    HCHK(cx->degen.ensure(sizeof(int) * std::max(1, NBg)));
    HCHK(hipMemsetAsync(cx->degen.p, 0, sizeof(int) * std::max(1, NBg), sa));
    if (sa != st) {  // the bootstrap waits for the set-up and for phase 2
      HCHK(handoff_spin(cx, sa));
      HCHK(hipEventRecord(cx->aux_ev, sa));
      HCHK(handoff_wait(cx, st, cx->aux_ev));
    }
    const int* wset_d = nsets > 1 ? cx->wset.as<int>() : nullptr;
    const double thresh = 16777216.0;  // 2^24: beyond this the sums' rounding order matters
    // rows whose sums left the exact range, in the reference's order (genes [g_lo, g_hi))
    bool exact_done = false;
    auto boot_exact = [&](int g_lo, int g_hi) -> int {
      ExactArgs xa{};
      xa.T = fused ? cx->E.as<double>() : cx->T.as<double>();
      xa.base_col = fused ? cx->base_col.as<int>() : nullptr;
      xa.G = G;
      xa.GS = GS;
      xa.draws = cx->draws.as<int>();
      xa.ndraw = ndraw;
      xa.nboot = s.nboot;
      xa.wset = wset_d;
      xa.ucl_off = u.ucl_off.as<long long>();
      xa.uci = u.uci.as<int>();
      xa.ld_uci = N;
      xa.norm_mult = (double)s.nboot;
      xa.degen = cx->degen.as<int>();
      xa.out = s.jp;
      xa.out_g = s.jp_g;
      xa.out_k = s.jp_k;
      xa.ngenes = NBg;
      xa.g_lo = g_lo;
      xa.g_hi = g_hi;
      HCHK(launch_boot_exact(xa, st));
      exact_done = true;
      return SCDE_OK;
    };
    ev = cx->mark_begin(SLOT_BOOT);
    if (fast) {
      Boot2Args b2{};
      b2.D = cx->E.as<double>();
      b2.ncols_p1 = ncols + 1;
      b2.ent = cx->ent.as<int2>();
      b2.nnz = cx->nnz.as<int>();
      b2.ent_stride = stride;
      b2.Wt = cx->Wt.as<double>();
      b2.Bp = Bp;
      b2.ncells = C;
      b2.wset = wset_d;
      b2.Z = cx->Z.as<double>();
      b2.G = G;
      b2.GS = GS;
      b2.nboot = s.nboot;
      b2.nb = nb;
      const int P = (s.nboot + nb - 1) / nb;
      b2.part_stride = (long long)NBg * GS;
      HCHK(cx->part.ensure(sizeof(double) * std::max<size_t>(1, (size_t)P * NBg * GS)));
      b2.part = cx->part.as<double>();
      b2.norm_mult = (double)s.nboot;
      b2.degen_thresh = thresh;
      b2.out = s.jp;
      b2.out_g = s.jp_g;
      b2.out_k = s.jp_k;
      b2.degen = cx->degen.as<int>();
      b2.ngenes = NBg;
      // the stretch mask's heuristic slack grows with the cells per call (the kernel's default reads
      // ncells, which counts both groups when fused): set here from the cells of one call
      b2.slack = std::isnan(cx->opt_skip_slack) ? 20.0 + 0.15 * Ccall : cx->opt_skip_slack;
      b2.U = stretch_skip ? cx->ubound.as<double>() : nullptr;
      b2.ZU = stretch_skip ? cx->zubound.as<double>() : nullptr;
      if (stretch_skip) {
        HCHK(cx->smask.ensure(sizeof(int) * std::max<size_t>(1, (size_t)P * NBg)));
        HCHK(cx->subuf.ensure(sizeof(double) * 8 * nb * std::max<size_t>(1, (size_t)P * NBg)));
        HCHK(cx->sredo.ensure(sizeof(int) * ((size_t)P * NBg + 1)));
        b2.mask = cx->smask.as<int>();
        b2.ubuf = cx->subuf.as<double>();
        b2.redo = cx->sredo.as<int>();
      }
      cx->st_boot_path = tpath ? 1 : 0;
      if (tpath) {
        HCHK(cx->sredo.ensure(sizeof(int) * (2 * (size_t)P * NBg + 1)));  // flags, list length, list
        b2.redo = cx->sredo.as<int>();
        TileBootArgs tb{};
        tb.W8p = cx->w8t.as<unsigned char>();
        tb.Bq = Bt;
        tb.UQ = cx->ubound.as<unsigned>();
        tb.ZUq = cx->zubound.as<int>();
        tb.nanflag = cx->qflags.as<int>();
        tb.maxgroups = cx->opt_tile_groups;
        tb.stats = cx->opt_skip_stats ? cx->qflags.as<int>() + 2 : nullptr;
        HCHK(cx->pmask.ensure(sizeof(unsigned) * std::max<size_t>(1, (size_t)P * NBg)));
        tb.pmask = cx->pmask.as<unsigned>();
        if (gene_sg > 0) {
          HCHK(cx->pwide.ensure(sizeof(int) * (1 + (size_t)P * NBg)));
          tb.wide = cx->pwide.as<int>();
          tb.gene = 1;
          tb.SG = gene_sg;
          tb.kcap = cx->opt_gene_rows;
          tb.list_cap = cx->opt_gene_list_cap;
          tb.W8g = cx->w8g.as<unsigned char>();
          if (cx->opt_gene_direct) {
            HCHK(cx->gdone.ensure(sizeof(int) * std::max(1, NBg)));
            tb.gdone = cx->gdone.as<int>();
          }
        }
        if (have_order) tb.order = cx->gorder.as<int>();
        if (nchunks > 1) {
          for (int k = 0; k < nchunks; ++k) {
            tb.g_lo = gch(k);
            tb.g_hi = gch(k + 1);
            HCHK(launch_boot_tiles(b2, tb, st));
            RCHK(boot_exact(tb.g_lo, tb.g_hi));
            if (!s.jp_host) continue;
            // chunk k's rows of the ngenes x ngrid column-major jp
            const size_t pitch = sizeof(double) * N;
            RCHK(dnl_push(cx, st, s.jp_host + tb.g_lo, pitch, s.jp + tb.g_lo, pitch,
                          sizeof(double) * (tb.g_hi - tb.g_lo), G));
          }
          jp_sent = s.jp_host != nullptr;
        } else {
          HCHK(launch_boot_tiles(b2, tb, st));
        }
        if (cx->opt_skip_stats) {
          int h[40];
          HCHK(hipMemcpyAsync(h, cx->qflags.p, sizeof(int) * 40, hipMemcpyDeviceToHost, st));
          HCHK(hipStreamSynchronize(st));
          for (int i = 0; i <= scde_ctx::kQMaxTilesHost; ++i) cx->st_tile_hist[i] += h[8 + i];
          cx->st_skip_slabs += h[2];
          cx->st_skip_kept += h[3];
          cx->st_skip_stretches += h[4];
          cx->st_skip_redo += h[5];
          cx->st_pair_redo += h[37];
          cx->st_boot_f64_fma += (double)h[6] * 64.0 * nb + (double)h[7] * nb * (double)round_up(G, 64);
        }
      } else {
        HCHK(launch_boot2(b2, st));
      }
      if (stretch_skip && cx->opt_skip_stats) {  // diagnostics: kept stretches, redo slabs
        std::vector<int> m((size_t)P * NBg), r((size_t)P * NBg), nz(NBg);
        HCHK(hipMemcpyAsync(m.data(), cx->smask.p, sizeof(int) * m.size(), hipMemcpyDeviceToHost, st));
        HCHK(hipMemcpyAsync(r.data(), cx->sredo.p, sizeof(int) * r.size(), hipMemcpyDeviceToHost, st));
        HCHK(hipMemcpyAsync(nz.data(), cx->nnz.p, sizeof(int) * nz.size(), hipMemcpyDeviceToHost, st));
        HCHK(hipStreamSynchronize(st));
        const int nst = (G + 63) / 64;
        long long kept = 0, redo = 0;
        double fma = 0;
        for (size_t i = 0; i < m.size(); ++i) {  // i = g * P + p
          const int k = __builtin_popcount((unsigned)m[i]);
          kept += k;
          redo += r[i] != 0;
          fma += (double)(k + (r[i] != 0 ? nst : 0)) * 64.0 * nb * nz[i / P];
        }
        cx->st_boot_f64_fma += fma;
        cx->st_skip_slabs += (double)m.size();
        cx->st_skip_stretches += (double)(m.size() * nst);
        cx->st_skip_kept += (double)kept;
        cx->st_skip_redo += (double)redo;
      }
    } else {
      BootArgs ba{};
      ba.T = cx->T.as<double>();
      ba.G = G;
      ba.GS = GS;
      ba.ent = cx->ent.as<int2>();
      ba.nnz = cx->nnz.as<int>();
      ba.ent_stride = stride;
      ba.base_col = cx->base_col.as<int>();
      ba.Wt = cx->Wt.as<double>();
      ba.ncells = C;
      ba.Bp = Bp;
      ba.nboot = s.nboot;
      ba.wset = wset_d;
      ba.Z = cx->Z.as<double>();
      ba.norm_mult = (double)s.nboot;
      ba.degen_thresh = thresh;
      ba.out = s.jp;
      ba.out_g = s.jp_g;
      ba.out_k = s.jp_k;
      ba.degen = cx->degen.as<int>();
      ba.ngenes = N;
      cx->st_boot_path = 3;
      HCHK(launch_boot(ba, st));
    }
    cx->mark_end(SLOT_BOOT, ev);
    if (!exact_done) RCHK(boot_exact(0, NBg));
  }
  if (s.jp_host && !jp_sent) {
    if (s.jp_g != 1 || s.jp_k != N) return fail(SCDE_EINTERNAL, "jp_host: jp not in R layout");
    const size_t bytes = sizeof(double) * (size_t)N * G;
    if (bytes) RCHK(dnl_push(cx, st, s.jp_host, bytes, s.jp, bytes, bytes, 1));
  }
  // ---- individual outputs (src/jpmatLogBoot.cpp:277-328)
  if (want_modes && s.modes && !s.modes_early) {
    HCHK(launch_modes(u.uci.as<int>(), N, N, C, u.ucl_off.as<long long>(), cx->maxi.as<int>(),
                      cx->mag.as<double>(), s.modes, 1, N, st));
    if (s.modes_host) {
      const size_t bytes = sizeof(double) * (size_t)N * C;
      RCHK(dnl_push(cx, st, s.modes_host, bytes, s.modes, bytes, bytes, 1));
    }
  }
  if (want_post && s.post)
    for (int c = 0; c < C; ++c)
      HCHK(launch_post(u.uci.as<int>(), N, N, c, u.ucl_off.as<long long>(), cx->T.as<double>(), G, GS,
                       s.post + (size_t)c * N * G, 1, N, st));
  return SCDE_OK;
  };
  if (rest) {
    *rest = rest_fn;
    return SCDE_OK;
  }
  return rest_fn();
}

std::mutex g_default_mu;
scde_ctx* g_default = nullptr;

int default_ctx(scde_ctx** out) {
  std::lock_guard<std::mutex> lk(g_default_mu);
  if (!g_default) {
    int dev = 0;
    if (const char* e = getenv("SCDE_DEVICE")) dev = atoi(e);
    if (const char* r = getenv("SCDE_RAND")) {
      if (!strcmp(r, "darwin")) g_rand_kind = SCDE_RAND_DARWIN;
      if (!strcmp(r, "glibc")) g_rand_kind = SCDE_RAND_GLIBC;
    }
    scde_ctx* c = nullptr;
    RCHK(scde_ctx_create(dev, &c));
    g_default = c;
  }
  *out = g_default;
  return SCDE_OK;
}

std::vector<double> marginals(const double* prior_x, int G) {
  // R/functions.R:575-577: log(pmax(10^x - 1, 0))
  std::vector<double> m(G);
  for (int k = 0; k < G; ++k) {
    double v = std::pow(10.0, prior_x[k]) - 1;
    if (v < 0) v = 0;
    m[k] = std::log(v);
  }
  return m;
}

// colnames of the ratio posterior as numbers: seq(x1-xn, xn-x1, length = 2n-1)
// formatted with 15 significant digits and parsed back (R/functions.R:3506, 5040)
std::vector<double> ratio_diffv(const double* x, int n) {
  const int m = 2 * n - 1;
  std::vector<double> rv(m);
  const double from = x[0] - x[n - 1], to = x[n - 1] - x[0];
  const double by = (to - from) / (m - 1);
  for (int i = 0; i < m; ++i) rv[i] = from + (double)i * by;
  rv[0] = from;
  rv[m - 1] = to;
  for (int i = 0; i < m; ++i) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.15g", rv[i]);
    rv[i] = strtod(buf, nullptr);
  }
  return rv;
}

int expectation_index(const std::vector<double>& diffv, double expectation) {
  const double target = expectation / std::log2(10.0);
  int zi = 0;
  double best = INFINITY;
  for (int i = 0; i < (int)diffv.size(); ++i) {
    const double d = std::fabs(diffv[i] - target);
    if (d < best) {
      best = d;
      zi = i;
    }
  }
  return zi;
}

// Reference seeding: one draw set per n.cores chunk overlapping this shard.
void seeding(int n_cores, long long gene_offset, long long N_total, int ngenes, std::vector<int>& seeds,
             std::vector<int>& wset) {
  seeds.clear();
  wset.clear();
  if (!(n_cores > 1 && N_total > n_cores)) {
    seeds.push_back(1);
    return;
  }
  const std::vector<long long> st = r_chunk_starts(N_total, n_cores);
  wset.assign(ngenes, 0);
  int cur = -1;
  long long last_chunk = -1;
  for (int g = 0; g < ngenes; ++g) {
    const long long gg = gene_offset + g;
    const long long ch = std::upper_bound(st.begin(), st.end(), gg) - st.begin() - 1;
    if (ch != last_chunk) {
      seeds.push_back((int)(st[ch] + 1));
      last_chunk = ch;
      cur = (int)seeds.size() - 1;
    }
    wset[g] = cur;
  }
  if (seeds.size() == 1) wset.clear();
}

void transpose_rows_to_colmajor(const double* rows, int N, int G, double* out) {
  for (int g = 0; g < N; ++g)
    for (int k = 0; k < G; ++k) out[(size_t)k * N + g] = rows[(size_t)g * G + k];
}

double pnorm_upper(double x);
double qnorm_host(double p, bool lower_tail);

}  // namespace

// =================================================================== C ABI
extern "C" {

const char* scde_last_error(void) { return g_err.c_str(); }

int scde_set_rand_kind(int kind) {
  if (kind != SCDE_RAND_GLIBC && kind != SCDE_RAND_DARWIN) return fail(SCDE_EARG, "unknown rand kind %d", kind);
  g_rand_kind = kind;
  return SCDE_OK;
}
int scde_get_rand_kind(void) { return g_rand_kind; }
int scde_version(void) { return 100; }

int scde_ctx_create(int device, scde_ctx** out) {
  FORK_GUARD();
  if (!out) return fail(SCDE_EARG, "null out");
  int n = 0;
  HCHK(hipGetDeviceCount(&n));
  if (n <= 0) return fail(SCDE_EHIP, "no HIP device");
  if (device < 0 || device >= n) return fail(SCDE_EARG, "device %d out of range (%d devices)", device, n);
  HCHK(hipSetDevice(device));
  auto* c = new scde_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(SCDE_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  c->home_stream = c->stream;
  // SCDE_OPTIONS="name=value,name=value": context options from the environment (tuning runs)
  if (const char* env = std::getenv("SCDE_OPTIONS")) {
    std::string all(env);
    size_t pos = 0;
    while (pos < all.size()) {
      size_t end = all.find(',', pos);
      if (end == std::string::npos) end = all.size();
      const std::string item = all.substr(pos, end - pos);
      pos = end + 1;
      const size_t eq = item.find('=');
      if (item.empty()) continue;
      int rc = SCDE_OK;
      if (eq == std::string::npos) {
        rc = fail(SCDE_EARG, "SCDE_OPTIONS item '%s' is not name=value", item.c_str());
      } else {
        // the whole value must be a number ("lanes=abc" or "lanes=" fail instead of becoming 0)
        const char* vs = item.c_str() + eq + 1;
        char* vend = nullptr;
        errno = 0;
        const double v = std::strtod(vs, &vend);
        if (*vs == '\0' || vend == vs || *vend != '\0' || errno == ERANGE)
          rc = fail(SCDE_EARG, "SCDE_OPTIONS item '%s': value is not a number", item.c_str());
        else
          rc = scde_ctx_set_option(c, item.substr(0, eq).c_str(), v);
      }
      if (rc != SCDE_OK) {
        scde_ctx_destroy(c);
        return rc;
      }
    }
  }
  *out = c;
  return SCDE_OK;
}

void scde_ctx_destroy(scde_ctx* ctx) {
  if (fork_guard() != SCDE_OK) return;  // a forked child leaves the parent's context alone
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  {
    std::lock_guard<std::mutex> lk(g_default_mu);
    if (ctx == g_default) g_default = nullptr;
  }
  delete ctx;
}

int scde_ctx_synchronize(scde_ctx* ctx) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  HCHK(hipSetDevice(ctx->device));
  return ctx->sync();
}

int scde_ctx_set_profiling(scde_ctx* ctx, int on) {
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  ctx->profile = on != 0;
  return SCDE_OK;
}

int scde_ctx_kernel_times(scde_ctx* ctx, double* ms, int64_t* launches, int nslots) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  RCHK(ctx->sync());
  for (int i = 0; i < nslots && i < NSLOTS; ++i) {
    if (ms) ms[i] = ctx->ms[i];
    if (launches) launches[i] = ctx->launches[i];
  }
  return SCDE_OK;
}

int scde_ctx_reset_kernel_times(scde_ctx* ctx) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  RCHK(ctx->sync());
  for (int i = 0; i < NSLOTS; ++i) {
    ctx->ms[i] = 0;
    ctx->launches[i] = 0;
  }
  return SCDE_OK;
}

int scde_ctx_set_option(scde_ctx* ctx, const char* name, double value) {
  if (!ctx || !name) return fail(SCDE_EARG, "null argument");
  const std::string n(name);
  if (n == "boot_skip") ctx->opt_boot_skip = value != 0;
  else if (n == "skip_slack") ctx->opt_skip_slack = value;
  else if (n == "boot_nb") ctx->opt_boot_nb = (int)value;
  else if (n == "skip_stats") ctx->opt_skip_stats = value != 0;
  else if (n == "wpca_ms") ctx->opt_wpca_ms = value != 0;
  else if (n == "boot_tiles") ctx->opt_boot_tiles = value != 0;
  else if (n == "boot_tiles_cells") ctx->opt_boot_tiles_cells = (int)value;
  else if (n == "tile_groups") ctx->opt_tile_groups = (int)value;
  else if (n == "tile_max_mult") ctx->opt_tile_max_mult = (int)value;
  else if (n == "tile_order") ctx->opt_tile_order = (value >= 1 && value <= 3) ? (int)value : 0;
  else if (n == "modes_overlap") ctx->opt_modes_overlap = value != 0;
  else if (n == "jp_chunks") ctx->opt_jp_chunks = std::max(1, std::min(64, (int)value));
  else if (n == "upload_u16") ctx->opt_upload_u16 = (value >= 0 && value <= 2) ? (int)value : 1;
  else if (n == "gene_list_cap") ctx->opt_gene_list_cap = std::max(0, (int)value);
  else if (n == "gene_rows") ctx->opt_gene_rows = std::max(1, std::min(4, (int)value));
  else if (n == "unique_fixed") ctx->opt_unique_fixed = value != 0;
  else if (n == "pipeline_mb") ctx->opt_pipeline_mb = value;
  else if (n == "pieces") ctx->opt_pieces = std::max(1, std::min((int)value, scde_ctx::kMaxPieces));
  else if (n == "tables_nt") ctx->opt_tables_nt = std::min(2, std::max(0, (int)value));
  else if (n == "lanes") {
    ctx->opt_lanes = value >= 2 ? 2 : 1;
    if (ctx->opt_lanes == 1 && ctx->peer) {  // one lane: the peer's workspace goes back to the device
      FORK_GUARD();
      HCHK(hipSetDevice(ctx->device));
      RCHK(ctx->sync());
      delete ctx->peer;
      ctx->peer = nullptr;
    }
  }
  else return fail(SCDE_EARG, "unknown option '%s'", name);
  return SCDE_OK;
}

int scde_ctx_inject_fault(scde_ctx* ctx, const char* where, int count) {
  if (!ctx || !where) return fail(SCDE_EARG, "null argument");
  if (std::string(where) == "u16_slot") ctx->fault_u16 = std::max(0, count);
  else if (std::string(where) == "handoff_spin") ctx->spin_cycles = std::max(0, count);
  else if (std::string(where) == "skip_lane_join") ctx->fault_skip_join = std::max(0, count);
  else return fail(SCDE_EARG, "unknown fault point '%s'", where);
  return SCDE_OK;
}

int scde_ctx_get_stat(scde_ctx* ctx, const char* name, double* value) {
  if (!ctx || !name || !value) return fail(SCDE_EARG, "null argument");
  const std::string n(name);
  if (n == "skip_slabs") *value = ctx->st_skip_slabs;
  else if (n == "skip_stretches") *value = ctx->st_skip_stretches;
  else if (n == "skip_kept") *value = ctx->st_skip_kept;
  else if (n == "boot_f64_fma") *value = ctx->st_boot_f64_fma;
  else if (n == "boot_path") *value = ctx->st_boot_path;
  else if (n == "skip_redo") *value = ctx->st_skip_redo;
  else if (n == "pair_redo") *value = ctx->st_pair_redo;
  else if (n == "degen") *value = ctx->st_degen;
  else if (n == "stream_syncs") *value = ctx->st_stream_syncs + (ctx->peer ? ctx->peer->st_stream_syncs : 0);
  else if (n == "arena_syncs") *value = ctx->st_arena_syncs + (ctx->peer ? ctx->peer->st_arena_syncs : 0);
  else if (n == "piece_wait_ms") *value = ctx->st_piece_wait_ms + (ctx->peer ? ctx->peer->st_piece_wait_ms : 0);
  else if (n == "piece_host_ms") *value = ctx->st_piece_host_ms + (ctx->peer ? ctx->peer->st_piece_host_ms : 0);
  else if (n == "buf_reallocs") *value = (double)g_buf_reallocs.load();
  else if (n == "handoff_spins") *value = (double)(ctx->st_spins.load() + (ctx->peer ? ctx->peer->st_spins.load() : 0));
  // (the upload worker and the 16-bit issuer update these under their mutexes)
  else if (n == "upload_wake_ms" || n == "upload_first_ms") {
    std::lock_guard<std::mutex> lk(ctx->upl.m);
    *value = n == "upload_wake_ms" ? ctx->upl.wake_ms : ctx->upl.first_ms;
  } else if (n == "u16_wait_ms" || n == "u16_issue_ms" || n == "u16_free_ms") {
    std::lock_guard<std::mutex> lk(ctx->u16.m);
    *value = n == "u16_wait_ms" ? ctx->u16.st_wait_ms : n == "u16_issue_ms" ? ctx->u16.st_issue_ms : ctx->u16.st_free_ms;
  }
  else if (n == "host_setup_ms") *value = ctx->st_host_ms[0];
  else if (n == "host_unique_ms") *value = ctx->st_host_ms[1];
  else if (n == "host_post_ms") *value = ctx->st_host_ms[2];
  else if (n == "host_tail_ms") *value = ctx->st_host_ms[3];
  else if (n.rfind("tiles_", 0) == 0 && atoi(n.c_str() + 6) >= 0 && atoi(n.c_str() + 6) <= 28)
    *value = ctx->st_tile_hist[atoi(n.c_str() + 6)];
  else return fail(SCDE_EARG, "unknown statistic '%s'", name);
  return SCDE_OK;
}

int scde_ctx_reset_stats(scde_ctx* ctx) {
  if (!ctx) return fail(SCDE_EARG, "null argument");
  ctx->st_skip_slabs = ctx->st_skip_kept = ctx->st_skip_stretches = ctx->st_skip_redo = ctx->st_degen = 0;
  ctx->st_pair_redo = 0;
  ctx->st_stream_syncs = ctx->st_arena_syncs = 0;
  if (ctx->peer) ctx->peer->st_stream_syncs = ctx->peer->st_arena_syncs = 0;
  ctx->st_piece_wait_ms = ctx->st_piece_host_ms = 0;
  if (ctx->peer) ctx->peer->st_piece_wait_ms = ctx->peer->st_piece_host_ms = 0;
  for (double& x : ctx->st_host_ms) x = 0;
  {
    std::lock_guard<std::mutex> lk(ctx->upl.m);
    ctx->upl.wake_ms = ctx->upl.first_ms = 0;
  }
  {
    std::lock_guard<std::mutex> lk(ctx->u16.m);
    ctx->u16.st_wait_ms = ctx->u16.st_issue_ms = ctx->u16.st_free_ms = 0;
  }
  ctx->st_boot_f64_fma = 0;
  ctx->st_spins = 0;
  if (ctx->peer) ctx->peer->st_spins = 0;
  for (double& x : ctx->st_tile_hist) x = 0;
  return SCDE_OK;
}

int scde_dev_alloc(scde_ctx* ctx, int64_t bytes, void** dptr) {
  FORK_GUARD();
  if (!ctx || !dptr || bytes < 0) return fail(SCDE_EARG, "bad args");
  HCHK(hipSetDevice(ctx->device));
  HCHK(hipMalloc(dptr, std::max<int64_t>(bytes, 1)));
  ctx->user_allocs.push_back(*dptr);
  return SCDE_OK;
}

int scde_dev_free(scde_ctx* ctx, void* dptr) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  auto it = std::find(ctx->user_allocs.begin(), ctx->user_allocs.end(), dptr);
  if (it == ctx->user_allocs.end()) return fail(SCDE_EARG, "pointer not owned by this context");
  ctx->user_allocs.erase(it);
  HCHK(hipFree(dptr));
  return SCDE_OK;
}

int scde_h2d(scde_ctx* ctx, void* dst, const void* src, int64_t bytes) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  HCHK(hipSetDevice(ctx->device));
  HCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return ctx->sync();
}

int scde_d2h(scde_ctx* ctx, void* dst, const void* src, int64_t bytes) {
  FORK_GUARD();
  if (!ctx) return fail(SCDE_EARG, "null ctx");
  HCHK(hipSetDevice(ctx->device));
  HCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return ctx->sync();
}

// ------------------------------------------------------------------ layer 1
// The posterior-mode matrix (ngenes x ncells doubles: 480 MB at config 4) to the host on the
// copy stream, after run_posterior's modes_ev: issued once every kernel of the call is queued
// (a pageable read-back can hold the host thread until it is done), it overlaps the bootstrap.
static int copy_modes_out(scde_ctx* cx, double* host, const double* dev, size_t n) {
  if (!cx->copy_stream) HCHK(hipStreamCreateWithFlags(&cx->copy_stream, hipStreamNonBlocking));
  HCHK(handoff_wait(cx, cx->copy_stream, cx->modes_ev));
  HCHK(hipMemcpyAsync(host, dev, sizeof(double) * n, hipMemcpyDeviceToHost, cx->copy_stream));
  return SCDE_OK;
}

static int logboot_common(bool batch, const double* models, int ncells, const int* ucl_vals, const int64_t* ucl_off,
                          const int* counti, int ngenes, const double* magnitudes, int ngrid, const int* batch_vals,
                          const int64_t* batch_off, const int* composition, int nbatch, int nboot, int seed,
                          int return_post, int local_theta, int square_logit_conc, int ensemble, double* jp,
                          double* modes, double* post) {
  if (!models || !ucl_vals || !ucl_off || !counti || !magnitudes || !jp)
    return fail(SCDE_EARG, "null input pointer");
  if (ncells <= 0 || ngenes < 0 || ngrid <= 0) return fail(SCDE_EARG, "bad dimensions");
  if (batch) {
    for (int k = 0; k < nbatch; ++k) {
      if (composition[k] > 0 && batch_off[k + 1] - batch_off[k] <= 0)
        return fail(SCDE_EARG, "batch %d has draws but no cells", k);
      for (int64_t i = batch_off[k]; i < batch_off[k + 1]; ++i)
        if (batch_vals[i] < 0 || batch_vals[i] >= ncells) return fail(SCDE_EARG, "BatchIL index out of range");
    }
  }
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  const size_t NG = (size_t)ngenes * ngrid;
  PostSpec s;
  s.ncells = ncells;
  s.models = models;
  s.localtheta = local_theta;
  s.squarelogit = square_logit_conc;
  s.mag = magnitudes;
  s.G = ngrid;
  s.nboot = nboot;
  s.postflag = return_post;
  s.ensemble = batch ? 0 : ensemble;
  s.batch_call = batch;
  s.ucl_host = ucl_vals;
  s.ucl_off_host = ucl_off;
  s.uci_host = counti;
  s.ngenes = ngenes;
  s.seeds = {seed};
  s.rand_kind = g_rand_kind;
  s.batch_vals = batch_vals;
  s.batch_off = batch_off;
  s.comp = composition;
  s.nbatch = nbatch;
  const bool want_modes = (batch ? return_post == 1 : (return_post == 1 || return_post == 3)) && modes;
  const bool want_post = (batch ? return_post == 2 : (return_post == 2 || return_post == 3)) && post;
  HCHK(cx->jpA.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  s.jp = cx->jpA.as<double>();
  s.jp_g = 1;  // R layout: ngenes x ngrid column-major
  s.jp_k = ngenes;
  if (want_modes) {
    HCHK(cx->jpB.ensure(sizeof(double) * std::max<size_t>(1, (size_t)ngenes * ncells)));
    s.modes = cx->jpB.as<double>();
    s.modes_early = ngenes > 0;
  }
  if (want_post) {
    HCHK(cx->outbuf.ensure(sizeof(double) * std::max<size_t>(1, NG * ncells)));
    s.post = cx->outbuf.as<double>();
  }
  cx->us[0].ready = false;
  RCHK(run_posterior(cx, s, cx->us[0]));
  if (s.modes_early) RCHK(copy_modes_out(cx, modes, s.modes, (size_t)ngenes * ncells));
  if (NG) HCHK(hipMemcpyAsync(jp, s.jp, sizeof(double) * NG, hipMemcpyDeviceToHost, cx->stream));
  if (want_post && NG)
    HCHK(hipMemcpyAsync(post, s.post, sizeof(double) * NG * ncells, hipMemcpyDeviceToHost, cx->stream));
  if (s.modes_early) HCHK(hipStreamSynchronize(cx->copy_stream));
  return cx->sync();
}

int scde_logBootPosterior(const double* models, int ncells, const int* ucl_vals, const int64_t* ucl_off,
                          const int* counti, int ngenes, const double* magnitudes, int ngrid, int nboot, int seed,
                          int return_post, int local_theta, int square_logit_conc, int ensemble, double* jp,
                          double* modes, double* post) {
  FORK_GUARD();
  return logboot_common(false, models, ncells, ucl_vals, ucl_off, counti, ngenes, magnitudes, ngrid, nullptr,
                        nullptr, nullptr, 0, nboot, seed, return_post, local_theta, square_logit_conc, ensemble, jp,
                        modes, post);
}

int scde_logBootBatchPosterior(const double* models, int ncells, const int* ucl_vals, const int64_t* ucl_off,
                               const int* counti, int ngenes, const double* magnitudes, int ngrid,
                               const int* batch_vals, const int64_t* batch_off, const int* composition, int nbatch,
                               int nboot, int seed, int return_post, int local_theta, int square_logit_conc,
                               double* jp, double* modes, double* post) {
  FORK_GUARD();
  if (!batch_vals || !batch_off || !composition) return fail(SCDE_EARG, "null batch input");
  return logboot_common(true, models, ncells, ucl_vals, ucl_off, counti, ngenes, magnitudes, ngrid, batch_vals,
                        batch_off, composition, nbatch, nboot, seed, return_post, local_theta, square_logit_conc, 0,
                        jp, modes, post);
}

// jpmat*: the matrices are the "cells", their rows the "genes", their columns the grid.
static int jpmat_common(const double* const* mats, int nmat, const int* type_off, const int* comp, int ntypes,
                        int nrows, int ncols, int nboot, int seed, double* out) {
  if (!mats || !out || nmat <= 0 || nrows < 0 || ncols <= 0) return fail(SCDE_EARG, "bad jpmat arguments");
  if (ncols > 4096) return fail(SCDE_EARG, "ncols > 4096 unsupported");
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  hipStream_t st = cx->stream;
  const int GS = (int)round_up(ncols, 16);
  const size_t per = (size_t)nrows * ncols;
  // stage matrices as row-major tables: column (m, r) = m * nrows + r
  HCHK(cx->T.ensure(sizeof(double) * std::max<size_t>(1, (size_t)nmat * nrows * GS)));
  HCHK(cx->in1.ensure(sizeof(double) * std::max<size_t>(1, per)));
  for (int m = 0; m < nmat; ++m) {
    HCHK(hipMemcpyAsync(cx->in1.p, mats[m], sizeof(double) * per, hipMemcpyHostToDevice, st));
    HCHK(launch_colmajor_to_rows(cx->in1.as<double>(), nrows, ncols, GS, cx->T.as<double>() + (size_t)m * nrows * GS,
                                 st));
  }
  // draws
  const int Bp = (int)round_up(std::max(nboot, 1), 16);
  int ndraw = 0;
  std::vector<int> draws;
  std::vector<double> W((size_t)nmat * Bp, 0.0);
  PlatformRand rng((unsigned int)seed, g_rand_kind);
  if (!type_off) {
    ndraw = nmat;
    draws.resize((size_t)std::max(nboot, 1) * ndraw);
    for (int b = 0; b < nboot; ++b)
      for (int j = 0; j < nmat; ++j) {
        const int rj = rng.draw(nmat);
        draws[(size_t)b * ndraw + j] = rj;
        W[(size_t)rj * Bp + b] += 1.0;
      }
  } else {
    for (int k = 0; k < ntypes; ++k) {
      ndraw += std::max(0, comp[k]);
      if (comp[k] > 0 && type_off[k + 1] - type_off[k] <= 0) return fail(SCDE_EARG, "type %d has no matrices", k);
    }
    draws.resize((size_t)std::max(nboot, 1) * std::max(ndraw, 1));
    for (int b = 0; b < nboot; ++b) {
      int d = 0;
      for (int k = 0; k < ntypes; ++k)
        for (int j = 0; j < comp[k]; ++j) {
          const int m = type_off[k] + rng.draw(type_off[k + 1] - type_off[k]);
          draws[(size_t)b * ndraw + d++] = m;
          W[(size_t)m * Bp + b] += 1.0;
        }
    }
  }
  // every row takes every matrix (no baseline)
  std::vector<int2> ent((size_t)std::max(1, nrows) * nmat);
  for (int r = 0; r < nrows; ++r)
    for (int m = 0; m < nmat; ++m) ent[(size_t)r * nmat + m] = make_int2(m, m * nrows + r);
  std::vector<int> nnz(std::max(1, nrows), nmat);
  RCHK(upload(cx, cx->ent, ent.data(), sizeof(int2) * ent.size()));
  RCHK(upload(cx, cx->nnz, nnz.data(), sizeof(int) * nnz.size()));
  RCHK(upload(cx, cx->Wt, W.data(), sizeof(double) * W.size()));
  RCHK(upload(cx, cx->draws, draws.data(), sizeof(int) * draws.size()));
  HCHK(cx->degen.ensure(sizeof(int) * std::max(1, nrows)));
  HCHK(hipMemsetAsync(cx->degen.p, 0, sizeof(int) * std::max(1, nrows), st));
  HCHK(cx->jpA.ensure(sizeof(double) * std::max<size_t>(1, per)));
  if (nboot == 0) {
    HCHK(hipMemsetAsync(cx->jpA.p, 0, sizeof(double) * std::max<size_t>(1, per), st));
  } else {
    BootArgs ba{};
    ba.T = cx->T.as<double>();
    ba.G = ncols;
    ba.GS = GS;
    ba.ent = cx->ent.as<int2>();
    ba.nnz = cx->nnz.as<int>();
    ba.ent_stride = nmat;
    ba.base_col = nullptr;
    ba.Wt = cx->Wt.as<double>();
    ba.ncells = nmat;
    ba.Bp = Bp;
    ba.nboot = nboot;
    ba.wset = nullptr;
    ba.Z = nullptr;
    ba.norm_mult = 1.0;  // jpmat* do not divide by nboot (src/jpmatLogBoot.cpp:36-38)
    ba.degen_thresh = 16777216.0;
    ba.out = cx->jpA.as<double>();
    ba.out_g = 1;
    ba.out_k = nrows;
    ba.degen = cx->degen.as<int>();
    ba.ngenes = nrows;
    hipEvent_t ev = cx->mark_begin(SLOT_BOOT);
    HCHK(launch_boot(ba, st));
    cx->mark_end(SLOT_BOOT, ev);
    ExactArgs xa{};
    xa.T = ba.T;
    xa.G = ncols;
    xa.GS = GS;
    xa.draws = cx->draws.as<int>();
    xa.ndraw = ndraw;
    xa.nboot = nboot;
    xa.wset = nullptr;
    xa.ucl_off = nullptr;
    xa.uci = nullptr;
    xa.ld_uci = 0;
    xa.norm_mult = 1.0;
    xa.degen = ba.degen;
    xa.out = ba.out;
    xa.out_g = 1;
    xa.out_k = nrows;
    xa.ngenes = nrows;
    HCHK(launch_boot_exact(xa, st));
  }
  if (per) HCHK(hipMemcpyAsync(out, cx->jpA.p, sizeof(double) * per, hipMemcpyDeviceToHost, st));
  return cx->sync();
}

int scde_jpmatLogBoot(const double* const* mats, int nmat, int nrows, int ncols, int nboot, int seed, double* out) {
  FORK_GUARD();
  return jpmat_common(mats, nmat, nullptr, nullptr, 0, nrows, ncols, nboot, seed, out);
}

int scde_jpmatLogBatchBoot(const double* const* mats, const int* type_off, const int* comp, int ntypes, int nrows,
                           int ncols, int nboot, int seed, double* out) {
  FORK_GUARD();
  if (!type_off || !comp || ntypes <= 0) return fail(SCDE_EARG, "bad jpmatLogBatchBoot arguments");
  return jpmat_common(mats, type_off[ntypes], type_off, comp, ntypes, nrows, ncols, nboot, seed, out);
}

static int ratio_common(const double* pmat1, const double* pmat2, int nrows, int n, const double* prior_y,
                        const double* diffv, int zi, int normalize, double* ratio, double* res) {
  if (!pmat1 || !pmat2 || nrows < 0 || n <= 0) return fail(SCDE_EARG, "bad ratio arguments");
  if (res && (!diffv || zi < 0 || zi >= 2 * n - 1)) return fail(SCDE_EARG, "bad diffv/zi");
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  hipStream_t st = cx->stream;
  const size_t per = (size_t)nrows * n, m = 2 * (size_t)n - 1;
  RCHK(upload(cx, cx->in1, pmat1, sizeof(double) * std::max<size_t>(1, per)));
  RCHK(upload(cx, cx->in2, pmat2, sizeof(double) * std::max<size_t>(1, per)));
  if (prior_y) RCHK(upload(cx, cx->prior_y, prior_y, sizeof(double) * n));
  if (res) RCHK(upload(cx, cx->diffv, diffv, sizeof(double) * m));
  HCHK(cx->ratio.ensure(sizeof(double) * std::max<size_t>(1, nrows * m)));
  HCHK(cx->res.ensure(sizeof(double) * std::max<size_t>(1, (size_t)nrows * 5)));
  RatioArgs ra{};
  ra.jp1 = cx->in1.as<double>();
  ra.j1g = 1;
  ra.j1k = nrows;
  ra.jp2 = cx->in2.as<double>();
  ra.j2g = 1;
  ra.j2k = nrows;
  ra.prior_y = prior_y ? cx->prior_y.as<double>() : nullptr;
  ra.n = n;
  ra.ngenes = nrows;
  ra.normalize = normalize;
  ra.ratio = cx->ratio.as<double>();
  ra.rg = 1;
  ra.ro = nrows;
  ra.diffv = res ? cx->diffv.as<double>() : nullptr;
  ra.zi = zi;
  ra.res = res ? cx->res.as<double>() : nullptr;
  ra.res_ld = nrows;
  hipEvent_t ev = cx->mark_begin(SLOT_RATIO);
  ra.window = cx->opt_ratio_window;
  ra.block = cx->opt_ratio_block;
  HCHK(launch_ratio_summary(ra, st));
  cx->mark_end(SLOT_RATIO, ev);
  if (ratio && nrows) HCHK(hipMemcpyAsync(ratio, ra.ratio, sizeof(double) * nrows * m, hipMemcpyDeviceToHost, st));
  if (res && nrows) HCHK(hipMemcpyAsync(res, ra.res, sizeof(double) * nrows * 5, hipMemcpyDeviceToHost, st));
  return cx->sync();
}

int scde_distribution_summary(const double* rpost, int nrows, int m, const double* diffv, int zi, double* res) {
  FORK_GUARD();
  if (!rpost || !diffv || !res || nrows < 0 || m < 1 || (m % 2) == 0) return fail(SCDE_EARG, "bad summary arguments");
  if (zi < 0 || zi >= m) return fail(SCDE_EARG, "zi out of range");
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  hipStream_t st = cx->stream;
  const int n = (m + 1) / 2;
  RCHK(upload(cx, cx->in1, rpost, sizeof(double) * std::max<size_t>(1, (size_t)nrows * m)));
  RCHK(upload(cx, cx->diffv, diffv, sizeof(double) * m));
  HCHK(cx->res.ensure(sizeof(double) * std::max<size_t>(1, (size_t)nrows * 5)));
  RatioArgs ra{};
  ra.n = n;
  ra.ngenes = nrows;
  ra.xin = cx->in1.as<double>();
  ra.xg = 1;
  ra.xo = nrows;
  ra.diffv = cx->diffv.as<double>();
  ra.zi = zi;
  ra.res = cx->res.as<double>();
  ra.res_ld = nrows;
  ra.window = cx->opt_ratio_window;
  ra.block = cx->opt_ratio_block;
  HCHK(launch_ratio_summary(ra, st));
  if (nrows) HCHK(hipMemcpyAsync(res, ra.res, sizeof(double) * nrows * 5, hipMemcpyDeviceToHost, st));
  return cx->sync();
}

int scde_matSlideMult(const double* m1, const double* m2, int nrows, int ncols, double* out) {
  FORK_GUARD();
  if (!out) return fail(SCDE_EARG, "null out");
  return ratio_common(m1, m2, nrows, ncols, nullptr, nullptr, 0, 0, out, nullptr);
}

int scde_ratio_summary(const double* pmat1, const double* pmat2, int nrows, int n, const double* prior_y,
                       const double* diffv, int zi, double* ratio, double* res) {
  FORK_GUARD();
  return ratio_common(pmat1, pmat2, nrows, n, prior_y, diffv, zi, 1, ratio, res);
}

// ------------------------------------------------------------------ layer 2
// Host counts of a host-count entry (de_run: the first group's range in pieces, then the
// second group's range; posteriors_run: the selected cells in pieces), copied on the context's
// copy stream by an UploadWorker.
struct HostUpload {
  const int* counts;
  int64_t ld;
  int ngenes, cut, C;
  bool u16 = false;  // ranges of >= 8 MB as 16-bit counts (upload_cols_u16)
};
// narrow n int32 counts to uint16, appending the counts outside [0, 65535] (negative ones
// included) to `exc` as (i0 + index, count): blocks of 256 narrowed by a vectorised loop, a
// block whose high halves are not all zero scanned again
// The block loop, compiled twice: for the baseline x86-64 target and for AVX2 (8 counts per
// instruction; chosen at run time when the CPU has it).  Returns the OR of the block's high halves.
static inline unsigned narrow_block(const int* s, unsigned short* d, size_t b0, size_t e) {
  unsigned b = 0;
  for (size_t i = b0; i < e; ++i) {
    const unsigned v = (unsigned)s[i];
    b |= v >> 16;
    d[i] = (unsigned short)v;
  }
  return b;
}
__attribute__((target("avx2"))) static unsigned narrow_block_avx2(const int* s, unsigned short* d, size_t b0,
                                                                   size_t e) {
  unsigned b = 0;
  for (size_t i = b0; i < e; ++i) {
    const unsigned v = (unsigned)s[i];
    b |= v >> 16;
    d[i] = (unsigned short)v;
  }
  return b;
}
static const bool g_have_avx2 = __builtin_cpu_supports("avx2");

static void narrow16(const int* s, unsigned short* d, size_t n, int i0, std::vector<int2>& exc) {
  for (size_t b0 = 0; b0 < n; b0 += 256) {
    const size_t e = std::min(n, b0 + 256);
    const unsigned b = g_have_avx2 ? narrow_block_avx2(s, d, b0, e) : narrow_block(s, d, b0, e);
    if (b)
      for (size_t i = b0; i < e; ++i)
        if ((unsigned)s[i] >> 16) exc.push_back(make_int2(i0 + (int)i, s[i]));
  }
}

// the narrowing pool's thread t: per job, its share of every slot, in sequence order
static void u16_thread(scde_ctx* ctx, int t) {
  auto& r = ctx->u16;
  using R = scde_ctx::U16Ring;
  long long seen = 0;
  std::unique_lock<std::mutex> lk(r.m);
  for (;;) {
    r.cv.wait(lk, [&] { return r.stop || r.job != seen; });
    if (r.stop) return;
    seen = r.job;
    const int* src = r.src;
    const size_t n = r.n;
    const long long q0 = r.q0;
    const int nslots = r.nslots, T = r.T;
    for (int sl = 0; sl < nslots; ++sl) {
      const long long q = q0 + sl;
      r.cv.wait(lk, [&] { return r.free_upto > q || r.abort; });
      if (r.abort) break;
      lk.unlock();
      const int k = (int)(q % R::kRing);
      const size_t off = (size_t)sl * R::kSlotCounts;
      const size_t m = std::min(R::kSlotCounts, n - off);
      const size_t a = (m * t / T) & ~size_t(15), e = (t + 1 == T) ? m : ((m * (t + 1) / T) & ~size_t(15));
      r.exc[k][t].clear();
      if (e > a) narrow16(src + off + a, r.pin + (size_t)k * R::kSlotCounts + a, e - a, (int)a, r.exc[k][t]);
      lk.lock();
      if (++r.fin[k] == T) r.cvf.notify_all();
    }
    if (--r.busy == 0) r.cvd.notify_all();
  }
}

// columns [lo, hi) of contiguous host counts as 16-bit counts through U16Ring, widened (and the
// counts outside [0, 65535] patched in) on the copy stream
static int upload_cols_u16(scde_ctx* ctx, const HostUpload& h, int lo, int hi) {
  auto& r = ctx->u16;
  using R = scde_ctx::U16Ring;
  if (!r.pin) {
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&r.pin), sizeof(unsigned short) * R::kRing * R::kSlotCounts,
                       hipHostMallocDefault));
    HCHK(hipMalloc(reinterpret_cast<void**>(&r.dev), sizeof(unsigned short) * R::kRing * R::kSlotCounts));
    for (auto& e : r.ev) HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync));
  }
  const int T = std::max(1, std::min(R::kMaxT, ctx->opt_upload_threads));
  if ((int)r.th.size() != T) {  // (re)build the pool (no job is running: the upload worker is its only user)
    if (!r.th.empty()) {
      {
        std::lock_guard<std::mutex> lk(r.m);
        r.stop = true;
      }
      r.cv.notify_all();
      for (auto& t : r.th) t.join();
      r.th.clear();
      r.stop = false;
    }
    {
      std::lock_guard<std::mutex> lk(r.m);
      r.T = T;
    }
    for (int t = 0; t < T; ++t) r.th.emplace_back(u16_thread, ctx, t);
  }
  const size_t n = (size_t)h.ngenes * (size_t)(hi - lo);
  const int* src = h.counts + (size_t)h.ld * lo;
  int* dst = static_cast<int*>(ctx->counts_in.p) + (size_t)h.ngenes * lo;
  const int nslots = (int)((n + R::kSlotCounts - 1) / R::kSlotCounts);
  const long long q0 = r.seq;
  std::unique_lock<std::mutex> lk(r.m);
  r.src = src;
  r.n = n;
  r.q0 = q0;
  r.nslots = nslots;
  r.abort = false;
  r.busy = T;
  ++r.job;
  r.cv.notify_all();
  int rc = SCDE_OK;
  // (the statistics are summed under r.m, where scde_ctx_get_stat reads them)
  double wait_ms = 0, issue_ms = 0, free_ms = 0;
  for (int sl = 0; sl < nslots; ++sl) {
    const long long q = q0 + sl;
    const int k = (int)(q % R::kRing);
    const auto tw = std::chrono::steady_clock::now();
    r.cvf.wait(lk, [&] { return r.fin[k] == T; });
    r.fin[k] = 0;
    lk.unlock();
    const auto ti = std::chrono::steady_clock::now();
    wait_ms += std::chrono::duration<double, std::milli>(ti - tw).count();
    const size_t off = (size_t)sl * R::kSlotCounts;
    const size_t m = std::min(R::kSlotCounts, n - off);
    unsigned short* dslot = r.dev + (size_t)k * R::kSlotCounts;
    hipError_t e = hipMemcpyAsync(dslot, r.pin + (size_t)k * R::kSlotCounts, sizeof(unsigned short) * m,
                                  hipMemcpyHostToDevice, ctx->copy_stream);
    if (e == hipSuccess && ctx->fault_u16 > 0 && sl == std::min(1, nslots - 1)) {  // test hook (scde_ctx_inject_fault)
      --ctx->fault_u16;
      e = hipErrorUnknown;
    }
    if (e == hipSuccess) e = handoff_spin(ctx, ctx->copy_stream);
    if (e == hipSuccess) e = hipEventRecord(r.ev[k], ctx->copy_stream);
    if (e == hipSuccess) e = launch_widen16(dslot, dst + off, m, ctx->copy_stream);
    // the slot's counts outside 16 bits (the threads' lists of ring slot k are complete and
    // untouched until the slot is freed again below)
    r.exc_all.clear();
    for (int t = 0; t < T; ++t) r.exc_all.insert(r.exc_all.end(), r.exc[k][t].begin(), r.exc[k][t].end());
    if (e == hipSuccess && !r.exc_all.empty()) {
      // (a pageable copy has read the host list when it returns; the patch follows it in stream order)
      e = ctx->excd.ensure(sizeof(int2) * std::max<size_t>(r.exc_all.size(), 65536));
      if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->excd.p, r.exc_all.data(), sizeof(int2) * r.exc_all.size(), hipMemcpyHostToDevice,
                           ctx->copy_stream);
      if (e == hipSuccess) e = launch_patch32(ctx->excd.as<int2>(), r.exc_all.size(), dst + off, ctx->copy_stream);
    }
    r.issued = q + 1;
    const auto tf = std::chrono::steady_clock::now();
    issue_ms += std::chrono::duration<double, std::milli>(tf - ti).count();
    // free the ring slot the threads need next (slot q + 1 reuses slot q + 1 - kRing's): wait for
    // that DMA, then let them write (only this thread writes free_upto)
    const long long f = q + 1 - R::kRing;
    const bool advance = e == hipSuccess && r.free_upto <= q + 1;
    if (advance && f >= 0) e = hipEventSynchronize(r.ev[f % R::kRing]);
    free_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf).count();
    lk.lock();
    if (e != hipSuccess) {
      rc = fail(SCDE_EHIP, "%s", hipGetErrorString(e));
      break;
    }
    if (advance) {
      r.free_upto = q + 2;
      r.cv.notify_all();
    }
  }
  if (rc != SCDE_OK) {
    r.abort = true;
    r.cv.notify_all();
  }
  r.cvd.wait(lk, [&] { return r.busy == 0; });
  for (auto& f : r.fin) f = 0;  // (an aborted job leaves partial counts)
  r.seq = r.issued;             // sequence numbers of slots never issued are reused
  r.st_wait_ms += wait_ms;
  r.st_issue_ms += issue_ms;
  r.st_free_ms += free_ms;
  if (rc != SCDE_OK) {
    // an error after slots were issued: free_upto may lag behind seq, and the next job's threads
    // would wait for a slot nobody frees.  Drain the copy stream -- every issued slot's DMA has then
    // finished (or failed) -- and open the whole ring to the next job.
    lk.unlock();
    (void)hipStreamSynchronize(ctx->copy_stream);
    (void)hipGetLastError();
    lk.lock();
    r.free_upto = r.seq + R::kRing;
  }
  lk.unlock();
  return rc;
}

// columns [lo, hi) of the host counts into counts_in, on the copy stream
static int upload_cols(scde_ctx* ctx, const HostUpload& h, int lo, int hi) {
  const size_t row = sizeof(int) * (size_t)h.ngenes;
  if (hi > lo && h.u16 && h.ld == h.ngenes && row * (size_t)(hi - lo) >= (size_t(8) << 20))
    return upload_cols_u16(ctx, h, lo, hi);
  if (hi > lo) {
    char* dst = static_cast<char*>(ctx->counts_in.p) + row * lo;
    const int* src = h.counts + (size_t)h.ld * lo;
    if (h.ld == h.ngenes)
      HCHK(hipMemcpyAsync(dst, src, row * (hi - lo), hipMemcpyHostToDevice, ctx->copy_stream));
    else
      HCHK(hipMemcpy2DAsync(dst, row, src, sizeof(int) * (size_t)h.ld, row, hi - lo, hipMemcpyHostToDevice,
                            ctx->copy_stream));
  }
  return SCDE_OK;
}

// The host-count uploads of one call, issued back to back from a worker thread: a pageable
// copy blocks its calling thread for the whole transfer, so issued from the caller's thread
// each piece would wait for the previous piece's unique-set build (a host sync) and PCIe would
// sit idle in between.  Column ranges [cols[j], cols[j+1]) go up on the copy stream in order,
// each followed by evs[j]; wait(n) returns once the first n are issued (their events recorded).
struct UploadWorker {
  scde_ctx* ctx = nullptr;
  int start(scde_ctx* c, const HostUpload& h, const std::vector<int>& cols, std::vector<hipEvent_t> evs) {
    if (cols.size() != evs.size() + 1)
      return fail(SCDE_EINTERNAL, "upload ranges: %d bounds for %d events", (int)cols.size(), (int)evs.size());
    std::vector<std::pair<int, int>> ranges;
    for (size_t j = 0; j + 1 < cols.size(); ++j) ranges.emplace_back(cols[j], cols[j + 1]);
    return start(c, h, std::move(ranges), std::move(evs));
  }
  // ranges[j] = [lo, hi) in any order (the interleaved two-group upload)
  int start(scde_ctx* c, const HostUpload& h, std::vector<std::pair<int, int>> ranges, std::vector<hipEvent_t> evs) {
    ctx = c;
    auto& u = c->upl;
    if (!u.th.joinable()) {
      u.th = std::thread([c] {
        auto& q = c->upl;
        (void)hipSetDevice(c->device);
        long long seen = 0;
        std::unique_lock<std::mutex> lk(q.m);
        for (;;) {
          q.cv.wait(lk, [&] { return q.stop || q.job != seen; });
          if (q.stop) return;
          seen = q.job;
          const int n = q.nranges;
          auto issue = q.issue;
          const auto t0 = q.t_start;
          q.wake_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
          lk.unlock();
          int rc = SCDE_OK;
          for (int j = 0; j < n && rc == SCDE_OK; ++j) {
            rc = issue(j);
            std::lock_guard<std::mutex> g(q.m);
            if (j == 0)
              q.first_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (rc != SCDE_OK) {
              q.err = rc;
              q.err_msg = g_err;  // g_err is thread-local: hand the worker's message to the caller
            } else {
              ++q.issued;
            }
            q.cv.notify_all();
          }
          lk.lock();
          q.busy = false;
          q.cv.notify_all();
        }
      });
    }
    const int nranges = (int)evs.size();  // (before the vectors move into the closure)
    if ((int)ranges.size() != nranges) return fail(SCDE_EINTERNAL, "upload ranges: %d ranges for %d events",
                                                   (int)ranges.size(), nranges);
    std::lock_guard<std::mutex> lk(u.m);
    u.issue = [c, h, ranges = std::move(ranges), evs = std::move(evs)](int j) -> int {
      RCHK(upload_cols(c, h, ranges[j].first, ranges[j].second));
      HCHK(handoff_spin(c, c->copy_stream));
      HCHK(hipEventRecord(evs[j], c->copy_stream));
      return SCDE_OK;
    };
    u.nranges = nranges;
    u.issued = 0;
    u.err = 0;
    u.err_msg.clear();
    u.busy = true;
    u.t_start = std::chrono::steady_clock::now();
    ++u.job;
    u.cv.notify_all();
    return SCDE_OK;
  }
  int wait(int n) {
    auto& u = ctx->upl;
    std::unique_lock<std::mutex> lk(u.m);
    u.cv.wait(lk, [&] { return u.issued >= n || u.err != 0 || !u.busy; });
    if (u.err) return fail(u.err, "count upload failed: %s", u.err_msg.c_str());
    return u.issued >= n ? SCDE_OK : fail(SCDE_EINTERNAL, "upload range %d never issued", n - 1);
  }
  // the job is finished (every range issued or failed) before the call returns: the next call's
  // job, and the caller's buffers, must not overlap it
  ~UploadWorker() {
    if (!ctx) return;
    auto& u = ctx->upl;
    std::unique_lock<std::mutex> lk(u.m);
    u.cv.wait(lk, [&] { return !u.busy; });
  }
};

// bound j (0..K) of K pieces over [0, total): equal pieces, or with taper decreasing ones
// (weights K, K - 1, .., 1: the last piece, whose unique sets and tables start only after the
// last byte has landed, is the smallest)
static long long piece_bound(long long total, int j, int K) { return total * j / K; }

static int ensure_piece_streams(scde_ctx* ctx) {
  if (!ctx->uq_stream) HCHK(hipStreamCreateWithFlags(&ctx->uq_stream, hipStreamNonBlocking));
  for (int j = 0; j < scde_ctx::kMaxPieces; ++j) {
    if (!ctx->piece_ev[j]) HCHK(hipEventCreateWithFlags(&ctx->piece_ev[j], hipEventDisableTiming));
    if (!ctx->piece_up_ev[j]) HCHK(hipEventCreateWithFlags(&ctx->piece_up_ev[j], hipEventDisableTiming));
  }
  return SCDE_OK;
}


// up (nullable): the host-count entry's upload, in pieces of the selected cells (cellidx
// strictly increasing), each piece's unique sets and tables starting as it lands
static int posteriors_run(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const int* cellidx,
                          int ncells_sel, const double* models_sel, int local_theta, int square_logit_conc,
                          const double* prior_x, int ngrid, int nboot, int n_cores, int64_t gene_offset,
                          int64_t ngenes_total, int return_post, int ensemble, const int* batch_vals,
                          const int64_t* batch_off, const int* composition, int nbatch, double* jp, double* modes,
                          double* post, const HostUpload* up);

int scde_posteriors_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const int* cellidx,
                        int ncells_sel, const double* models_sel, int local_theta, int square_logit_conc,
                        const double* prior_x, int ngrid, int nboot, int n_cores, int64_t gene_offset,
                        int64_t ngenes_total, int return_post, int ensemble, const int* batch_vals,
                        const int64_t* batch_off, const int* composition, int nbatch, double* jp, double* modes,
                        double* post) {
  FORK_GUARD();
  return posteriors_run(ctx, counts_dev, ld, ngenes, cellidx, ncells_sel, models_sel, local_theta, square_logit_conc,
                        prior_x, ngrid, nboot, n_cores, gene_offset, ngenes_total, return_post, ensemble, batch_vals,
                        batch_off, composition, nbatch, jp, modes, post, nullptr);
}

static int posteriors_run(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const int* cellidx,
                          int ncells_sel, const double* models_sel, int local_theta, int square_logit_conc,
                          const double* prior_x, int ngrid, int nboot, int n_cores, int64_t gene_offset,
                          int64_t ngenes_total, int return_post, int ensemble, const int* batch_vals,
                          const int64_t* batch_off, const int* composition, int nbatch, double* jp, double* modes,
                          double* post, const HostUpload* up) {
  if (!ctx || !counts_dev || !cellidx || !models_sel || !prior_x || !jp) return fail(SCDE_EARG, "null argument");
  if (ngenes < 0 || ncells_sel <= 0 || ngrid <= 0) return fail(SCDE_EARG, "bad dimensions");
  HCHK(hipSetDevice(ctx->device));
  const bool batch = batch_vals != nullptr;
  std::vector<double> mm(models_sel, models_sel + (size_t)ncells_sel * 12);
  for (int c = 0; c < ncells_sel; ++c) {
    double& ca = mm[(size_t)c + (size_t)ncells_sel * 4];
    if (ca < 1e-10) ca = 1e-10;  // R/functions.R:579-583
  }
  const std::vector<double> mag = marginals(prior_x, ngrid);
  PostSpec s;
  s.ncells = ncells_sel;
  s.models = mm.data();
  s.localtheta = local_theta;
  s.squarelogit = square_logit_conc;
  s.mag = mag.data();
  s.G = ngrid;
  s.nboot = nboot;
  s.postflag = return_post;
  s.ensemble = batch ? 0 : ensemble;
  s.batch_call = batch;
  s.counts_dev = counts_dev;
  s.ld = ld;
  s.cellidx_host = cellidx;
  s.ngenes = ngenes;
  seeding(n_cores, gene_offset, ngenes_total, ngenes, s.seeds, s.wset);
  s.rand_kind = g_rand_kind;
  s.batch_vals = batch_vals;
  s.batch_off = batch_off;
  s.comp = composition;
  s.nbatch = nbatch;
  const size_t NG = (size_t)ngenes * ngrid;
  HCHK(ctx->jpA.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  s.jp = ctx->jpA.as<double>();
  s.jp_g = 1;
  s.jp_k = ngenes;
  const bool want_modes = (batch ? return_post == 1 : (return_post == 1 || return_post == 3)) && modes;
  const bool want_post = (batch ? return_post == 2 : (return_post == 2 || return_post == 3)) && post;
  if (want_modes) {
    HCHK(ctx->jpB.ensure(sizeof(double) * std::max<size_t>(1, (size_t)ngenes * ncells_sel)));
    s.modes = ctx->jpB.as<double>();
    s.modes_early = ngenes > 0;
  }
  if (want_post) {
    HCHK(ctx->outbuf.ensure(sizeof(double) * std::max<size_t>(1, NG * ncells_sel)));
    s.post = ctx->outbuf.as<double>();
  }
  ctx->us[0].ready = false;
  std::vector<int> piece_c, piece_col;
  UploadWorker uw;
  if (up) {
    const int K = std::max(1, std::min(ctx->opt_pieces, scde_ctx::kMaxPieces));
    for (int j = 0; j <= K; ++j) piece_c.push_back((int)piece_bound(ncells_sel, j, K));
    piece_col.push_back(0);  // piece j uploads columns [piece_col[j], piece_col[j + 1])
    for (int j = 0; j < K; ++j)
      piece_col.push_back(piece_c[j + 1] > piece_c[j] ? cellidx[piece_c[j + 1] - 1] + 1 : piece_col.back());
    RCHK(ensure_piece_streams(ctx));
    RCHK(uw.start(ctx, *up, piece_col, std::vector<hipEvent_t>(ctx->piece_up_ev, ctx->piece_up_ev + K)));
    s.npieces = K;
    s.piece_c = piece_c.data();
    s.piece_stream = ctx->uq_stream;
    s.piece_ev = ctx->piece_ev;
    s.piece_ready = [&](int j) {
      RCHK(uw.wait(j + 1));
      HCHK(handoff_wait(ctx, ctx->uq_stream, ctx->piece_up_ev[j]));
      return SCDE_OK;
    };
  }
  // read-backs from the Downloader thread while the tables and the bootstrap run (modes piece by
  // piece, jp in gene chunks); every queued read-back has landed before this call returns, on
  // every return path (they write into the caller's buffers)
  struct DrainDownloads {
    scde_ctx* cx;
    bool on;
    ~DrainDownloads() {
      if (on) (void)dnl_wait(cx);
    }
  } drain{ctx, ctx->opt_modes_overlap != 0};
  if (drain.on) {
    if (s.modes_early) s.modes_host = modes;
    s.jp_host = jp;
    s.jp_chunks = ctx->opt_jp_chunks;
  }
  RCHK(run_posterior(ctx, s, ctx->us[0]));
  if (s.modes_early && !drain.on)  // after the bootstrap, on the main stream (profiling runs: no blits beside it)
    HCHK(hipMemcpyAsync(modes, s.modes, sizeof(double) * (size_t)ngenes * ncells_sel, hipMemcpyDeviceToHost,
                        ctx->stream));
  if (NG && !drain.on) HCHK(hipMemcpyAsync(jp, s.jp, sizeof(double) * NG, hipMemcpyDeviceToHost, ctx->stream));
  if (want_post && NG)
    HCHK(hipMemcpyAsync(post, s.post, sizeof(double) * NG * ncells_sel, hipMemcpyDeviceToHost, ctx->stream));
  if (drain.on) {
    drain.on = false;
    RCHK(dnl_wait(ctx));
  }
  return ctx->sync();
}

// The second lane of a DE call (opt_lanes = 2): the peer context runs the second group's
// posterior on its own streams and workspace, concurrently with the first group's on this
// context's stream.  Both groups' launches then share the CUs: the second group's small set-up
// kernels and its tables fill the first group's tails instead of waiting behind them.
// The continuations of two lanes' posteriors (draws, set-up kernels, bootstrap launch): with
// option rest_thread the second runs on a host thread of its own beside the first, so its set-up
// does not queue behind the first lane's host-side set-up and bootstrap launch and the two
// bootstraps can overlap; else one after the other.  (Each continuation touches only its own
// context's buffers and streams; a shared unique set is read-only there.)
static int run_rests(scde_ctx* ctx, const std::function<int()>& rest0, const std::function<int()>& rest1) {
  int rc1 = SCDE_OK;
  std::string err1;
  std::thread t1([&] {
    rc1 = hipSetDevice(ctx->device) == hipSuccess ? rest1() : fail(SCDE_EHIP, "hipSetDevice failed");
    if (rc1 != SCDE_OK) err1 = g_err;  // g_err is thread-local
  });
  const int rc0 = rest0();
  const std::string err0 = g_err;
  t1.join();
  if (rc0 != SCDE_OK) return fail(rc0, "%s", err0.c_str());
  if (rc1 != SCDE_OK) return fail(rc1, "%s", err1.c_str());
  return SCDE_OK;
}

static int lane_peer(scde_ctx* cx, scde_ctx** out) {
  if (!cx->peer) {
    scde_ctx* p = nullptr;
    RCHK(scde_ctx_create(cx->device, &p));
    cx->peer = p;
    for (auto& e : cx->lane_ev)
      if (!e) HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  scde_ctx* p = cx->peer;
  p->opt_boot_skip = cx->opt_boot_skip;
  p->opt_skip_slack = cx->opt_skip_slack;
  p->opt_boot_nb = cx->opt_boot_nb;
  p->opt_skip_stats = cx->opt_skip_stats;
  p->opt_wpca_ms = cx->opt_wpca_ms;
  p->opt_boot_tiles = cx->opt_boot_tiles;
  p->opt_boot_tiles_cells = cx->opt_boot_tiles_cells;
  p->opt_tile_groups = cx->opt_tile_groups;
  p->opt_tile_max_mult = cx->opt_tile_max_mult;
  p->opt_tile_order = cx->opt_tile_order;
  p->opt_jp_chunks = cx->opt_jp_chunks;
  p->opt_unique_fixed = cx->opt_unique_fixed;
  p->opt_gene_rows = cx->opt_gene_rows;
  p->opt_gene_list_cap = cx->opt_gene_list_cap;
  p->opt_tables_nt = cx->opt_tables_nt;
  p->spin_cycles = cx->spin_cycles;
  p->profile = cx->profile;
  *out = p;
  return SCDE_OK;
}

// the peer's statistics added into the context's (and cleared on the peer)
static void merge_peer_stats(scde_ctx* cx) {
  scde_ctx* p = cx->peer;
  if (!p) return;
  cx->st_skip_slabs += p->st_skip_slabs;
  cx->st_skip_kept += p->st_skip_kept;
  cx->st_skip_stretches += p->st_skip_stretches;
  cx->st_skip_redo += p->st_skip_redo;
  cx->st_degen += p->st_degen;
  cx->st_pair_redo += p->st_pair_redo;
  cx->st_boot_f64_fma += p->st_boot_f64_fma;
  for (int i = 0; i <= scde_ctx::kQMaxTilesHost; ++i) cx->st_tile_hist[i] += p->st_tile_hist[i];
  if (p->st_boot_path >= 0) cx->st_boot_path = p->st_boot_path;
  (void)scde_ctx_reset_stats(p);
  p->st_boot_path = -1;
}

// up (nullable): the host-count entry's upload.  With it the groups start one after the other,
// each once its columns are in HBM; without, both unique tables are built first (their host
// syncs back to back), then the two posteriors.  With two lanes the second group's posterior
// runs on the peer context, beside the first's.
static int de_run(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const scde_de_params* p,
                  double* results, double* jp1, double* jp2, double* ratio, const HostUpload* up);

int scde_expression_difference_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes,
                                   const scde_de_params* p, double* results, double* jp1, double* jp2,
                                   double* ratio) {
  FORK_GUARD();
  return de_run(ctx, counts_dev, ld, ngenes, p, results, jp1, jp2, ratio, nullptr);
}

static int de_run(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const scde_de_params* p,
                  double* results, double* jp1, double* jp2, double* ratio, const HostUpload* up) {
  if (!ctx || !counts_dev || !p || !p->models || !p->groups || !p->prior_x || !p->prior_y)
    return fail(SCDE_EARG, "null argument");
  if (ngenes < 0 || p->ncells <= 0 || p->ngrid <= 1) return fail(SCDE_EARG, "bad dimensions");
  HCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int C = p->ncells, G = p->ngrid;
  using hclock = std::chrono::steady_clock;
  auto hlap = [&, t = hclock::now()](int slot) mutable {
    const auto now = hclock::now();
    ctx->st_host_ms[slot] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  };
  // split cells by group (R/functions.R:372-374, tapply over levels)
  std::vector<int> idx[2];
  for (int c = 0; c < C; ++c)
    if (p->groups[c] == 0 || p->groups[c] == 1) idx[p->groups[c]].push_back(c);
  if (idx[0].empty() || idx[1].empty()) return fail(SCDE_EARG, "both groups need at least one cell");
  const std::vector<double> mag = marginals(p->prior_x, G);
  std::vector<int> seeds, wset;
  seeding(p->n_cores, p->gene_offset, p->ngenes_total > 0 ? p->ngenes_total : ngenes, ngenes, seeds, wset);
  const size_t NG = (size_t)ngenes * G;
  HCHK(ctx->jpA.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  HCHK(ctx->jpB.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  std::vector<double> mm[2];
  PostSpec specs[2];
  for (int gi = 0; gi < 2; ++gi) {
    const int Cg = (int)idx[gi].size();
    mm[gi].assign((size_t)Cg * 12, NAN);
    for (int j = 0; j < 12; ++j)
      for (int c = 0; c < Cg; ++c) mm[gi][(size_t)c + (size_t)Cg * j] = p->models[(size_t)idx[gi][c] + (size_t)C * j];
    for (int c = 0; c < Cg; ++c) {
      double& ca = mm[gi][(size_t)c + (size_t)Cg * 4];
      if (ca < 1e-10) ca = 1e-10;
    }
    PostSpec& s = specs[gi];
    s.ncells = Cg;
    s.models = mm[gi].data();
    s.localtheta = p->local_theta;
    s.squarelogit = p->square_logit_conc;
    s.mag = mag.data();
    s.G = G;
    s.nboot = p->nboot;
    s.counts_dev = counts_dev;
    s.ld = ld;
    s.cellidx_host = idx[gi].data();
    s.ngenes = ngenes;
    s.seeds = seeds;
    s.wset = wset;
    s.rand_kind = p->rand_kind;
    s.jp = (gi == 0 ? ctx->jpA : ctx->jpB).as<double>();
    s.jp_g = G;  // gene-major rows for the ratio kernel
    s.jp_k = 1;
  }
  hlap(0);
  const double* jp_dev[2] = {ctx->jpA.as<double>(), ctx->jpB.as<double>()};
  {
    scde_ctx* lane = ctx;  // the context that runs the second group's posterior
    if (ctx->opt_lanes >= 2) RCHK(lane_peer(ctx, &lane));
    if (up) {
      // group by group, each after its columns have arrived (the first range ends with the
      // last cell of the group whose cells end first)
      int max0 = 0, max1 = 0;
      for (int c : idx[0]) max0 = std::max(max0, c);
      for (int c : idx[1]) max1 = std::max(max1, c);
      const int first = max0 <= max1 ? 0 : 1;
      // the first group's range in pieces, then the second group's range, uploaded back to back by
      // a worker thread: each piece's unique sets and tables start as it lands
      const int K = std::max(1, std::min(ctx->opt_pieces, scde_ctx::kMaxPieces));
      std::vector<int> piece_c, cols;
      const std::vector<int>& ix = idx[first];
      for (int j = 0; j <= K; ++j) {
        const int a = (int)piece_bound(up->cut, j, K);
        cols.push_back(a);
        piece_c.push_back((int)(std::lower_bound(ix.begin(), ix.end(), a) - ix.begin()));
      }
      RCHK(ensure_piece_streams(ctx));
      UploadWorker uw;
      cols.push_back(up->C);
      std::vector<hipEvent_t> evs(ctx->piece_up_ev, ctx->piece_up_ev + K);
      evs.push_back(ctx->up_ev[1]);
      RCHK(uw.start(ctx, *up, cols, evs));
      {
        const int gi = first;
        ctx->us[gi].ready = false;
        PostSpec& sf = specs[gi];
        sf.npieces = K;
        sf.piece_c = piece_c.data();
        sf.piece_stream = ctx->uq_stream;
        sf.piece_ev = ctx->piece_ev;
        sf.piece_ready = [&](int j) {
          RCHK(uw.wait(j + 1));
          HCHK(handoff_wait(ctx, ctx->uq_stream, ctx->piece_up_ev[j]));
          return SCDE_OK;
        };
        hlap(1);
        RCHK(run_posterior(ctx, sf, ctx->us[gi]));
        hlap(2);
      }
      {
        // the second group, once its range is in HBM: its unique sets on the peer lane (or on
        // the unique stream with one lane), so their host sync waits for its small kernels only
        const int gi = 1 - first;
        ctx->us[gi].ready = false;
        RCHK(uw.wait(K + 1));
        const PostSpec* sp[1] = {&specs[gi]};
        UniqueSet* usp[1] = {&ctx->us[gi]};
        if (lane != ctx) {
          HCHK(handoff_wait(lane, lane->stream, ctx->up_ev[1]));
          RCHK(build_unique_sets(lane, sp, usp, 1));
          hlap(1);
          RCHK(run_posterior(lane, specs[gi], ctx->us[gi]));
          HCHK(handoff_spin(lane, lane->stream));
          HCHK(hipEventRecord(ctx->lane_ev[1], lane->stream));
          HCHK(lane_join(ctx));
        } else {
          if (!ctx->uq_ev) HCHK(hipEventCreateWithFlags(&ctx->uq_ev, hipEventDisableTiming));
          HCHK(handoff_wait(ctx, ctx->uq_stream, ctx->up_ev[1]));
          const hipStream_t main = ctx->stream;
          ctx->stream = ctx->uq_stream;
          const int rc = build_unique_sets(ctx, sp, usp, 1);
          ctx->stream = main;
          RCHK(rc);
          HCHK(handoff_spin(ctx, ctx->uq_stream));
          HCHK(hipEventRecord(ctx->uq_ev, ctx->uq_stream));
          HCHK(handoff_wait(ctx, ctx->stream, ctx->uq_ev));
          hlap(1);
          RCHK(run_posterior(ctx, specs[gi], ctx->us[gi]));
        }
        hlap(2);
      }
    } else {
      // both groups' unique tables first (two host syncs, GPU otherwise idle), then the
      // heavy per-group kernels back to back on the stream
      ctx->us[0].ready = ctx->us[1].ready = false;
      const PostSpec* sp[2] = {&specs[0], &specs[1]};
      UniqueSet* up[2] = {&ctx->us[0], &ctx->us[1]};
      HCHK(handoff_spin(ctx, ctx->stream));  // (test hook: the peer's inputs start late)
      RCHK(build_unique_sets(ctx, sp, up, 2));
      hlap(1);
      if (lane != ctx) {
        HCHK(handoff_spin(ctx, ctx->stream));
        HCHK(hipEventRecord(ctx->lane_ev[0], ctx->stream));
        HCHK(handoff_wait(lane, lane->stream, ctx->lane_ev[0]));
      }
      if (lane != ctx) {
        // both groups' tables first, then both bootstraps
        std::function<int()> rest0, rest1;
        RCHK(run_posterior(ctx, specs[0], ctx->us[0], &rest0));
        RCHK(run_posterior(lane, specs[1], ctx->us[1], &rest1));
        RCHK(run_rests(ctx, rest0, rest1));
      } else {
        RCHK(run_posterior(ctx, specs[0], ctx->us[0]));
        RCHK(run_posterior(ctx, specs[1], ctx->us[1]));
      }
      if (lane != ctx) {
        HCHK(handoff_spin(lane, lane->stream));
        HCHK(hipEventRecord(ctx->lane_ev[1], lane->stream));
        HCHK(lane_join(ctx));
      }
      hlap(2);
    }
  }
  // ratio posterior + summary
  const std::vector<double> diffv = ratio_diffv(p->prior_x, G);
  const int zi = expectation_index(diffv, p->expectation);
  const size_t m = 2 * (size_t)G - 1;
  RCHK(upload(ctx, ctx->prior_y, p->prior_y, sizeof(double) * G));
  RCHK(upload(ctx, ctx->diffv, diffv.data(), sizeof(double) * m));
  const int ncol = p->compute_cz ? 6 : 5;
  HCHK(ctx->res.ensure(sizeof(double) * std::max<size_t>(1, (size_t)ngenes * ncol)));
  if (ratio) HCHK(ctx->ratio.ensure(sizeof(double) * std::max<size_t>(1, (size_t)ngenes * m)));
  RatioArgs ra{};
  ra.jp1 = jp_dev[0];
  ra.j1g = G;
  ra.j1k = 1;
  ra.jp2 = jp_dev[1];
  ra.j2g = G;
  ra.j2k = 1;
  ra.prior_y = ctx->prior_y.as<double>();
  ra.n = G;
  ra.ngenes = ngenes;
  ra.normalize = 1;
  ra.ratio = ratio ? ctx->ratio.as<double>() : nullptr;
  ra.rg = 1;
  ra.ro = ngenes;
  ra.diffv = ctx->diffv.as<double>();
  ra.zi = zi;
  ra.res = ctx->res.as<double>();
  ra.res_ld = ngenes;
  hipEvent_t ev = ctx->mark_begin(SLOT_RATIO);
  ra.window = ctx->opt_ratio_window;
  ra.block = ctx->opt_ratio_block;
  HCHK(launch_ratio_summary(ra, st));
  ctx->mark_end(SLOT_RATIO, ev);
  if (p->compute_cz && ngenes) {
    size_t wb = 0;
    HCHK(launch_bh_cz(nullptr, ngenes, nullptr, nullptr, &wb, st));
    HCHK(ctx->bhw.ensure(wb));
    HCHK(launch_bh_cz(ra.res + (size_t)4 * ngenes, ngenes, ra.res + (size_t)5 * ngenes, ctx->bhw.p, &wb, st));
  }
  if (results && ngenes)
    HCHK(hipMemcpyAsync(results, ra.res, sizeof(double) * ngenes * ncol, hipMemcpyDeviceToHost, st));
  if (ratio && ngenes) HCHK(hipMemcpyAsync(ratio, ra.ratio, sizeof(double) * ngenes * m, hipMemcpyDeviceToHost, st));
  std::vector<double> tmp;
  if ((jp1 || jp2) && NG) tmp.resize(NG);
  if (jp1 && NG) {
    HCHK(hipMemcpyAsync(tmp.data(), jp_dev[0], sizeof(double) * NG, hipMemcpyDeviceToHost, st));
    RCHK(ctx->sync());
    transpose_rows_to_colmajor(tmp.data(), ngenes, G, jp1);
  }
  if (jp2 && NG) {
    HCHK(hipMemcpyAsync(tmp.data(), jp_dev[1], sizeof(double) * NG, hipMemcpyDeviceToHost, st));
    RCHK(ctx->sync());
    transpose_rows_to_colmajor(tmp.data(), ngenes, G, jp2);
  }
  const int rc = ctx->sync();
  merge_peer_stats(ctx);
  hlap(3);
  return rc;
}

// Batch-corrected scde.expression.difference (R/functions.R:321-399), device resident:
// batch posteriors over all cells with each group's batch composition, the group
// posteriors, three ratio posteriors (batch, groups, and the 1601-column second level of
// the two with skip.prior.adjustment) and their summaries with device BH.
int scde_expression_difference_batch_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes,
                                         const scde_de_params* p, const double* batch_models,
                                         const int* batch_codes, int nbatch, double* results, double* jp1,
                                         double* jp2, double* ratio, double* adj_ratio, double* batch_ratio) {
  FORK_GUARD();
  if (!ctx || !counts_dev || !p || !p->models || !p->groups || !p->prior_x || !p->prior_y || !batch_codes ||
      !results)
    return fail(SCDE_EARG, "null argument");
  if (ngenes < 0 || p->ncells <= 0 || p->ngrid <= 1 || nbatch < 1) return fail(SCDE_EARG, "bad dimensions");
  HCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int C = p->ncells, G = p->ngrid, N = ngenes;
  const double* bm = batch_models ? batch_models : p->models;
  std::vector<int> idx[2];
  for (int c = 0; c < C; ++c)
    if (p->groups[c] == 0 || p->groups[c] == 1) idx[p->groups[c]].push_back(c);
  if (idx[0].empty() || idx[1].empty()) return fail(SCDE_EARG, "both groups need at least one cell");
  // BatchIL (0-based cell indices per batch level) and table(batch[ii]) per group; code -1 is
  // an NA batch: tapply (R/functions.R:570) and table leave such cells out of every level
  std::vector<int> bvals;
  std::vector<int64_t> boff(nbatch + 1, 0);
  for (int c = 0; c < C; ++c)
    if (batch_codes[c] < -1 || batch_codes[c] >= nbatch) return fail(SCDE_EARG, "batch code out of range");
  for (int k = 0; k < nbatch; ++k) {
    for (int c = 0; c < C; ++c)
      if (batch_codes[c] == k) bvals.push_back(c);
    boff[k + 1] = (int64_t)bvals.size();
  }
  std::vector<int> comp[2];
  for (int gi = 0; gi < 2; ++gi) {
    comp[gi].assign(nbatch, 0);
    for (int c : idx[gi])
      if (batch_codes[c] >= 0) comp[gi][batch_codes[c]]++;
  }
  const std::vector<double> mag = marginals(p->prior_x, G);
  std::vector<int> seeds, wset;
  seeding(p->n_cores, p->gene_offset, p->ngenes_total > 0 ? p->ngenes_total : N, N, seeds, wset);
  const size_t NG = (size_t)N * G;
  HCHK(ctx->jpA.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  HCHK(ctx->jpB.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  HCHK(ctx->in1.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  HCHK(ctx->in2.ensure(sizeof(double) * std::max<size_t>(1, NG)));
  // model matrices with the slope clamp (R/functions.R:579-583)
  auto clamp_mm = [](std::vector<double>& m, int n) {
    for (int c = 0; c < n; ++c)
      if (m[(size_t)c + (size_t)n * 4] < 1e-10) m[(size_t)c + (size_t)n * 4] = 1e-10;
  };
  std::vector<double> mm[2], mmb(bm, bm + (size_t)C * 12);
  clamp_mm(mmb, C);
  std::vector<int> allc(C);
  for (int c = 0; c < C; ++c) allc[c] = c;
  PostSpec sg[2], sb[2];
  for (int gi = 0; gi < 2; ++gi) {
    const int Cg = (int)idx[gi].size();
    mm[gi].assign((size_t)Cg * 12, NAN);
    for (int j = 0; j < 12; ++j)
      for (int c = 0; c < Cg; ++c) mm[gi][(size_t)c + (size_t)Cg * j] = p->models[(size_t)idx[gi][c] + (size_t)C * j];
    clamp_mm(mm[gi], Cg);
    for (int pass = 0; pass < 2; ++pass) {
      PostSpec& s = pass == 0 ? sg[gi] : sb[gi];
      s.ncells = pass == 0 ? Cg : C;
      s.models = pass == 0 ? mm[gi].data() : mmb.data();
      s.localtheta = p->local_theta;
      s.squarelogit = p->square_logit_conc;
      s.mag = mag.data();
      s.G = G;
      s.nboot = p->nboot;
      s.counts_dev = counts_dev;
      s.ld = ld;
      s.cellidx_host = pass == 0 ? idx[gi].data() : allc.data();
      s.ngenes = N;
      s.seeds = seeds;
      s.wset = wset;
      s.rand_kind = p->rand_kind;
      s.jp_g = G;
      s.jp_k = 1;
      if (pass == 1) {
        s.batch_call = true;
        s.batch_vals = bvals.data();
        s.batch_off = boff.data();
        s.comp = comp[gi].data();
        s.nbatch = nbatch;
      }
    }
    sg[gi].jp = (gi == 0 ? ctx->jpA : ctx->jpB).as<double>();
    sb[gi].jp = (gi == 0 ? ctx->in1 : ctx->in2).as<double>();
  }
  // unique tables: group 0 cells, group 1 cells, all cells (shared by both batch runs)
  {
    for (auto& u : ctx->us) u.ready = false;
    const PostSpec* sp[3] = {&sg[0], &sg[1], &sb[0]};
    UniqueSet* up[3] = {&ctx->us[0], &ctx->us[1], &ctx->us[2]};
    RCHK(build_unique_sets(ctx, sp, up, 3));
  }
  scde_ctx* lane = ctx;  // the second batch posterior and the second group's run on the peer lane
  if (ctx->opt_lanes >= 2) RCHK(lane_peer(ctx, &lane));
  if (lane != ctx) {
    HCHK(handoff_spin(ctx, ctx->stream));
    HCHK(hipEventRecord(ctx->lane_ev[0], ctx->stream));
    HCHK(handoff_wait(lane, lane->stream, ctx->lane_ev[0]));
    std::function<int()> rest0, rest1;
    RCHK(run_posterior(ctx, sb[0], ctx->us[2], &rest0));
    ctx->us[2].ready = true;  // same cells, same counts: reuse for the second batch run
    RCHK(run_posterior(lane, sb[1], ctx->us[2], &rest1));
    RCHK(run_rests(ctx, rest0, rest1));
    RCHK(run_posterior(ctx, sg[0], ctx->us[0], &rest0));
    RCHK(run_posterior(lane, sg[1], ctx->us[1], &rest1));
    RCHK(run_rests(ctx, rest0, rest1));
    HCHK(handoff_spin(lane, lane->stream));
    HCHK(hipEventRecord(ctx->lane_ev[1], lane->stream));
    HCHK(lane_join(ctx));
  } else {
    RCHK(run_posterior(ctx, sb[0], ctx->us[2]));
    ctx->us[2].ready = true;  // same cells, same counts: reuse for the second batch run
    RCHK(run_posterior(ctx, sb[1], ctx->us[2]));
    RCHK(run_posterior(ctx, sg[0], ctx->us[0]));
    RCHK(run_posterior(ctx, sg[1], ctx->us[1]));
  }
  // three ratio posteriors + summaries
  const std::vector<double> dv1 = ratio_diffv(p->prior_x, G);
  const int m = 2 * G - 1, m2 = 2 * m - 1;
  const std::vector<double> dv2 = ratio_diffv(dv1.data(), m);
  RCHK(upload(ctx, ctx->prior_y, p->prior_y, sizeof(double) * G));
  RCHK(upload(ctx, ctx->diffv, dv1.data(), sizeof(double) * m));
  RCHK(upload(ctx, ctx->outbuf, dv2.data(), sizeof(double) * m2));
  HCHK(ctx->ratio.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * m)));
  HCHK(ctx->part.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * m)));  // batch ratio
  if (adj_ratio) HCHK(ctx->E.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * m2)));
  HCHK(ctx->res.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * 18)));
  double* res = ctx->res.as<double>();
  size_t wb = 0;
  HCHK(launch_bh_cz(nullptr, N, nullptr, nullptr, &wb, st));
  HCHK(ctx->bhw.ensure(wb));
  auto ratio_pass = [&](const double* a1, long long a1g, long long a1k, const double* a2, long long a2g,
                        long long a2k, const double* py, int n, const double* dv, int zi, double* rout,
                        double* rres) -> int {
    RatioArgs ra{};
    ra.jp1 = a1;
    ra.j1g = a1g;
    ra.j1k = a1k;
    ra.jp2 = a2;
    ra.j2g = a2g;
    ra.j2k = a2k;
    ra.prior_y = py;
    ra.n = n;
    ra.ngenes = N;
    ra.normalize = 1;
    ra.ratio = rout;
    ra.rg = 1;
    ra.ro = N;
    ra.diffv = dv;
    ra.zi = zi;
    ra.res = rres;
    ra.res_ld = N;
    hipEvent_t ev = ctx->mark_begin(SLOT_RATIO);
    ra.window = ctx->opt_ratio_window;
    ra.block = ctx->opt_ratio_block;
    HCHK(launch_ratio_summary(ra, st));
    ctx->mark_end(SLOT_RATIO, ev);
    if (N) HCHK(launch_bh_cz(rres + (size_t)4 * N, N, rres + (size_t)5 * N, ctx->bhw.p, &wb, st));
    return SCDE_OK;
  };
  // results blocks: [0] batch.adjusted, [1] results, [2] batch.effect (each N x 6)
  double* r_adj = res;
  double* r_res = res + (size_t)6 * N;
  double* r_bat = res + (size_t)12 * N;
  const double* py = ctx->prior_y.as<double>();
  RCHK(ratio_pass(ctx->in1.as<double>(), G, 1, ctx->in2.as<double>(), G, 1, py, G, ctx->diffv.as<double>(),
                  expectation_index(dv1, 0.0), ctx->part.as<double>(), r_bat));
  RCHK(ratio_pass(ctx->jpA.as<double>(), G, 1, ctx->jpB.as<double>(), G, 1, py, G, ctx->diffv.as<double>(),
                  expectation_index(dv1, p->expectation), ctx->ratio.as<double>(), r_res));
  RCHK(ratio_pass(ctx->ratio.as<double>(), 1, N, ctx->part.as<double>(), 1, N, nullptr, m,
                  ctx->outbuf.as<double>(), expectation_index(dv2, p->expectation),
                  adj_ratio ? ctx->E.as<double>() : nullptr, r_adj));
  if (N) {
    HCHK(hipMemcpyAsync(results, res, sizeof(double) * (size_t)N * 18, hipMemcpyDeviceToHost, st));
    if (ratio) HCHK(hipMemcpyAsync(ratio, ctx->ratio.p, sizeof(double) * (size_t)N * m, hipMemcpyDeviceToHost, st));
    if (batch_ratio)
      HCHK(hipMemcpyAsync(batch_ratio, ctx->part.p, sizeof(double) * (size_t)N * m, hipMemcpyDeviceToHost, st));
    if (adj_ratio)
      HCHK(hipMemcpyAsync(adj_ratio, ctx->E.p, sizeof(double) * (size_t)N * m2, hipMemcpyDeviceToHost, st));
  }
  std::vector<double> tmp;
  for (int gi = 0; gi < 2 && NG; ++gi) {
    double* out = gi == 0 ? jp1 : jp2;
    if (!out) continue;
    tmp.resize(NG);
    HCHK(hipMemcpyAsync(tmp.data(), (gi == 0 ? ctx->jpA : ctx->jpB).p, sizeof(double) * NG, hipMemcpyDeviceToHost,
                        st));
    RCHK(ctx->sync());
    transpose_rows_to_colmajor(tmp.data(), N, G, out);
  }
  const int rc = ctx->sync();
  merge_peer_stats(ctx);
  return rc;
}

// ------------------------------------------------------------------ host-count entry points
// The R-level calls as the .Call shim makes them: counts are the caller's host matrix
// (int32, column-major, leading dimension ld >= ngenes, ncols columns).  They are copied
// into the context's staging buffer (dense, ld = ngenes) on its stream and the resident
// pipeline runs on them; everything the caller gets back is host memory.
static int stage_counts(scde_ctx*& ctx, const int* counts, int64_t ld, int ngenes, int ncols, const int** dev) {
  if (!ctx) RCHK(default_ctx(&ctx));
  if (!counts) return fail(SCDE_EARG, "null argument");
  if (ngenes < 0 || ncols <= 0 || ld < ngenes) return fail(SCDE_EARG, "bad dimensions");
  HCHK(hipSetDevice(ctx->device));
  const size_t row = sizeof(int) * (size_t)ngenes;
  HCHK(ctx->counts_in.ensure(std::max<size_t>(1, row * ncols)));
  if (ngenes > 0) {
    if (ld == ngenes)
      HCHK(hipMemcpyAsync(ctx->counts_in.p, counts, row * ncols, hipMemcpyHostToDevice, ctx->stream));
    else
      HCHK(hipMemcpy2DAsync(ctx->counts_in.p, row, counts, sizeof(int) * (size_t)ld, row, ncols,
                            hipMemcpyHostToDevice, ctx->stream));
  }
  *dev = ctx->counts_in.as<int>();
  return SCDE_OK;
}

int scde_expression_difference_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes,
                                    const scde_de_params* p, double* results, double* jp1, double* jp2,
                                    double* ratio) {
  FORK_GUARD();
  if (!p || !p->groups) return fail(SCDE_EARG, "null argument");
  if (!ctx) RCHK(default_ctx(&ctx));
  if (!counts) return fail(SCDE_EARG, "null argument");
  const int C = p->ncells;
  if (ngenes < 0 || C <= 0 || ld < ngenes) return fail(SCDE_EARG, "bad dimensions");
  HCHK(hipSetDevice(ctx->device));
  // Small matrices upload in one piece and keep the batched unique-table build: the
  // per-group build costs extra host syncs, which a short transfer does not repay (two lanes,
  // one piece vs pipelined: 2,500 x 1,000 counts 1.84 vs 2.29 ms per call, 5,000 x 1,000 2.89-2.92
  // vs 3.20-3.22, 20k x 200 4.66 vs 4.87; from 32 MB the pipeline wins: 10,000 x 1,000
  // 4.72-4.92 vs 5.00-5.14)
  const size_t kPipelineBytes = (size_t)std::max(0.0, ctx->opt_pipeline_mb) * (size_t(1) << 20);
  if (ngenes == 0 || sizeof(int) * (size_t)ngenes * C < kPipelineBytes) {
    const int* dev = nullptr;
    RCHK(stage_counts(ctx, counts, ld, ngenes, C, &dev));
    return de_run(ctx, dev, ngenes, ngenes, p, results, jp1, jp2, ratio, nullptr);
  }
  // two column ranges: up to the last cell of the group whose cells end first, and the rest
  int max0 = -1, max1 = -1;
  for (int c = 0; c < C; ++c) {
    if (p->groups[c] == 0) max0 = c;
    if (p->groups[c] == 1) max1 = c;
  }
  if (max0 < 0 || max1 < 0) return fail(SCDE_EARG, "both groups need at least one cell");
  const int cut = std::min(max0, max1) + 1;
  if (!ctx->copy_stream) HCHK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  for (auto& e : ctx->up_ev)
    if (!e) HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const size_t row = sizeof(int) * (size_t)ngenes;
  HCHK(ctx->counts_in.ensure(std::max<size_t>(1, row * C)));
  // the previous call's kernels may still read counts_in: the copies wait for them
  HCHK(handoff_spin(ctx, ctx->stream));
  HCHK(hipEventRecord(ctx->up_ev[1], ctx->stream));
  HCHK(handoff_wait(ctx, ctx->copy_stream, ctx->up_ev[1]));
  // (a DE call's upload hides behind the first group's unique sets and tables: as int32, unless
  // upload_u16 = 2 -- config 3 measured 6.78 ms per step with int32 against 7.22 with 16-bit counts,
  // whose narrowing threads then share the CPU with the lanes' threads)
  const HostUpload h{counts, ld, ngenes, cut, C, ctx->opt_upload_u16 == 2};
  return de_run(ctx, ctx->counts_in.as<int>(), ngenes, ngenes, p, results, jp1, jp2, ratio, &h);
}

int scde_expression_difference_batch_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes,
                                          const scde_de_params* p, const double* batch_models,
                                          const int* batch_codes, int nbatch, double* results, double* jp1,
                                          double* jp2, double* ratio, double* adj_ratio, double* batch_ratio) {
  FORK_GUARD();
  if (!p) return fail(SCDE_EARG, "null argument");
  const int* dev = nullptr;
  RCHK(stage_counts(ctx, counts, ld, ngenes, p->ncells, &dev));
  return scde_expression_difference_batch_dev(ctx, dev, ngenes, ngenes, p, batch_models, batch_codes, nbatch,
                                              results, jp1, jp2, ratio, adj_ratio, batch_ratio);
}

int scde_posteriors_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes, int ncells_total,
                         const int* cellidx, int ncells_sel, const double* models_sel, int local_theta,
                         int square_logit_conc, const double* prior_x, int ngrid, int nboot, int n_cores,
                         int64_t gene_offset, int64_t ngenes_total, int return_post, int ensemble,
                         const int* batch_vals, const int64_t* batch_off, const int* composition, int nbatch,
                         double* jp, double* modes, double* post) {
  FORK_GUARD();
  if (!cellidx) return fail(SCDE_EARG, "null argument");
  for (int i = 0; i < ncells_sel; ++i)
    if (cellidx[i] < 0 || cellidx[i] >= ncells_total) return fail(SCDE_EARG, "cell index %d out of range", cellidx[i]);
  if (!ctx) RCHK(default_ctx(&ctx));
  bool increasing = ncells_sel > 0;
  for (int i = 1; i < ncells_sel && increasing; ++i) increasing = cellidx[i] > cellidx[i - 1];
  if (ngenes > 0 && counts && ld >= ngenes && increasing && ctx->opt_pieces > 1 &&
      sizeof(int) * (size_t)ngenes * ncells_total >= (size_t)std::max(0.0, ctx->opt_pipeline_mb) * (size_t(1) << 20)) {
    // the selected cells' columns in pieces on the copy stream, each piece's unique sets and
    // tables starting as it lands
    HCHK(hipSetDevice(ctx->device));
    if (!ctx->copy_stream) HCHK(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    for (auto& e : ctx->up_ev)
      if (!e) HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HCHK(ctx->counts_in.ensure(sizeof(int) * (size_t)ngenes * ncells_total));
    // the previous call's kernels may still read counts_in: the copies wait for them
    HCHK(handoff_spin(ctx, ctx->stream));
    HCHK(hipEventRecord(ctx->up_ev[1], ctx->stream));
    HCHK(handoff_wait(ctx, ctx->copy_stream, ctx->up_ev[1]));
    const HostUpload h{counts, ld, ngenes, 0, ncells_total, ctx->opt_upload_u16 != 0};
    return posteriors_run(ctx, ctx->counts_in.as<int>(), ngenes, ngenes, cellidx, ncells_sel, models_sel, local_theta,
                          square_logit_conc, prior_x, ngrid, nboot, n_cores, gene_offset, ngenes_total, return_post,
                          ensemble, batch_vals, batch_off, composition, nbatch, jp, modes, post, &h);
  }
  const int* dev = nullptr;
  RCHK(stage_counts(ctx, counts, ld, ngenes, ncells_total, &dev));
  return scde_posteriors_dev(ctx, dev, ngenes, ngenes, cellidx, ncells_sel, models_sel, local_theta,
                             square_logit_conc, prior_x, ngrid, nboot, n_cores, gene_offset, ngenes_total,
                             return_post, ensemble, batch_vals, batch_off, composition, nbatch, jp, modes, post);
}

// pagoda.varnorm's posterior-mode consumer (R/functions.R:1414-1507): modes from
// scde.posteriors' joint posteriors -- dataset-wide and per batch level -- and the weight
// matrices 1 - mfp * sfp.  The magnitudes are as.numeric(colnames(jp)) = exp(marginals)
// through R's 15-significant-digit as.character (R/functions.R:640-643).
static int vn_posterior_jp(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, const int* cellidx, int C,
                           const double* models, int mld, int local_theta, int sq, const double* prior_x, int G,
                           int nboot, int n_cores, double* jp_dev) {
  std::vector<double> mm((size_t)C * 12);
  for (int j = 0; j < 12; ++j)
    for (int c = 0; c < C; ++c) mm[(size_t)c + (size_t)C * j] = models[(size_t)cellidx[c] + (size_t)mld * j];
  for (int c = 0; c < C; ++c) {
    double& ca = mm[(size_t)c + (size_t)C * 4];
    if (ca < 1e-10) ca = 1e-10;  // R/functions.R:579-583
  }
  const std::vector<double> mag = marginals(prior_x, G);
  PostSpec s;
  s.ncells = C;
  s.models = mm.data();
  s.localtheta = local_theta;
  s.squarelogit = sq;
  s.mag = mag.data();
  s.G = G;
  s.nboot = nboot;
  s.postflag = 0;
  s.counts_dev = counts_dev;
  s.ld = ld;
  s.cellidx_host = cellidx;
  s.ngenes = ngenes;
  seeding(n_cores, 0, ngenes, ngenes, s.seeds, s.wset);
  s.rand_kind = g_rand_kind;
  s.jp = jp_dev;
  s.jp_g = 1;
  s.jp_k = ngenes;
  ctx->us[0].ready = false;
  return run_posterior(ctx, s, ctx->us[0]);
}

int scde_pagoda_varnorm_weights_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, int ncells,
                                    const double* models, int local_theta, int square_logit_conc,
                                    const double* prior_x, int ngrid, int nboot, int n_cores, const int* batch_codes,
                                    int nbatch, int use_expected_value, double* modes, double* matw,
                                    double* bmatw) {
  FORK_GUARD();
  if (!ctx || !counts_dev || !models || !prior_x || !modes || !matw) return fail(SCDE_EARG, "null argument");
  if (ngenes < 0 || ncells <= 0 || ngrid <= 0 || ld < ngenes) return fail(SCDE_EARG, "bad dimensions");
  const bool batch = batch_codes && nbatch > 1;
  if (batch && !bmatw) return fail(SCDE_EARG, "bmatw required with a batch");
  HCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int N = ngenes, C = ncells, G = ngrid;
  // as.numeric(colnames(jp)): exp(marginals) with 15 significant digits
  const std::vector<double> marg = marginals(prior_x, G);
  std::vector<double> mag(G);
  for (int k = 0; k < G; ++k) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.15g", std::exp(marg[k]));
    mag[k] = strtod(buf, nullptr);
  }
  RCHK(upload(ctx, ctx->diffv, mag.data(), sizeof(double) * G));
  const int nm = batch ? 1 + nbatch : 1;
  HCHK(ctx->res.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * nm)));
  HCHK(ctx->jpB.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * G)));
  double* dmodes = ctx->res.as<double>();
  std::vector<int> allc(C);
  for (int c = 0; c < C; ++c) allc[c] = c;
  // dataset-wide modes, then one set per batch level
  for (int m = 0; m < nm; ++m) {
    std::vector<int> cells;
    if (m == 0) {
      cells = allc;
    } else {
      for (int c = 0; c < C; ++c) {
        if (batch_codes[c] < 0 || batch_codes[c] >= nbatch) return fail(SCDE_EARG, "batch code out of range");
        if (batch_codes[c] == m - 1) cells.push_back(c);
      }
      if (cells.empty()) return fail(SCDE_EARG, "batch level %d has no cells", m - 1);
    }
    if (N > 0) {
      RCHK(vn_posterior_jp(ctx, counts_dev, ld, N, cells.data(), (int)cells.size(), models, C, local_theta,
                           square_logit_conc, prior_x, G, nboot, n_cores, ctx->jpB.as<double>()));
      HCHK(launch_vn_modes(ctx->jpB.as<double>(), 1, N, N, G, ctx->diffv.as<double>(), use_expected_value,
                           dmodes + (size_t)m * N, st));
    }
  }
  // weight matrices
  RCHK(upload(ctx, ctx->models, models, sizeof(double) * (size_t)C * 12));
  RCHK(upload(ctx, ctx->in1, allc.data(), sizeof(int) * C));
  HCHK(ctx->outbuf.ensure(sizeof(double) * std::max<size_t>(1, (size_t)N * C)));
  std::vector<long long> off(C, 0);
  for (int pass = 0; pass < (batch ? 2 : 1); ++pass) {
    if (pass == 1)
      for (int c = 0; c < C; ++c) off[c] = (long long)(1 + batch_codes[c]) * N;
    RCHK(upload(ctx, ctx->in2, off.data(), sizeof(long long) * C));
    HCHK(launch_vn_matw(counts_dev, ld, N, ctx->in1.as<int>(), C, ctx->models.as<double>(), C, square_logit_conc,
                        dmodes, ctx->in2.as<long long>(), ctx->outbuf.as<double>(), st));
    if ((size_t)N * C)
      HCHK(hipMemcpyAsync(pass == 0 ? matw : bmatw, ctx->outbuf.p, sizeof(double) * (size_t)N * C,
                          hipMemcpyDeviceToHost, st));
    RCHK(ctx->sync());  // outbuf / in2 are reused by the next pass
  }
  if (N) HCHK(hipMemcpyAsync(modes, dmodes, sizeof(double) * (size_t)N * nm, hipMemcpyDeviceToHost, st));
  return ctx->sync();
}

int scde_pagoda_varnorm_weights_host(scde_ctx* ctx, const int* counts, int64_t ld, int ngenes, int ncells,
                                     const double* models, int local_theta, int square_logit_conc,
                                     const double* prior_x, int ngrid, int nboot, int n_cores,
                                     const int* batch_codes, int nbatch, int use_expected_value, double* modes,
                                     double* matw, double* bmatw) {
  FORK_GUARD();
  const int* dev = nullptr;
  RCHK(stage_counts(ctx, counts, ld, ngenes, ncells, &dev));
  return scde_pagoda_varnorm_weights_dev(ctx, dev, ngenes, ngenes, ncells, models, local_theta, square_logit_conc,
                                         prior_x, ngrid, nboot, n_cores, batch_codes, nbatch, use_expected_value,
                                         modes, matw, bmatw);
}

// ------------------------------------------------------------------ BH (host)
// scde.expression.prior (R/functions.R:225-254) on device-resident counts (prior.hip).
int scde_expression_prior_dev(scde_ctx* ctx, const int* counts_dev, int64_t ld, int ngenes, int ncells,
                              const double* models, int square_logit_conc, int length_out, double pseudo_count,
                              double bw, double max_quantile, const double* max_value, double* x, double* y,
                              double* lp, double* grid_weight, double* max_value_out) {
  FORK_GUARD();
  if (!ctx || !counts_dev || !models || !x || !y) return fail(SCDE_EARG, "null argument");
  if (ngenes <= 0 || ncells <= 0 || ld < ngenes) return fail(SCDE_EARG, "bad dimensions");
  // density grid n <= 4096: k_prior_conv stages y and the 2n kernel values in LDS (96 KiB of 160)
  if (length_out < 1 || length_out > 2047) return fail(SCDE_EARG, "length.out must be in [1, 2047]");
  if (!(bw > 0)) return fail(SCDE_EARG, "bw must be positive");
  if (!max_value && !(max_quantile >= 0 && max_quantile <= 1)) return fail(SCDE_EARG, "'probs' outside [0,1]");
  if ((long long)ngenes * ncells > 0x7fffffffLL) return fail(SCDE_EARG, "ngenes x ncells too large");
  HCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const int N = ngenes, C = ncells, L = length_out;
  // per-cell constants: corr.b, corr.a, conc.b, conc.a, conc.a2 (model columns 3, 4, 0, 1, 11)
  std::vector<double> cellp((size_t)5 * C);
  const int mcol[5] = {3, 4, 0, 1, 11};
  for (int j = 0; j < 5; ++j)
    for (int c = 0; c < C; ++c)
      cellp[(size_t)j * C + c] = (j == 4 && !square_logit_conc) ? 0.0 : models[(size_t)mcol[j] * C + c];
  RCHK(upload(ctx, ctx->pr_cell, cellp.data(), sizeof(double) * cellp.size()));
  const int nb = prior_blocks(N, C, 2048);
  HCHK(ctx->pr_part.ensure(sizeof(double) * 6 * nb));
  HCHK(ctx->pr_occ.ensure(sizeof(int) * 256 * (size_t)prior_items(N, C)));
  HCHK(ctx->pr_stats.ensure(sizeof(double) * 4));
  const long long NC = (long long)N * C;
  const bool need_sort = !max_value && max_quantile < 1.0;
  if (need_sort) HCHK(ctx->pr_v.ensure(sizeof(double) * NC));
  hipEvent_t ev = ctx->mark_begin(SLOT_PRIOR_STATS);
  HCHK(launch_prior_stats(counts_dev, ld, N, C, ctx->pr_cell.as<double>(), square_logit_conc,
                          need_sort ? ctx->pr_v.as<double>() : nullptr, ctx->pr_occ.as<int>(),
                          ctx->pr_part.as<double>(), nb,
                          ctx->pr_stats.as<double>(), st));
  ctx->mark_end(SLOT_PRIOR_STATS, ev);
  double stats[4];
  HCHK(hipMemcpyAsync(stats, ctx->pr_stats.p, sizeof(stats), hipMemcpyDeviceToHost, st));
  RCHK(ctx->sync());
  const double wsum = stats[0];
  const long long nfin = (long long)stats[3];
  // totMass = sum(weights[is.finite(x)]) / sum(weights), 1 when every x is finite
  const double tot_mass = nfin == NC ? 1.0 : stats[1] / stats[0];
  double mv;
  if (max_value) {
    mv = *max_value;
  } else if (nfin == 0) {
    return fail(SCDE_EARG, "no finite expression magnitudes for quantile()");
  } else if (!need_sort) {
    mv = stats[2];  // quantile(x, 1) = max
  } else {
    // quantile(x[x < Inf], p, type = 7): the finite values sort first
    size_t wb = 0;
    HCHK(launch_sort_doubles(nullptr, nullptr, NC, nullptr, &wb, st));
    HCHK(ctx->pr_sortw.ensure(wb));
    HCHK(ctx->pr_sorted.ensure(sizeof(double) * NC));
    HCHK(launch_sort_doubles(ctx->pr_v.as<double>(), ctx->pr_sorted.as<double>(), NC, ctx->pr_sortw.p, &wb, st));
    const double index = 1 + (double)std::max<long long>(nfin - 1, 0) * max_quantile;
    const long long lo = (long long)std::floor(index), hi = (long long)std::ceil(index);
    double xl = 0, xh = 0;
    HCHK(hipMemcpyAsync(&xl, ctx->pr_sorted.as<double>() + (lo - 1), sizeof(double), hipMemcpyDeviceToHost, st));
    HCHK(hipMemcpyAsync(&xh, ctx->pr_sorted.as<double>() + (hi - 1), sizeof(double), hipMemcpyDeviceToHost, st));
    RCHK(ctx->sync());
    mv = xl;
    if (index > lo && xh != xl) {
      const double h = index - lo;
      mv = (1 - h) * xl + h * xh;
    }
  }
  if (!(mv > 0) || !std::isfinite(mv)) return fail(SCDE_EARG, "max.value must be positive and finite");
  const int n = prior_grid_n(L);
  HCHK(ctx->pr_hist.ensure(sizeof(unsigned long long) * (size_t)n));
  HCHK(ctx->pr_work.ensure(sizeof(double) * 3 * (size_t)n));
  HCHK(ctx->pr_out.ensure(sizeof(double) * 4 * (size_t)(L + 1)));
  ev = ctx->mark_begin(SLOT_PRIOR_BIN);
  HCHK(launch_prior_bin(counts_dev, ld, N, C, ctx->pr_cell.as<double>(), square_logit_conc, ctx->pr_occ.as<int>(),
                        wsum, mv, bw, L, ctx->pr_hist.as<unsigned long long>(), nb, st));
  ctx->mark_end(SLOT_PRIOR_BIN, ev);
  ev = ctx->mark_begin(SLOT_PRIOR_TAIL);
  HCHK(launch_prior_tail(tot_mass, mv, bw, L, pseudo_count / (double)N, ctx->pr_hist.as<unsigned long long>(),
                         ctx->pr_work.as<double>(), ctx->pr_out.as<double>(), st));
  ctx->mark_end(SLOT_PRIOR_TAIL, ev);
  const size_t m = (size_t)L + 1;
  double* outs[4] = {x, y, lp, grid_weight};
  for (int k = 0; k < 4; ++k)
    if (outs[k])
      HCHK(hipMemcpyAsync(outs[k], ctx->pr_out.as<double>() + k * m, sizeof(double) * m, hipMemcpyDeviceToHost, st));
  if (max_value_out) *max_value_out = mv;
  return ctx->sync();
}

int scde_bh_cz_dev(scde_ctx* ctx, const double* z_dev, int64_t n, double* cz_dev) {
  FORK_GUARD();
  if (!ctx || n < 0 || (n > 0 && (!z_dev || !cz_dev))) return fail(SCDE_EARG, "bad arguments");
  if (n > 0x7fffffff) return fail(SCDE_EARG, "n too large");
  if (n == 0) return SCDE_OK;
  HCHK(hipSetDevice(ctx->device));
  size_t wb = 0;
  HCHK(launch_bh_cz(nullptr, (int)n, nullptr, nullptr, &wb, ctx->stream));
  HCHK(ctx->bhw.ensure(wb));
  HCHK(launch_bh_cz(z_dev, (int)n, cz_dev, ctx->bhw.p, &wb, ctx->stream));
  return ctx->sync();
}

int scde_bh_cz(const double* z, int64_t n, double* cz) {
  if (n < 0 || (n > 0 && (!z || !cz))) return fail(SCDE_EARG, "bad arguments");
  // p.adjust(p, "BH"): i <- n:1; o <- order(p, decreasing = TRUE); pmin(1, cummin(n/i * p[o]))[ro]
  // NA (NaN) p-values are dropped from the adjustment and stay NA, as in R.
  std::vector<double> p(n);
  std::vector<int64_t> o;
  o.reserve(n);
  for (int64_t i = 0; i < n; ++i) {
    p[i] = pnorm_upper(std::fabs(z[i]));
    if (!std::isnan(p[i])) o.push_back(i);
  }
  const int64_t lp = (int64_t)o.size();
  if (lp <= 1) {  // `if (n <= 1) return(p0)`: nothing to adjust
    for (int64_t i = 0; i < n; ++i) {
      const double s = (z[i] > 0) ? 1.0 : (z[i] < 0 ? -1.0 : (std::isnan(z[i]) ? NAN : 0.0));
      cz[i] = s * qnorm_host(p[i], false);
    }
    return SCDE_OK;
  }
  std::stable_sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return p[a] > p[b]; });
  std::vector<double> adj(n, NAN);
  double cm = INFINITY;
  for (int64_t r = 0; r < lp; ++r) {
    const double i = (double)(lp - r);
    const double v = ((double)lp / i) * p[o[r]];
    if (v < cm) cm = v;
    adj[o[r]] = cm < 1 ? cm : 1;
  }
  for (int64_t i = 0; i < n; ++i) {
    const double s = (z[i] > 0) ? 1.0 : (z[i] < 0 ? -1.0 : (std::isnan(z[i]) ? NAN : 0.0));
    cz[i] = s * qnorm_host(adj[i], false);
  }
  return SCDE_OK;
}


// ------------------------------------------------------------------ weighted PCA
// R's RNG (src/main/RNG.c) for the host mirror of the R glue: set.seed scrambling,
// Mersenne-Twister unif_rand (with fixup), R >= 3.6 rejection sample().
int scde_r_set_seed(uint32_t seed, uint32_t* state) {
  if (!state) return fail(SCDE_EARG, "null state");
  for (int j = 0; j < 50; ++j) seed = 69069u * seed + 1u;
  for (int j = 0; j < 625; ++j) {
    seed = 69069u * seed + 1u;
    state[j] = seed;
  }
  state[0] = 624;
  return SCDE_OK;
}

static double r_mt_genrand(uint32_t* st) {
  static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
  uint32_t* mt = st + 1;
  int mti = (int)st[0];
  uint32_t y;
  if (mti >= 624) {
    int kk;
    for (kk = 0; kk < 624 - 397; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < 623; ++kk) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk - 227] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
    mti = 0;
  }
  y = mt[mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  st[0] = (uint32_t)mti;
  return (double)y * 2.3283064365386963e-10;
}

static double r_unif_rand(uint32_t* st) {
  const double i2_32m1 = 2.328306437080797e-10;
  const double x = r_mt_genrand(st);
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

int scde_r_unif_rand(uint32_t* state, int64_t n, double* out) {
  if (!state || (n > 0 && !out)) return fail(SCDE_EARG, "null argument");
  for (int64_t i = 0; i < n; ++i) out[i] = r_unif_rand(state);
  return SCDE_OK;
}

int scde_r_sample(uint32_t* state, int n, int k, int* out) {
  if (!state || (k > 0 && !out)) return fail(SCDE_EARG, "null argument");
  if (k > n || k < 0) return fail(SCDE_EARG, "cannot take a sample larger than the population");
  std::vector<int> x(std::max(n, 1));
  for (int i = 0; i < n; ++i) x[i] = i;
  for (int i = 0; i < k; ++i) {
    double dv = 0;
    const double dn = (double)n;
    if (dn > 0) {
      const int bits = (int)std::ceil(std::log2(dn));
      do {
        int64_t v = 0;
        for (int b = 0; b <= bits; b += 16) v = 65536 * v + (int)std::floor(r_unif_rand(state) * 65536);
        dv = (double)(v & ((((int64_t)1) << bits) - 1));
      } while (dn <= dv);
    }
    const int j = (int)dv;
    out[i] = x[j] + 1;
    x[j] = x[--n];
  }
  return SCDE_OK;
}

// set_random_matrices (src/bwpca.cpp:41-57) over the platform rand() (srand(seed) first):
// ind = 0..n-1 per shuffle; per column libstdc++ std::random_shuffle (j = rand() % (i+1)).
int scde_shuffle_perms(unsigned int seed, int nshuffles, int d, int n, int* perms) {
  if (nshuffles > 0 && d > 0 && n > 0 && !perms) return fail(SCDE_EARG, "null perms");
  PlatformRand rng(seed, g_rand_kind);
  std::vector<int> ind(std::max(n, 1));
  for (int s = 0; s < nshuffles; ++s) {
    for (int i = 0; i < n; ++i) ind[i] = i;
    for (int c = 0; c < d; ++c) {
      for (int i = 1; i < n; ++i) {
        const int j = rng.next() % (i + 1);
        if (i != j) std::swap(ind[i], ind[j]);
      }
      std::memcpy(perms + ((int64_t)s * d + c) * n, ind.data(), sizeof(int) * n);
    }
  }
  return SCDE_OK;
}

}  // extern "C"

namespace {
// smoothing coefficients (src/bwpca.cpp:86-100): A (2np+1) x 4, A[:, j] = x^j,
// smoothc = A solve(A^T A, e_0); solved by partial-pivot LU like the K x K systems.
std::vector<double> wpca_smooth_coef(int smooth) {
  const int np = smooth / 2, L = 2 * np + 1;
  std::vector<double> X((size_t)L * 4), sc(L);
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < L; ++i) X[i + j * L] = std::pow((double)(i - np), (double)j);
  double A[16], b[4] = {1, 0, 0, 0};
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 4; ++k) {
      double s = 0;
      for (int i = 0; i < L; ++i) s += X[i + k * L] * X[i + j * L];
      A[k + j * 4] = s;
    }
  int piv[4];
  for (int j = 0; j < 4; ++j) {
    int p = j;
    for (int i = j + 1; i < 4; ++i)
      if (std::fabs(A[i + j * 4]) > std::fabs(A[p + j * 4])) p = i;
    piv[j] = p;
    if (p != j)
      for (int l = 0; l < 4; ++l) std::swap(A[j + l * 4], A[p + l * 4]);
    const double r = 1.0 / A[j + j * 4];
    for (int i = j + 1; i < 4; ++i) A[i + j * 4] *= r;
    for (int l = j + 1; l < 4; ++l)
      for (int i = j + 1; i < 4; ++i) A[i + l * 4] -= A[i + j * 4] * A[j + l * 4];
  }
  for (int j = 0; j < 4; ++j)
    if (piv[j] != j) std::swap(b[j], b[piv[j]]);
  for (int l = 0; l < 4; ++l)
    for (int i = l + 1; i < 4; ++i) b[i] -= b[l] * A[i + l * 4];
  for (int l = 3; l >= 0; --l) {
    b[l] /= A[l + l * 4];
    for (int i = 0; i < l; ++i) b[i] -= b[l] * A[i + l * 4];
  }
  for (int i = 0; i < L; ++i) {
    double s = 0;
    for (int j = 0; j < 4; ++j) s += X[i + j * L] * b[j];
    sc[i] = s;
  }
  return sc;
}

template <class T>
hipError_t upload(Buf& b, const T* src, size_t n, hipStream_t st) {
  hipError_t e = b.ensure(sizeof(T) * std::max<size_t>(n, 1));
  if (e != hipSuccess || n == 0) return e;
  return hipMemcpyAsync(b.p, src, sizeof(T) * n, hipMemcpyHostToDevice, st);
}
}  // namespace

extern "C" {

int scde_bwpca_batch_dev(scde_ctx* ctx, const double* M_dev, const double* W_dev, int64_t ld, int ncells,
                         int64_t mcols, int nprob, const int* d, const int* npcs, const int* nstarts,
                         const int64_t* col_off, const int* cols, int64_t ncols, const int64_t* perm_off,
                         const int* perms, int64_t nperms, const int64_t* start_off, const double* starts,
                         int64_t nstart_vals, int smooth, double em_tol, int em_maxiter, double* rotation,
                         double* scores, double* scoreweights, double* colmeans, double* stats, int* iterations) {
  FORK_GUARD();
  if (!ctx || !M_dev || !W_dev) return fail(SCDE_EARG, "null argument");
  if (nprob < 0 || ncells <= 0 || ld < ncells || mcols <= 0) return fail(SCDE_EARG, "bad dimensions");
  if (nprob == 0) return SCDE_OK;
  if (!d || !npcs || !nstarts || !col_off || !cols || !start_off || !starts || !rotation || !scores || !stats)
    return fail(SCDE_EARG, "null problem array");
  const int n = ncells;
  for (int64_t i = 0; i < ncols; ++i)
    if (cols[i] < 0 || cols[i] >= mcols) return fail(SCDE_EARG, "column index %d out of range", cols[i]);
  for (int64_t i = 0; i < nperms; ++i)
    if (perms[i] < 0 || perms[i] >= n) return fail(SCDE_EARG, "permutation index out of range");
  std::vector<WpcaProb> P(nprob);
  int64_t o_rot = 0, o_sc = 0, o_var = 0;
  for (int p = 0; p < nprob; ++p) {
    if (d[p] <= 0) return fail(SCDE_EARG, "problem %d: no columns", p);
    if (nstarts[p] <= 0) return fail(SCDE_EARG, "problem %d: nstarts must be positive", p);
    const int K = std::min(npcs[p], d[p]);
    if (K < 1 || K > wpca_max_k()) return fail(SCDE_EARG, "problem %d: npcs must be in [1, %d]", p, wpca_max_k());
    if (col_off[p] < 0 || col_off[p] + d[p] > ncols) return fail(SCDE_EARG, "problem %d: cols out of range", p);
    if (perm_off && perm_off[p] >= 0 && perm_off[p] + (int64_t)d[p] * n > nperms)
      return fail(SCDE_EARG, "problem %d: perms out of range", p);
    if (start_off[p] < 0 || start_off[p] + (int64_t)nstarts[p] * d[p] * K > nstart_vals)
      return fail(SCDE_EARG, "problem %d: starts out of range", p);
    WpcaProb& q = P[p];
    q.d = d[p];
    q.K = K;
    q.nstarts = nstarts[p];
    q.pad = 0;
    q.col_off = col_off[p];
    q.perm_off = perm_off ? perm_off[p] : -1;
    q.start_off = start_off[p];
    q.out_rot = o_rot;
    q.out_sc = o_sc;
    q.out_var = o_var;
    o_rot += (int64_t)d[p] * K;
    o_sc += (int64_t)n * K;
    o_var += K + 2;
  }
  const int64_t tot_sc = o_sc;
  for (auto& q : P) {  // output layout: [rot | scores | scoreweights | colmeans | stats]
    q.out_sc += o_rot;
    q.out_pcw = q.out_sc + tot_sc;
    q.out_cm = q.out_sc + 2 * tot_sc;
    q.out_var += o_rot + 3 * tot_sc;
  }
  const int64_t out_total = o_rot + 3 * tot_sc + o_var;
  const int L = smooth > 0 ? 2 * (smooth / 2) + 1 : 0;
  std::vector<double> sc = L > 0 ? wpca_smooth_coef(smooth) : std::vector<double>(1, 0.0);
  constexpr int kLdsCap = 160 * 1024 - 2048;
  HCHK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  HCHK(upload(ctx->wp_cols, cols, (size_t)ncols, st));
  HCHK(upload(ctx->wp_perms, perms, (size_t)(perms ? nperms : 0), st));
  HCHK(upload(ctx->wp_starts, starts, (size_t)nstart_vals, st));
  HCHK(upload(ctx->wp_smooth, sc.data(), sc.size(), st));
  HCHK(ctx->wp_out.ensure(sizeof(double) * out_total));
  // problems grouped by K; within a group by work (d x nstarts) descending, in chunks
  // whose scratch stays under a budget
  std::vector<int> order(nprob);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    if (P[a].K != P[b].K) return P[a].K < P[b].K;
    return (int64_t)P[a].d * P[a].nstarts > (int64_t)P[b].d * P[b].nstarts;
  });
  const int64_t kScratchBudget = (int64_t)1 << 28;  // doubles (2 GiB)
  std::vector<int64_t> iters_all;
  std::vector<double> stat_h;
  if (iterations) {
    int64_t tot = 0;
    for (auto& q : P) tot += q.nstarts;
    iters_all.assign(tot, 0);
  }
  std::vector<int64_t> it_base(nprob, 0);
  {
    int64_t b = 0;
    for (int p = 0; p < nprob; ++p) {
      it_base[p] = b;
      b += P[p].nstarts;
    }
  }
  size_t pos = 0;
  while (pos < order.size()) {
    const int K = P[order[pos]].K;
    const int NM = K + K * (K + 1) / 2;
    // chunk: same K, scratch within budget
    size_t end = pos;
    int dmax = 0;
    int64_t need = 0;
    while (end < order.size() && P[order[end]].K == K) {
      const WpcaProb& q = P[order[end]];
      const int dm = std::max(dmax, q.d);
      const bool cl = (size_t)(dm + n) * K * sizeof(double) <= (size_t)kLdsCap;
      const int64_t per = (int64_t)q.nstarts * ((int64_t)q.d * K + 2LL * n * K + (cl ? 0 : (int64_t)n * K) +
                                                (int64_t)q.d * (NM + 1));
      if (end > pos && need + per > kScratchBudget) break;
      need += per;
      dmax = dm;
      ++end;
    }
    const bool cl = (size_t)(dmax + n) * K * sizeof(double) <= (size_t)kLdsCap;
    int64_t so = 0, stt = 0;
    for (size_t i = pos; i < end; ++i) {
      WpcaProb& q = P[order[i]];
      q.sE_off = so;
      so += (int64_t)q.nstarts * q.d * K;
      q.sC_off = so;
      so += (int64_t)q.nstarts * 2 * n * K;
      q.sW_off = so;
      if (!cl) so += (int64_t)q.nstarts * n * K;
      q.mom_off = so;
      so += (int64_t)q.nstarts * q.d * (NM + 1);
      q.stat_off = stt;
      stt += q.nstarts;
    }
    HCHK(ctx->wp_scratch.ensure(sizeof(double) * std::max<int64_t>(so, 1)));
    HCHK(ctx->wp_stat.ensure(sizeof(double) * 4 * std::max<int64_t>(stt, 1)));
    // block list: problems in groups of 8 (one per XCD under round-robin dispatch);
    // the starts of a problem sit 8 blocks apart, on the same XCD, sharing its columns in L2
    std::vector<int2> blocks;
    std::vector<WpcaProb> chunk;
    std::vector<int> kidx;
    for (size_t i = pos; i < end; ++i) {
      chunk.push_back(P[order[i]]);
      kidx.push_back((int)(i - pos));
    }
    // npcs = 1 without smoothing: one workgroup per group of wpca_ms_group() starts
    const bool ms = K == 1 && L == 0 && wpca_ms_ok(n, dmax) && ctx->opt_wpca_ms;
    const int sstep = ms ? wpca_ms_group() : 1;
    for (size_t g0 = 0; g0 < chunk.size(); g0 += 8) {
      const size_t g1 = std::min(chunk.size(), g0 + 8);
      int smax = 0;
      for (size_t i = g0; i < g1; ++i) smax = std::max(smax, chunk[i].nstarts);
      for (int s = 0; s < smax; s += sstep)
        for (size_t x = 0; x < 8; ++x) {
          const size_t i = g0 + x;
          if (i < g1 && s < chunk[i].nstarts) blocks.push_back(make_int2((int)i, s));
          else blocks.push_back(make_int2(-1, 0));  // keeps the 8-block stride
        }
    }
    // drop trailing padding
    while (!blocks.empty() && blocks.back().x < 0) blocks.pop_back();
    HCHK(upload(ctx->wp_probs, chunk.data(), chunk.size(), st));
    HCHK(upload(ctx->wp_blocks, blocks.data(), blocks.size(), st));
    HCHK(upload(ctx->wp_kidx, kidx.data(), kidx.size(), st));
    WpcaLaunch a;
    a.M = M_dev;
    a.W = W_dev;
    a.ld = ld;
    a.n = n;
    a.dmax = dmax;
    a.probs = ctx->wp_probs.as<WpcaProb>();
    a.blocks = ctx->wp_blocks.as<int2>();
    a.cols = ctx->wp_cols.as<int>();
    a.perms = ctx->wp_perms.as<int>();
    a.starts = ctx->wp_starts.as<double>();
    a.maxiter = em_maxiter;
    a.tol = em_tol;
    a.smoothc = ctx->wp_smooth.as<double>();
    a.L = L;
    a.scratch = ctx->wp_scratch.as<double>();
    a.stat = ctx->wp_stat.as<double>();
    a.out = ctx->wp_out.as<double>();
    a.lds_cap = kLdsCap;
    hipEvent_t ev = ctx->mark_begin(SLOT_WPCA_EM);
    if (!blocks.empty()) {
      if (ms) HCHK(launch_wpca_ms(a, (int)blocks.size(), st));
      else HCHK(launch_wpca_em(K, a, (int)blocks.size(), st));
    }
    ctx->mark_end(SLOT_WPCA_EM, ev);
    ev = ctx->mark_begin(SLOT_WPCA_FINAL);
    HCHK(launch_wpca_final(K, a, ctx->wp_kidx.as<int>(), (int)chunk.size(), st));
    ctx->mark_end(SLOT_WPCA_FINAL, ev);
    if (iterations) {
      stat_h.resize((size_t)4 * stt);
      HCHK(hipMemcpyAsync(stat_h.data(), a.stat, sizeof(double) * 4 * stt, hipMemcpyDeviceToHost, st));
      RCHK(ctx->sync());
      for (size_t i = 0; i < chunk.size(); ++i)
        for (int s = 0; s < chunk[i].nstarts; ++s)
          iters_all[it_base[order[pos + i]] + s] = (int64_t)stat_h[(size_t)4 * (chunk[i].stat_off + s) + 2];
    }
    pos = end;
  }
  std::vector<double> out_h(out_total);
  HCHK(hipMemcpyAsync(out_h.data(), ctx->wp_out.p, sizeof(double) * out_total, hipMemcpyDeviceToHost, st));
  RCHK(ctx->sync());
  std::memcpy(rotation, out_h.data(), sizeof(double) * o_rot);
  std::memcpy(scores, out_h.data() + o_rot, sizeof(double) * tot_sc);
  if (scoreweights) std::memcpy(scoreweights, out_h.data() + o_rot + tot_sc, sizeof(double) * tot_sc);
  if (colmeans) std::memcpy(colmeans, out_h.data() + o_rot + 2 * tot_sc, sizeof(double) * tot_sc);
  std::memcpy(stats, out_h.data() + o_rot + 3 * tot_sc, sizeof(double) * o_var);
  if (iterations)
    for (size_t i = 0; i < iters_all.size(); ++i) iterations[i] = (int)iters_all[i];
  return SCDE_OK;
}

// .Call("baileyWPCA", ...) (src/bwpca.cpp:59; bwpca.h:8) on host buffers.
int scde_baileyWPCA(const double* mat, const double* matw, int n, int d, int npcs, int nstarts, int smooth,
                    double em_tol, int em_maxiter, const double* starts, int nshuffles, const int* perms,
                    double* rotation, double* scores, double* scoreweights, double* var, double* totvar,
                    double* randvar) {
  FORK_GUARD();
  if (!mat || !matw || !starts || !rotation || !scores || !var || !totvar) return fail(SCDE_EARG, "null argument");
  if (n <= 0 || d <= 0) return fail(SCDE_EARG, "bad dimensions");
  if (nshuffles < 0 || (nshuffles > 0 && (!perms || !randvar))) return fail(SCDE_EARG, "bad shuffles");
  if (nstarts <= 0) return fail(SCDE_EARG, "nstarts must be positive");
  const int K = std::min(npcs, d);
  if (K < 1) return fail(SCDE_EARG, "npcs must be positive");
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  const size_t nd = (size_t)n * d;
  HCHK(upload(cx->wp_M, mat, nd, cx->stream));
  HCHK(upload(cx->wp_W, matw, nd, cx->stream));
  const int np = 1 + nshuffles;
  std::vector<int> dv(np, d), kv(np, npcs), sv(np, nstarts), cols(d);
  std::vector<int64_t> co(np, 0), po(np, -1), so(np);
  std::iota(cols.begin(), cols.end(), 0);
  for (int q = 0; q < np; ++q) {
    so[q] = (int64_t)q * nstarts * d * K;
    if (q > 0) po[q] = (int64_t)(q - 1) * d * n;
  }
  std::vector<double> rot((size_t)np * d * K), sco((size_t)np * n * K), pcw((size_t)np * n * K),
      stats((size_t)np * (K + 2));
  RCHK(scde_bwpca_batch_dev(cx, cx->wp_M.as<double>(), cx->wp_W.as<double>(), n, n, d, np, dv.data(), kv.data(),
                            sv.data(), co.data(), cols.data(), d, po.data(), perms,
                            nshuffles > 0 ? (int64_t)nshuffles * d * n : 0, so.data(), starts,
                            (int64_t)np * nstarts * d * K, smooth, em_tol, em_maxiter, rot.data(), sco.data(),
                            pcw.data(), nullptr, stats.data(), nullptr));
  std::memcpy(rotation, rot.data(), sizeof(double) * d * K);
  std::memcpy(scores, sco.data(), sizeof(double) * n * K);
  if (scoreweights) std::memcpy(scoreweights, pcw.data(), sizeof(double) * n * K);
  std::memcpy(var, stats.data(), sizeof(double) * K);
  *totvar = stats[K];
  for (int s = 0; s < nshuffles; ++s) randvar[s] = *totvar - stats[(size_t)(1 + s) * (K + 2) + K + 1];
  return SCDE_OK;
}

// ------------------------------------------------------------------ PAGODA helpers
// .Call("winsorizeMatrix", Mat, Trim) (src/pagoda.cpp:6-31; pagoda.h:5).  mat: nrow x ncol.
int scde_winsorizeMatrix(const double* mat, int nrow, int ncol, double trim, double* out) {
  FORK_GUARD();
  if (!mat || !out) return fail(SCDE_EARG, "null argument");
  if (nrow < 0 || ncol < 0) return fail(SCDE_EARG, "bad dimensions");
  const size_t nel = (size_t)nrow * ncol;
  const int ntr = (int)std::round(ncol * trim);
  if (nel == 0 || ntr == 0) {
    if (nel) std::memcpy(out, mat, sizeof(double) * nel);
    return SCDE_OK;
  }
  if (ntr < 0 || ntr > ncol - 1)  // the reference indexes sorted[ntr] and sorted[ncol - ntr - 1]
    return fail(SCDE_EARG, "winsorizeMatrix: trim %g out of range for %d columns", trim, ncol);
  int NP = 1;
  while (NP < ncol) NP <<= 1;
  if (NP > 8192 && ntr > 32) return fail(SCDE_EARG, "winsorizeMatrix: ncol > 8192 needs round(ncol * trim) <= 32");
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  HCHK(upload(cx->pg_a, mat, nel, cx->stream));
  HCHK(cx->pg_b.ensure(sizeof(double) * nel));
  HCHK(launch_winsorize(cx->pg_a.as<double>(), nrow, ncol, ntr, cx->pg_b.as<double>(), cx->stream));
  HCHK(hipMemcpyAsync(out, cx->pg_b.p, sizeof(double) * nel, hipMemcpyDeviceToHost, cx->stream));
  return cx->sync();
}

// .Call("matWCorr", Mat, Matw) (src/pagoda.cpp:41-65; pagoda.h:6).  mat, matw: nrow x ncol;
// out: ncol x ncol (identity diagonal, c(j, i) for j > i, upper triangle 0).
int scde_matWCorr(const double* mat, const double* matw, int nrow, int ncol, double* out) {
  FORK_GUARD();
  if (!mat || !matw || !out) return fail(SCDE_EARG, "null argument");
  if (nrow < 0 || ncol < 0) return fail(SCDE_EARG, "bad dimensions");
  if (ncol == 0) return SCDE_OK;
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  const size_t nel = (size_t)nrow * ncol, nout = (size_t)ncol * ncol;
  HCHK(upload(cx->pg_a, mat, nel, cx->stream));
  HCHK(upload(cx->pg_b, matw, nel, cx->stream));
  HCHK(cx->pg_c.ensure(sizeof(double) * nout));
  HCHK(launch_matwcorr(cx->pg_a.as<double>(), cx->pg_b.as<double>(), nrow, ncol, cx->pg_c.as<double>(),
                       cx->stream));
  HCHK(hipMemcpyAsync(out, cx->pg_c.p, sizeof(double) * nout, hipMemcpyDeviceToHost, cx->stream));
  return cx->sync();
}

// .Call("matCorr", X, Y) = arma::cor(x, y) (src/pagoda.cpp:33-38; pagoda.h:8).  x: nrow x nx,
// y: nrow x ny; out: nx x ny.
int scde_matCorr(const double* x, int nrow, int nx, const double* y, int ny, double* out) {
  FORK_GUARD();
  if (!x || !y || !out) return fail(SCDE_EARG, "null argument");
  if (nrow < 0 || nx < 0 || ny < 0) return fail(SCDE_EARG, "bad dimensions");
  if ((size_t)nx * ny == 0) return SCDE_OK;
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  HCHK(upload(cx->pg_a, x, (size_t)nrow * nx, cx->stream));
  HCHK(upload(cx->pg_b, y, (size_t)nrow * ny, cx->stream));
  HCHK(cx->pg_c.ensure(sizeof(double) * (size_t)nx * ny));
  HCHK(cx->pg_d.ensure(sizeof(double) * 2 * ((size_t)nx + ny)));
  HCHK(launch_matcorr(cx->pg_a.as<double>(), nrow, nx, cx->pg_b.as<double>(), ny, cx->pg_d.as<double>(),
                      cx->pg_c.as<double>(), cx->stream));
  HCHK(hipMemcpyAsync(out, cx->pg_c.p, sizeof(double) * (size_t)nx * ny, hipMemcpyDeviceToHost, cx->stream));
  return cx->sync();
}

// .Call("plSemicompleteCor2", Pl) (src/pagoda.cpp:67-117; pagoda.h:7).  List element p:
// gene indices idx[off[p] .. off[p+1]) (increasing), values val[...].  r: np x np
// correlations over the shared genes (1 on the diagonal); n: np x np union sizes (0 on it).
int scde_plSemicompleteCor2(int np, const int64_t* off, const int* idx, const double* val, double* r, int* n) {
  FORK_GUARD();
  if (np < 0 || (np > 0 && (!off || !r || !n))) return fail(SCDE_EARG, "null argument");
  if (np == 0) return SCDE_OK;
  const int64_t tot = off[np];
  if (off[0] != 0 || tot < 0) return fail(SCDE_EARG, "bad offsets");
  for (int p = 0; p < np; ++p) {
    if (off[p + 1] < off[p]) return fail(SCDE_EARG, "bad offsets");
    for (int64_t e = off[p] + 1; e < off[p + 1]; ++e)
      if (idx[e] <= idx[e - 1]) return fail(SCDE_EARG, "list %d: gene indices must increase", p);
  }
  scde_ctx* cx = nullptr;
  RCHK(default_ctx(&cx));
  HCHK(hipSetDevice(cx->device));
  std::vector<long long> offl(off, off + np + 1);
  HCHK(upload(cx->pg_a, offl.data(), offl.size(), cx->stream));
  HCHK(upload(cx->pg_b, idx, (size_t)tot, cx->stream));
  HCHK(upload(cx->pg_c, val, (size_t)tot, cx->stream));
  const size_t nn = (size_t)np * np;
  HCHK(cx->pg_d.ensure(sizeof(double) * nn));
  HCHK(cx->pg_e.ensure(sizeof(int) * nn));
  HCHK(launch_plcor(np, cx->pg_a.as<long long>(), cx->pg_b.as<int>(), cx->pg_c.as<double>(), cx->pg_d.as<double>(),
                    cx->pg_e.as<int>(), cx->stream));
  HCHK(hipMemcpyAsync(r, cx->pg_d.p, sizeof(double) * nn, hipMemcpyDeviceToHost, cx->stream));
  HCHK(hipMemcpyAsync(n, cx->pg_e.p, sizeof(int) * nn, hipMemcpyDeviceToHost, cx->stream));
  return cx->sync();
}
}  // extern "C"

namespace {

// R pnorm upper tail (Cody, R nmath pnorm.c pnorm_both), x >= 0 path used by BH
double pnorm_upper(double x) {
  static const double a[5] = {2.2352520354606839287, 161.02823106855587881, 1067.6894854603709582,
                              18154.981253343561249, 0.065682337918207449113};
  static const double b[4] = {47.20258190468824187, 976.09855173777669322, 10260.932208618978205,
                              45507.789335026729956};
  static const double c[9] = {0.39894151208813466764, 8.8831497943883759412, 93.506656132177855979,
                              597.27027639480026226,  2494.5375852903726711, 6848.1904505362823326,
                              11602.651437647350124,  9842.7148383839780218, 1.0765576773720192317e-8};
  static const double d[8] = {22.266688044328115691, 235.38790178262499861, 1519.377599407554805,
                              6485.558298266760755,  18615.571640885098091, 34900.952721145977266,
                              38912.003286093271411, 19685.429676859990727};
  static const double pp[6] = {0.21589853405795699,     0.1274011611602473639, 0.022235277870649807,
                               0.001421619193227893466, 2.9112874951168792e-5, 0.02307344176494017303};
  static const double q[5] = {1.28426009614491121, 0.468238212480865118, 0.0659881378689285515,
                              0.00378239633202758244, 7.29751555083966205e-5};
  const double M_1_SQRT_2PI = 0.398942280401432677939946059934, M_SQRT_32 = 5.656854249492380195206754896838;
  if (std::isnan(x)) return x;
  const double y = std::fabs(x);
  double xnum, xden, temp, xsq, del, cum, ccum;
  if (y <= 0.67448975) {
    if (y > DBL_EPSILON * 0.5) {
      xsq = x * x;
      xnum = a[4] * xsq;
      xden = xsq;
      for (int i = 0; i < 3; ++i) {
        xnum = (xnum + a[i]) * xsq;
        xden = (xden + b[i]) * xsq;
      }
    } else {
      xnum = xden = 0.0;
    }
    temp = x * (xnum + a[3]) / (xden + b[3]);
    cum = 0.5 + temp;
    ccum = 0.5 - temp;
  } else if (y <= M_SQRT_32) {
    xnum = c[8] * y;
    xden = y;
    for (int i = 0; i < 7; ++i) {
      xnum = (xnum + c[i]) * y;
      xden = (xden + d[i]) * y;
    }
    temp = (xnum + c[7]) / (xden + d[7]);
    xsq = std::trunc(y * 16) / 16;
    del = (y - xsq) * (y + xsq);
    cum = std::exp(-xsq * xsq * 0.5) * std::exp(-del * 0.5) * temp;
    ccum = 1.0 - cum;
    if (x > 0.) std::swap(cum, ccum);
  } else if ((-37.5193 < x && x < 8.2924) || (-8.2924 < x && x < 37.5193)) {
    xsq = 1.0 / (x * x);
    xnum = pp[5] * xsq;
    xden = xsq;
    for (int i = 0; i < 4; ++i) {
      xnum = (xnum + pp[i]) * xsq;
      xden = (xden + q[i]) * xsq;
    }
    temp = xsq * (xnum + pp[4]) / (xden + q[4]);
    temp = (M_1_SQRT_2PI - temp) / y;
    xsq = std::trunc(x * 16) / 16;
    del = (x - xsq) * (x + xsq);
    cum = std::exp(-xsq * xsq * 0.5) * std::exp(-del * 0.5) * temp;
    ccum = 1.0 - cum;
    if (x > 0.) std::swap(cum, ccum);
  } else {
    if (x > 0) {
      cum = 1.;
      ccum = 0.;
    } else {
      cum = 0.;
      ccum = 1.;
    }
  }
  return ccum;
}

double qnorm_host(double p, bool lower_tail) {
  if (std::isnan(p)) return p;
  if (p < 0 || p > 1) return NAN;
  if (p == 0) return lower_tail ? -INFINITY : INFINITY;
  if (p == 1) return lower_tail ? INFINITY : -INFINITY;
  const double p_ = lower_tail ? p : (0.5 - p + 0.5);
  const double q = p_ - 0.5;
  double r, val;
  if (std::fabs(q) <= .425) {
    r = .180625 - q * q;
    return q *
           (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
             133.14166789178437745) * r + 3.387132872796366608) /
           (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.);
  }
  if (q < 0)
    r = lower_tail ? p : (0.5 - p + 0.5);
  else
    r = lower_tail ? (0.5 - p + 0.5) : p;
  r = std::sqrt(-std::log(r));
  if (r <= 5.) {
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r + .24178072517745061177) * r +
                1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
             4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + .0151986665636164571966) * r +
                .14810397642748007459) * r + .68976733498510000455) * r + 1.6763848301838038494) * r +
             2.05319162663775882187) * r + 1.);
  } else {
    r += -5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + .0012426609473880784386) * r +
                .026532189526576123093) * r + .29656057182850489123) * r + 1.7848265399172913358) * r +
             5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
                7.868691311456132591e-4) * r + .0148753612908506148525) * r + .13692988092273580531) * r +
             .59983220655588793769) * r + 1.);
  }
  if (q < 0.0) val = -val;
  return val;
}

}  // namespace
