// bootq.hip -- the bootstrap joint posterior (logBootPosterior phase B,
// src/jpmatLogBoot.cpp:224-273; batch draws 473-496) in exact fixed-point arithmetic on the
// int8 matrix cores.
//
// The reference adds, per boot b and grid point k, the log-posterior column of every drawn
// cell: row_b[k] = sum_c W[b,c] T[c, uci(g,c)][k] (W = draw multiplicities), then takes a
// softmax over k and averages over boots.  Here every table value is a fixed-point integer
// q = round(T * 2^36) (T <= 0; below -2^18 it saturates), the baseline-delta columns
// D = q[c,u] - q[c,0] are exact integers (|D| < 2^55), stored as seven balanced base-256
// digits, and with W <= 127 a row is
//     row_b[k] = Z_b[k] + sum_l 256^l sum_e W[b,e] digit_l(D_e[k])
// -- seven int8 x int8 -> int32 products per (boot, point), exact in any summation order.
// v_mfma_i32_16x16x64_i8 does 16 boots x 16 grid points x 64 entries per instruction.
// The only rounding is the quantisation: |error| <= 2^-37 per table value, <= C 2^-37 per
// row (1.5e-8 at C = 2000), far under SURVEY §8(d)'s 1e-6 relative bar on jp.
//
// Saturation: a drawn cell whose value saturates makes row_b[k] <= -2^18 both in the
// integers and in the reference's doubles, so those points sit far below the e^-50
// softmax cut whenever the boot's maximum is above -2^18 + 51; boots whose maximum is not
// (and any NaN in a table) flag the gene, which the exact FP64 path (k_boot_exact, on T
// tables built only then) recomputes in the reference's cell order.
//
// Work skipping: per 16-point tile t and column, the tables kernel stores the column's
// maximum rounded up to 2^-8 (UQ); UB_bt = ZU_bt + sum_e W[b,e] UQ_e,t >= every row value
// in the tile, again on the int8 matrix cores (4 digits).  A tile is computed when some boot
// has UB_bt >= max_t' UB_bt' - 50 - slack; after the exact row maxima M_b are known every
// skipped tile must satisfy UB_bt < M_b - 51 for every live boot, else it is computed too
// (in the same block, before any softmax term is formed).  Skipped tiles therefore only
// ever hold terms the e^-50 cut zeroes, and because the per-boot sums and the jp rows add
// tile partials in tile order (absent tiles contribute exact zeros) the output is bit for
// bit the one computed with every tile.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdint>

#include "device_math.h"
#include "kernels.h"

namespace scde {


constexpr int kQWaves = 8;        // waves per k_bootq block (one gene)
constexpr int kQSlab = 32;        // boots per slab (two 16-boot MFMA tiles)
constexpr int kQSlotsPerWave = 4; // computed tiles whose rows a wave holds: 8 x 4 >= 28 tiles
constexpr int kQMaxTiles = 28;    // G <= 448

constexpr int kZChunk = 64;  // cells per baseline-sum block

__device__ __forceinline__ int sbyte(unsigned long long p, int l) { return (int)(signed char)(p >> (8 * l)); }

// sum_l d_l 256^l 2^-36 from seven digit sums (|d_l| < 2^22): pairs exact in int32, then
// FP64 steps exact up to 2^53
__device__ __forceinline__ double qcombine(int d0, int d1, int d2, int d3, int d4, int d5, int d6) {
  const int p0 = d0 + 256 * d1, p1 = d2 + 256 * d3, p2 = d4 + 256 * d5;
  double v = (double)d6;
  v = fma(v, 65536.0, (double)p2);
  v = fma(v, 65536.0, (double)p1);
  return fma(v, 65536.0, (double)p0) * 0x1p-36;
}

// ------------------------------------------------------------------ baseline digit sums
// Zq[set][l][k][Bp] = sum over cells with a baseline column of W8[set][c][b] * digit_l(DQ[bc][k]).
// Block: 64 grid points (lanes) x 8 boots x a chunk of kZChunk cells, 4 waves over the chunk's
// cells (c = wave mod 4); exact integer partials combine by LDS then global atomics (order-free;
// Zq is zeroed first).
__global__ __launch_bounds__(256) void k_zq(const unsigned long long* __restrict__ DQ, int G, int GS,
                                            const int* __restrict__ base_col, int ncells,
                                            const unsigned char* __restrict__ W8, int Bp, int* __restrict__ Zq) {
  __shared__ int part[7][8][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = (ncells + kZChunk - 1) / kZChunk;
  const int b0 = blockIdx.x * 8, k = blockIdx.y * 64 + lane, set = blockIdx.z / nch;
  const int c0 = (blockIdx.z % nch) * kZChunk, c1 = min(ncells, c0 + kZChunk);
  for (int i = threadIdx.x; i < 7 * 8 * 64; i += 256) (&part[0][0][0])[i] = 0;
  __syncthreads();
  int acc[8][7];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int l = 0; l < 7; ++l) acc[r][l] = 0;
  const unsigned char* W = W8 + (long long)set * ncells * Bp + b0;
  if (k < GS) {
    for (int c = c0 + wid; c < c1; c += 4) {
      const int bc = base_col[c];
      if (bc < 0) continue;
      const unsigned long long p = DQ[(long long)bc * GS + k];
      const unsigned long long w8 = *reinterpret_cast<const unsigned long long*>(W + (long long)c * Bp);
#pragma unroll
      for (int l = 0; l < 7; ++l) {
        const int d = sbyte(p, l);
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r][l] += d * (int)((w8 >> (8 * r)) & 0xff);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int l = 0; l < 7; ++l) atomicAdd(&part[l][r][lane], acc[r][l]);
  __syncthreads();
  if (k < GS)
    for (int i = wid; i < 7 * 8; i += 4) {
      const int l = i >> 3, rr = i & 7;
      const int v = part[l][rr][lane];
      if (v) atomicAdd(Zq + (((long long)set * 7 + l) * GS + k) * Bp + b0 + rr, v);
    }
}

// ZUq[set][l][t][Bp] = sum over baseline cells of W8[set][c][b] * digit_l(UQ[bc][t]), l < 4.
// Block per (set, 32 boots, chunk of kZChunk cells); thread = (tile, boot); global atomics
// (exact; ZUq is zeroed first).
__global__ __launch_bounds__(1024) void k_zuq(const unsigned* __restrict__ UQ, const int* __restrict__ base_col,
                                              int ncells, const unsigned char* __restrict__ W8, int Bp,
                                              int* __restrict__ ZUq) {
  const int nch = (ncells + kZChunk - 1) / kZChunk;
  const int t = threadIdx.x >> 5, b = blockIdx.x * 32 + (threadIdx.x & 31), set = blockIdx.y / nch;
  const int c0 = (blockIdx.y % nch) * kZChunk, c1 = min(ncells, c0 + kZChunk);
  const unsigned char* W = W8 + (long long)set * ncells * Bp + b;
  int acc[4] = {0, 0, 0, 0};
  for (int c = c0; c < c1; ++c) {
    const int bc = base_col[c];
    if (bc < 0) continue;
    const int w = W[(long long)c * Bp];
    const unsigned u = UQ[(long long)bc * kQTiles + t];
#pragma unroll
    for (int l = 0; l < 4; ++l) acc[l] += w * (int)(signed char)(u >> (8 * l));
  }
#pragma unroll
  for (int l = 0; l < 4; ++l)
    if (acc[l]) atomicAdd(ZUq + (((long long)set * 4 + l) * kQTiles + t) * Bp + b, acc[l]);
}

// ------------------------------------------------------------------ the bootstrap
// One 512-thread block per gene; boots in slabs of 32 (two 16-boot MFMA tiles).  Per slab:
//   1. the slab's multiplicities of the gene's entries -> LDS Wa[boot][entry] (the A
//      fragments, 16 entries per ds_read_b128);
//   2. tile bounds UB[32 boots][28 tiles] (waves 0-3, one 16 x 16 output tile each);
//   3. kept tiles; each wave computes its share (klist slots w, w+8, ...): per 64-entry
//      step every lane loads its grid point's 16 entries (u64 digit words), transposes them
//      into seven digit planes (v_perm_b32), and issues 2 x 7 MFMAs; the seven int32
//      accumulators combine into one double per (boot, point), kept in registers;
//   4. per-boot maxima (f32, tile-wise in LDS), the post-check and further tiles;
//   5. exp (terms below e^-50 of the maximum are zero), per-boot sums in tile order, jp row
//      += sum_b p_b[k] / (S_b nboot) in slab order.
__global__ __launch_bounds__(512) void k_bootq(BootQArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char qsm[];
  __shared__ double ub[kQSlab][kQMaxTiles + 1];
  __shared__ float tmax[kQMaxTiles][kQSlab];
  __shared__ double tsum[kQMaxTiles][kQSlab];
  __shared__ double jprow[kQMaxTiles * 16];
  __shared__ double etab[64];
  __shared__ float Mb[kQSlab];
  __shared__ double invb[kQSlab];
  __shared__ int klist[kQMaxTiles];
  __shared__ int nk_s, flag_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int g = blockIdx.x;
  if (g >= a.ngenes) return;
  if (*a.nanflag) {  // a NaN in some table: the exact path takes every gene
    if (tid == 0) {
      a.degen[g] = 1;
      atomicAdd(a.ndegen, 1);
    }
    return;
  }
  const int G = a.G, GS = a.GS, C = a.ncells, Bp = a.Bp;
  const int NT = (G + 15) / 16;
  const int n = a.nnz[g];
  const int ES = a.ent_stride;
  const int KP = (n + 63) & ~63;
  const int WS = ES + 16;  // Wa row stride (bytes)
  int* scol = reinterpret_cast<int*>(qsm);
  int* scell = scol + ES;
  unsigned char* Wa = reinterpret_cast<unsigned char*>(scell + ES);
  {
    const int2* E = a.ent + (long long)g * ES;
    for (int e = tid; e < KP; e += 512) {
      const int2 x = E[e];
      scol[e] = x.y;
      scell[e] = x.x;
    }
  }
  if (tid < 64) etab[tid] = kExp2Frac64[tid];
  for (int k = tid; k < kQMaxTiles * 16; k += 512) jprow[k] = 0.0;
  const int set = a.wset ? a.wset[g] : 0;
  const unsigned char* W8T = a.W8T + (long long)set * Bp * C;
  const int* Zq = a.Zq + (long long)set * 7 * GS * Bp;
  const int* ZUq = a.ZUq + (long long)set * 4 * kQTiles * Bp;
  const double slack = a.slack;
  const int nslab = (a.nboot + kQSlab - 1) / kQSlab;
  bool gene_degen = false;
  __syncthreads();
  for (int s = 0; s < nslab; ++s) {
    const int b0 = s * kQSlab;
    // ---- 1. multiplicities of the gene's entries, [boot][entry] bytes
    {
      const int nq = KP >> 2;
      for (int i = tid; i < kQSlab * nq; i += 512) {
        const int rr = i / nq, q = i - rr * nq;
        const unsigned char* wr = W8T + (long long)(b0 + rr) * C;
        const int4 cc = *reinterpret_cast<const int4*>(scell + 4 * q);
        const unsigned v = (unsigned)wr[cc.x] | ((unsigned)wr[cc.y] << 8) | ((unsigned)wr[cc.z] << 16) |
                           ((unsigned)wr[cc.w] << 24);
        *reinterpret_cast<unsigned*>(Wa + rr * WS + 4 * q) = v;
      }
      for (int i = tid; i < kQMaxTiles * kQSlab; i += 512) {
        (&tmax[0][0])[i] = -INFINITY;
        (&tsum[0][0])[i] = 0.0;
      }
    }
    __syncthreads();
    // ---- 2. tile bounds: wave w < 4 -> boot tile w & 1, tiles 16 (w >> 1) .. + 15
    if (wid < 4) {
      const int bt = wid & 1, tg = wid >> 1, t = 16 * tg + r;
      i32x4 acc[4];
#pragma unroll
      for (int l = 0; l < 4; ++l)
        acc[l] = *reinterpret_cast<const i32x4*>(ZUq + ((long long)l * kQTiles + t) * Bp + b0 + 16 * bt + 4 * h);
      for (int e0 = 0; e0 < KP; e0 += 64) {
        const i32x4 af = *reinterpret_cast<const i32x4*>(Wa + (16 * bt + r) * WS + e0 + 16 * h);
        unsigned u[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) u[j] = a.UQ[(long long)scol[e0 + 16 * h + j] * kQTiles + t];
        unsigned pl[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) tr4(u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3], pl[0][q], pl[1][q], pl[2][q], pl[3][q]);
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          const i32x4 bf = {(int)pl[l][0], (int)pl[l][1], (int)pl[l][2], (int)pl[l][3]};
          acc[l] = mfma_i8(af, bf, acc[l]);
        }
      }
      if (t < kQMaxTiles)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const long long v = (((long long)acc[3][q] * 256 + acc[2][q]) * 256 + acc[1][q]) * 256 + acc[0][q];
          ub[16 * bt + 4 * h + q][t] = (double)v * 0x1p-8;
        }
    }
    __syncthreads();
    // ---- 3. tiles to compute
    if (wid == 0) {
      const bool live = lane < kQSlab && b0 + lane < a.nboot;
      double m = -INFINITY;
      if (live)
        for (int t = 0; t < NT; ++t) m = fmax(m, ub[lane][t]);
      unsigned keep = 0;
      if (live)
        for (int t = 0; t < NT; ++t)
          if (ub[lane][t] >= m - 50.0 - slack) keep |= 1u << t;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) keep |= (unsigned)__shfl_xor((int)keep, o, 64);
      if (lane == 0) {
        int nk = 0;
        for (int t = 0; t < NT; ++t)
          if ((keep >> t) & 1) klist[nk++] = t;
        nk_s = nk;
      }
    }
    __syncthreads();
    // ---- 4. rows of the kept tiles, maxima, post-check (more tiles if it fails)
    double rows[kQSlotsPerWave][8];
    int done = 0, rounds = 0;
    for (;;) {
      const int nk = nk_s;
#pragma unroll
      for (int j = 0; j < kQSlotsPerWave; ++j) {
        const int slot = wid + kQWaves * j;
        if (slot < done || slot >= nk) continue;
        const int t = klist[slot];
        const int kk = 16 * t + r;
        i32x4 acc[2][7];
#pragma unroll
        for (int bt = 0; bt < 2; ++bt)
#pragma unroll
          for (int l = 0; l < 7; ++l)
            acc[bt][l] = *reinterpret_cast<const i32x4*>(Zq + ((long long)l * GS + kk) * Bp + b0 + 16 * bt + 4 * h);
        // the next 64-entry step's column words are in flight while this one is consumed
        auto fetch = [&](int e0, unsigned long long (&x)[16]) {
          const int4* cp = reinterpret_cast<const int4*>(scol + e0 + 16 * h);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int4 cc = cp[q];
            const int cj[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) x[4 * q + i] = a.DQ[(unsigned long long)(unsigned)(cj[i] * GS + kk)];
          }
        };
        unsigned long long xn[16];
        if (KP > 0) fetch(0, xn);
        for (int e0 = 0; e0 < KP; e0 += 64) {
          unsigned lo[16], hi[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            lo[i] = (unsigned)xn[i];
            hi[i] = (unsigned)(xn[i] >> 32);
          }
          if (e0 + 64 < KP) fetch(e0 + 64, xn);
          const i32x4 af0 = *reinterpret_cast<const i32x4*>(Wa + r * WS + e0 + 16 * h);
          const i32x4 af1 = *reinterpret_cast<const i32x4*>(Wa + (16 + r) * WS + e0 + 16 * h);
          unsigned pl[8][4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            tr4(lo[4 * q], lo[4 * q + 1], lo[4 * q + 2], lo[4 * q + 3], pl[0][q], pl[1][q], pl[2][q], pl[3][q]);
            tr4(hi[4 * q], hi[4 * q + 1], hi[4 * q + 2], hi[4 * q + 3], pl[4][q], pl[5][q], pl[6][q], pl[7][q]);
          }
#pragma unroll
          for (int l = 0; l < 7; ++l) {
            const i32x4 bf = {(int)pl[l][0], (int)pl[l][1], (int)pl[l][2], (int)pl[l][3]};
            acc[0][l] = mfma_i8(af0, bf, acc[0][l]);
            acc[1][l] = mfma_i8(af1, bf, acc[1][l]);
          }
        }
        // seven digit sums -> one double (pairs exact in int32, then exact FP64 steps to 2^51)
        float mx[8];
#pragma unroll
        for (int bt = 0; bt < 2; ++bt)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            double v = qcombine(acc[bt][0][q], acc[bt][1][q], acc[bt][2][q], acc[bt][3][q], acc[bt][4][q],
                                acc[bt][5][q], acc[bt][6][q]);
            v = kk < G ? v : -INFINITY;
            rows[j][4 * bt + q] = v;
            mx[4 * bt + q] = (float)v;
          }
        // tile maxima per boot: over the 16 lanes of this lane group
#pragma unroll
        for (int o = 1; o < 16; o <<= 1)
#pragma unroll
          for (int i = 0; i < 8; ++i) mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], o, 64));
        if (r < 8) {
          float v = mx[0];
#pragma unroll
          for (int i = 1; i < 8; ++i) v = (r == i) ? mx[i] : v;
          tmax[t][16 * (r >> 2) + 4 * h + (r & 3)] = v;
        }
      }
      __syncthreads();
      if (wid == 0) {
        const bool live = lane < kQSlab && b0 + lane < a.nboot;
        float m = -INFINITY;
        if (lane < kQSlab)
          for (int t = 0; t < NT; ++t) m = fmaxf(m, tmax[t][lane]);
        if (lane < kQSlab) Mb[lane] = m;
        unsigned kept = 0;
        for (int i = 0; i < nk; ++i) kept |= 1u << klist[i];
        unsigned fail = 0;
        if (live)
          for (int t = 0; t < NT; ++t)
            if (!((kept >> t) & 1) && !(ub[lane][t] < (double)m - 51.0)) fail |= 1u << t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) fail |= (unsigned)__shfl_xor((int)fail, o, 64);
        const bool bad = live && !((double)m >= -kQSat + 51.0);  // saturation may matter (or NaN)
        const bool anybad = __ballot(bad) != 0;
        if (lane == 0) {
          int nn = nk;
          for (int t = 0; t < NT; ++t)
            if ((fail >> t) & 1) klist[nn++] = t;
          nk_s = nn;
          flag_s = anybad ? 1 : 0;
        }
      }
      __syncthreads();
      done = nk;
      ++rounds;
      if (nk_s == nk) break;
    }
    if (flag_s) {  // uniform: the exact path recomputes this gene
      gene_degen = true;
      break;
    }
    if (a.stats && tid == 0) {
      atomicAdd(&a.stats[0], 1);
      atomicAdd(&a.stats[1], nk_s);
      atomicAdd(&a.stats[2], NT);
      atomicAdd(&a.stats[3], rounds - 1);
      atomicAdd(&a.stats[4 + nk_s], 1);  // histogram of tiles per slab
      atomicAdd(&a.stats[33], nk_s * (KP >> 6));  // 64-entry steps of the row MFMAs (14 each)
      atomicAdd(&a.stats[34], KP >> 6);           // ... of the bound MFMAs (16 each)
    }
    // ---- 5. softmax terms, per-boot sums (tile order), jp
    const int nk = nk_s;
#pragma unroll
    for (int j = 0; j < kQSlotsPerWave; ++j) {
      const int slot = wid + kQWaves * j;
      if (slot >= nk) continue;
      const int t = klist[slot];
      double sm[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int b = 16 * (i >> 2) + 4 * h + (i & 3);
        const double d = rows[j][i] - (double)Mb[b];
        const bool need = d >= -50.0;
        double e = 0.0;
        if (__ballot(need)) e = need ? exp_tab(d, etab) : 0.0;
        rows[j][i] = e;
        sm[i] = e;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int i = 0; i < 8; ++i) sm[i] += __shfl_xor(sm[i], o, 64);
      if (r < 8) {
        double v = sm[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) v = (r == i) ? sm[i] : v;
        tsum[t][16 * (r >> 2) + 4 * h + (r & 3)] = v;
      }
    }
    __syncthreads();
    if (wid == 0 && lane < kQSlab) {
      double S = 0.0;
      for (int t = 0; t < NT; ++t) S += tsum[t][lane];
      invb[lane] = (b0 + lane < a.nboot) ? 1.0 / (S * a.norm_mult) : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kQSlotsPerWave; ++j) {
      const int slot = wid + kQWaves * j;
      if (slot >= nk) continue;
      const int t = klist[slot];
      double pj = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i) pj = fma(rows[j][i], invb[16 * (i >> 2) + 4 * h + (i & 3)], pj);
      pj += __shfl_xor(pj, 16, 64);
      pj += __shfl_xor(pj, 32, 64);
      const int kk = 16 * t + r;
      if (h == 0 && kk < G) jprow[kk] += pj;
    }
    __syncthreads();
  }
  if (gene_degen) {
    if (tid == 0) {
      a.degen[g] = 1;
      atomicAdd(a.ndegen, 1);
    }
    return;
  }
  for (int k = tid; k < G; k += 512) a.out[(long long)g * a.out_g + (long long)k * a.out_k] = jprow[k];
}

size_t bootq_lds_bytes(int ent_stride) { return (size_t)ent_stride * 8 + (size_t)kQSlab * (ent_stride + 16); }

hipError_t launch_zq(const unsigned long long* DQ, int G, int GS, const int* base_col, int ncells,
                     const unsigned char* W8, int Bp, int nsets, int* Zq, hipStream_t s) {
  if (Bp % 8 || GS % 64) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(Zq, 0, sizeof(int) * (size_t)nsets * 7 * GS * Bp, s);
  if (e != hipSuccess) return e;
  const int nch = (ncells + kZChunk - 1) / kZChunk;
  hipLaunchKernelGGL(k_zq, dim3(Bp / 8, GS / 64, nsets * nch), dim3(256), 0, s, DQ, G, GS, base_col, ncells, W8, Bp,
                     Zq);
  return hipGetLastError();
}

hipError_t launch_zuq(const unsigned* UQ, const int* base_col, int ncells, const unsigned char* W8, int Bp, int nsets,
                      int* ZUq, hipStream_t s) {
  if (Bp % 32) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(ZUq, 0, sizeof(int) * (size_t)nsets * 4 * kQTiles * Bp, s);
  if (e != hipSuccess) return e;
  const int nch = (ncells + kZChunk - 1) / kZChunk;
  hipLaunchKernelGGL(k_zuq, dim3(Bp / 32, nsets * nch), dim3(1024), 0, s, UQ, base_col, ncells, W8, Bp, ZUq);
  return hipGetLastError();
}

hipError_t launch_bootq(const BootQArgs& a, hipStream_t s) {
  if (a.ngenes <= 0) return hipSuccess;
  if (a.G > kQMaxTiles * 16 || a.Bp % kQSlab || a.ent_stride % 64 || a.GS % 64) return hipErrorInvalidValue;
  const size_t shm = bootq_lds_bytes(a.ent_stride);
  hipLaunchKernelGGL(k_bootq, dim3(a.ngenes), dim3(512), shm, s, a);
  return hipGetLastError();
}

}  // namespace scde
