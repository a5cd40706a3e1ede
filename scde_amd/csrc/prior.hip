// prior.hip -- scde.expression.prior (R/functions.R:225-254) on device-resident counts.
//
// The producer of the DE path's `prior` input.  Per (gene, cell):
//   mag  = (log(count) - corr.b) / corr.a                       scde.expression.magnitude (694-697)
//   fail = 1 / (exp(mag conc.a [+ mag^2 conc.a2] + conc.b) + 1)  scde.failure.probability (725-750)
//   v    = log10(exp(mag) + 1),  w = 1 - fail (NaN fail -> 0)
// then density(c(-v, v), bw, weights = c(w, w) / (2 sum w), n = 2L + 1, from = -max, to = max)
// (stats::density.default, gaussian kernel, pre-4.4 grid), its upper half + pseudo count,
// normalised; lp and grid.weight.
//
// Kernels:
//   k_prior_occ    element pass 1.  v and w depend only on (cell, count): per (cell, gene
//                  tile) the counts < 256 are histogrammed in LDS (zeros by ballot) and each
//                  (cell, count) present is evaluated once; larger counts per element.
//                  Double-double sums of w (all, finite v; exact w * multiplicity), max and
//                  count of finite v.  k_prior_vals writes v itself for quantile(p < 1).
//   k_prior_bin    element pass 2: C_BinDist linear binning of +-v from the same (cell,
//                  count) multiplicities (+ the large counts per element).  Each bin term
//                  w_i (1 - fx) is rounded to a 2^-60 fixed point and summed in int64 (LDS
//                  histogram per block, integer atomics into the global one): deterministic
//                  and order-independent, so k copies add exactly k times one term.
//   k_prior_kords  dnorm(kords, sd = bw) on the 2n circular lags (nmath dnorm4).
//   k_prior_conv   the FFT cross-correlation of R as the direct sum over the n nonzero bins
//                  (y = histogram * 2^-60 * totMass), LDS-staged.
//   k_prior_final  approx(rule = 1) at the upper-half output points, pseudo count,
//                  double-double normalisation, lp, grid.weight.
// Work items of the element passes are (cell, 2048-gene tile): cell constants are
// wave-uniform and the count loads are coalesced down a column.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <hipcub/hipcub.hpp>

#include "device_math.h"
#include "kernels.h"

namespace scde {
namespace {

constexpr int kPriorBlock = 256;
constexpr int kPriorGenesPerThread = 16;
constexpr int kPriorSmall = kPriorBlock;  // counts below this are histogrammed per (cell, tile)
constexpr int kPriorTile = kPriorBlock * kPriorGenesPerThread;
constexpr double kFix = 1152921504606846976.0;  // 2^60
constexpr double kInvFix = 1.0 / 1152921504606846976.0;

struct PriorCell {
  double cb, ca, kb, ka, ka2;
};

__device__ inline void prior_elem(int count, const PriorCell& p, int sq, double& v, double& w) {
  const double mag = (log((double)count) - p.cb) / p.ca;
  double e = mag * p.ka;
  if (sq) e = e + (mag * mag) * p.ka2;
  double f = 1.0 / (exp(e + p.kb) + 1.0);
  if (isnan(f)) f = 0.0;
  w = 1.0 - f;
  v = log10(exp(mag) + 1.0);
}

__device__ inline PriorCell load_cell(const double* cellp, int C, int c) {
  PriorCell p;
  p.cb = cellp[c];
  p.ca = cellp[C + c];
  p.kb = cellp[2 * C + c];
  p.ka = cellp[3 * C + c];
  p.ka2 = cellp[4 * C + c];
  return p;
}

// exact w * k as a double-double (k < 2^31)
__device__ inline dd dd_mul_int(double w, int k) {
  const double kk = (double)k;
  const double hi = __dmul_rn(w, kk);
  return dd{hi, fma(w, kk, -hi)};
}

__device__ inline void stats_add(dd& sa, dd& sf, double& vmax, double& nfin, double v, double w, int k) {
  const dd t = k == 1 ? dd{w, 0.0} : dd_mul_int(w, k);
  sa = dd_add(sa, t);
  if (v < INFINITY) {
    sf = dd_add(sf, t);
    vmax = fmax(vmax, v);
    nfin += (double)k;
  }
}

__device__ inline void block_stats_out(dd sa, dd sf, double vmax, double nfin, double* __restrict__ out6) {
  __shared__ double red[6][kPriorBlock];
  const int tid = threadIdx.x;
  red[0][tid] = sa.hi;
  red[1][tid] = sa.lo;
  red[2][tid] = sf.hi;
  red[3][tid] = sf.lo;
  red[4][tid] = vmax;
  red[5][tid] = nfin;
  __syncthreads();
  for (int s = kPriorBlock / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const dd a = dd_add(dd{red[0][tid], red[1][tid]}, dd{red[0][tid + s], red[1][tid + s]});
      const dd b = dd_add(dd{red[2][tid], red[3][tid]}, dd{red[2][tid + s], red[3][tid + s]});
      red[0][tid] = a.hi;
      red[1][tid] = a.lo;
      red[2][tid] = b.hi;
      red[3][tid] = b.lo;
      red[4][tid] = fmax(red[4][tid], red[4][tid + s]);
      red[5][tid] += red[5][tid + s];
    }
    __syncthreads();
  }
  if (tid < 6) out6[tid] = red[tid][0];
}

// Appends `cnt` to the block's LDS queue on the lanes where `take` holds (wave-aggregated:
// one LDS atomic per wave, slots by mbcnt).  Call from wave-uniform control flow.
__device__ inline void queue_push(bool take, int cnt, int* queue, int* qn) {
  const unsigned long long m = __ballot(take);
  if (!m) return;
  int base = 0;
  if (__lane_id() == 0) base = atomicAdd(qn, __popcll(m));
  base = __builtin_amdgcn_readfirstlane(base);
  const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
  if (take) queue[base + r] = cnt;
}

// Element pass 1.  Per work item (cell c, tile of kPriorTile genes): occurrences of each
// count < kPriorSmall in LDS (zeros by ballot), written to occ[item][kPriorSmall]; larger
// (or negative) counts are evaluated per element.  Then each (c, count) present is evaluated
// once and enters the sums with its multiplicity.  Per-block partials:
// [S_all.hi, S_all.lo, S_fin.hi, S_fin.lo, max finite v, n finite v].
__global__ __launch_bounds__(kPriorBlock) void k_prior_occ(const int* __restrict__ counts, long long ld, int N,
                                                           int C, const double* __restrict__ cellp, int sq,
                                                           int* __restrict__ occ_out,
                                                           double* __restrict__ partials) {
  __shared__ int occ[kPriorSmall];
  __shared__ int queue[kPriorTile];
  __shared__ int qn;
  const int tid = threadIdx.x;
  const int ntiles = (N + kPriorTile - 1) / kPriorTile;
  const long long items = (long long)ntiles * C;
  dd sa{0.0, 0.0}, sf{0.0, 0.0};
  double vmax = -INFINITY, nfin = 0.0;
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const int c = (int)(it / ntiles), tile = (int)(it % ntiles);
    const PriorCell p = load_cell(cellp, C, c);
    const int* col = counts + (long long)c * ld;
    occ[tid] = 0;
    if (tid == 0) qn = 0;
    __syncthreads();
    int zeros = 0;
    const int g0 = tile * kPriorTile + tid;
    int cv[kPriorGenesPerThread];  // all loads in flight before any LDS atomic
#pragma unroll
    for (int k = 0; k < kPriorGenesPerThread; ++k) {
      const int g = g0 + k * kPriorBlock;
      cv[k] = g < N ? __builtin_nontemporal_load(col + g) : 1;
    }
#pragma unroll
    for (int k = 0; k < kPriorGenesPerThread; ++k) {
      const int g = g0 + k * kPriorBlock;
      const int cnt = cv[k];
      zeros += __popcll(__ballot(cnt == 0));
      if (g < N && cnt != 0 && (unsigned)cnt < (unsigned)kPriorSmall) atomicAdd(&occ[cnt], 1);
      // large (or negative) counts: queued, then evaluated by full waves
      queue_push(g < N && (unsigned)cnt >= (unsigned)kPriorSmall, cnt, queue, &qn);
    }
    if (zeros && __lane_id() == 0) atomicAdd(&occ[0], zeros);
    __syncthreads();
    for (int q = tid; q < qn; q += kPriorBlock) {
      double v, w;
      prior_elem(queue[q], p, sq, v, w);
      stats_add(sa, sf, vmax, nfin, v, w, 1);
    }
    const int o = occ[tid];
    occ_out[it * kPriorSmall + tid] = o;
    if (o) {
      double v, w;
      prior_elem(tid, p, sq, v, w);
      stats_add(sa, sf, vmax, nfin, v, w, o);
    }
    __syncthreads();
  }
  block_stats_out(sa, sf, vmax, nfin, partials + (long long)blockIdx.x * 6);
}

// v per element in R order (the quantile path only)
__global__ __launch_bounds__(kPriorBlock) void k_prior_vals(const int* __restrict__ counts, long long ld, int N, int C,
                                                            const double* __restrict__ cellp, int sq,
                                                            double* __restrict__ vout) {
  const long long e = (long long)blockIdx.x * kPriorBlock + threadIdx.x;
  if (e >= (long long)N * C) return;
  const int c = (int)(e / N), g = (int)(e % N);
  double v, w;
  prior_elem(counts[(long long)c * ld + g], load_cell(cellp, C, c), sq, v, w);
  vout[e] = v;
}

// One block: partials (nb x 6) -> out[0..3] = S_all, S_fin (rounded dd), max, nfinite.
__global__ __launch_bounds__(kPriorBlock) void k_prior_stats_reduce(const double* __restrict__ partials, int nb,
                                                                    double* __restrict__ out) {
  const int tid = threadIdx.x;
  dd sa{0.0, 0.0}, sf{0.0, 0.0};
  double vmax = -INFINITY, nfin = 0.0;
  for (int b = tid; b < nb; b += kPriorBlock) {
    const double* q = partials + (long long)b * 6;
    sa = dd_add(sa, dd{q[0], q[1]});
    sf = dd_add(sf, dd{q[2], q[3]});
    vmax = fmax(vmax, q[4]);
    nfin += q[5];
  }
  __shared__ double fin[6];
  block_stats_out(sa, sf, vmax, nfin, fin);
  __syncthreads();
  if (tid == 0) {
    out[0] = dd_to_d(dd{fin[0], fin[1]});
    out[1] = dd_to_d(dd{fin[2], fin[3]});
    out[2] = fin[4];
    out[3] = fin[5];
  }
}

__device__ inline void fix_add(unsigned long long* h, int i, double t, unsigned long long mult) {
  const unsigned long long q = __double2ull_rn(t * kFix);
  if (q) atomicAdd(h + i, q * mult);
}

// C_BinDist (stats/src/massdist.c) for `mult` copies of one value: each copy's terms are
// rounded to the fixed point, so mult copies add exactly mult times that integer.
__device__ inline void bin_one(double x, double wi, double lo, double xdelta, int n, unsigned long long* h,
                               unsigned long long mult) {
  if (!isfinite(x)) return;
  const double xpos = (x - lo) / xdelta;
  if (!(xpos >= -1.0 && xpos < (double)n)) return;
  const int ix = (int)floor(xpos);
  const double fx = xpos - ix;
  const int ixmax = n - 2;
  if (ix >= 0 && ix <= ixmax) {
    fix_add(h, ix, wi * (1 - fx), mult);
    fix_add(h, ix + 1, wi * fx, mult);
  } else if (ix == -1) {
    fix_add(h, 0, wi * fx, mult);
  } else if (ix == ixmax + 1) {
    fix_add(h, ix, wi * (1 - fx), mult);
  }
}

// Element pass 2: the same work items; each (cell, small count) present bins with its
// multiplicity from pass 1, the large counts are re-read and binned per element.  LDS
// histogram per block, integer-added into the global histogram (exact, order-free).
__global__ __launch_bounds__(kPriorBlock) void k_prior_bin(const int* __restrict__ counts, long long ld, int N, int C,
                                                           const double* __restrict__ cellp, int sq,
                                                           const int* __restrict__ occ_in, double wsum, double lo,
                                                           double xdelta, int n,
                                                           unsigned long long* __restrict__ hist_out) {
  extern __shared__ unsigned long long hist[];
  __shared__ int queue[kPriorTile];
  __shared__ int qn;
  const int tid = threadIdx.x;
  for (int j = tid; j < n; j += kPriorBlock) hist[j] = 0ull;
  const int ntiles = (N + kPriorTile - 1) / kPriorTile;
  const long long items = (long long)ntiles * C;
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const int c = (int)(it / ntiles), tile = (int)(it % ntiles);
    const PriorCell p = load_cell(cellp, C, c);
    if (tid == 0) qn = 0;
    __syncthreads();
    const int o = occ_in[it * kPriorSmall + tid];
    if (o) {
      double v, w;
      prior_elem(tid, p, sq, v, w);
      const double wi = (w / wsum) * 0.5;  // c(wts/2, wts/2), wts = w / sum(w)
      bin_one(-v, wi, lo, xdelta, n, hist, (unsigned long long)o);
      bin_one(v, wi, lo, xdelta, n, hist, (unsigned long long)o);
    }
    const int* col = counts + (long long)c * ld;
    const int g0 = tile * kPriorTile + tid;
    int cv[kPriorGenesPerThread];
#pragma unroll
    for (int k = 0; k < kPriorGenesPerThread; ++k) {
      const int g = g0 + k * kPriorBlock;
      cv[k] = g < N ? __builtin_nontemporal_load(col + g) : 0;
    }
#pragma unroll
    for (int k = 0; k < kPriorGenesPerThread; ++k)
      queue_push(g0 + k * kPriorBlock < N && (unsigned)cv[k] >= (unsigned)kPriorSmall, cv[k], queue, &qn);
    __syncthreads();
    for (int q = tid; q < qn; q += kPriorBlock) {
      double v, w;
      prior_elem(queue[q], p, sq, v, w);
      const double wi = (w / wsum) * 0.5;
      bin_one(-v, wi, lo, xdelta, n, hist, 1ull);
      bin_one(v, wi, lo, xdelta, n, hist, 1ull);
    }
    __syncthreads();
  }
  __syncthreads();
  for (int j = tid; j < n; j += kPriorBlock)
    if (hist[j]) atomicAdd(hist_out + j, hist[j]);
}

// seq.int(from, to, length.out = len)[i]
__device__ inline double r_seq_at(double from, double to, int len, int i) {
  if (len > 1 && i == len - 1) return to;
  const double by = len > 1 ? (to - from) / (double)(len - 1) : 0.0;
  return from + (double)i * by;
}

// nmath dnorm4(x, 0, sigma, FALSE)
__device__ inline double r_dnorm0(double x, double sigma) {
  constexpr double kInvSqrt2Pi = 0.398942280401432677939946059934;
  x = fabs(x / sigma);
  if (x >= 2 * sqrt(DBL_MAX)) return 0.0;
  if (x < 5) return kInvSqrt2Pi * exp(-0.5 * x * x) / sigma;
  if (x > sqrt(-2 * M_LN2 * (DBL_MIN_EXP + 1 - DBL_MANT_DIG))) return 0.0;
  const double x1 = ldexp(rint(ldexp(x, 16)), -16);
  const double x2 = x - x1;
  return kInvSqrt2Pi / sigma * (exp(-0.5 * x1 * x1) * exp((-0.5 * x2 - x1) * x2));
}

// kords <- seq.int(0, 2*(up-lo), length.out = 2n); kords[(n+2):(2n)] <- -kords[n:2]; dnorm(kords, sd = bw)
__global__ void k_prior_kords(int n, double span, double bw, double* __restrict__ K) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * n) return;
  const double k = j > n ? -r_seq_at(0.0, span, 2 * n, 2 * n - j) : r_seq_at(0.0, span, 2 * n, j);
  K[j] = r_dnorm0(k, bw);
}

// Re(fft(fft(y) * Conj(fft(kords)), inverse = TRUE))[k] / (2n) = sum_a y[a] kords[(a - k) mod 2n],
// y = BinDist(...) * totMass (zero beyond n-1); pmax(0, .).  A direct sum instead of R's FFT:
// y and kords staged in LDS, 64 outputs per block (one per lane), the 4 waves split the
// lags and combine in a fixed order.
__global__ __launch_bounds__(kPriorBlock) void k_prior_conv(const unsigned long long* __restrict__ hist,
                                                            double tot_mass, const double* __restrict__ K, int n,
                                                            double* __restrict__ dens) {
  extern __shared__ double sm[];
  double* y = sm;
  double* Ks = sm + n;
  const int tid = threadIdx.x;
  for (int j = tid; j < n; j += kPriorBlock) y[j] = ((double)hist[j] * kInvFix) * tot_mass;
  for (int j = tid; j < 2 * n; j += kPriorBlock) Ks[j] = K[j];
  __syncthreads();
  const int lane = tid & 63, part = tid >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int mask = 2 * n - 1, q = n / 4;
  double s = 0.0;
  if (k < n)
    for (int a = part * q; a < (part + 1) * q; ++a) s = fma(y[a], Ks[(a - k) & mask], s);
  __shared__ double red[4][64];
  red[part][lane] = s;
  __syncthreads();
  if (part == 0 && k < n) dens[k] = fmax(0.0, ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
}

// approx(xords, dens, xout = x, rule = 1) at the upper-half points x[L..2L]; NA -> 0;
// + pseudo.count / nrow; / sum (double-double); lp; grid.weight.  One block.
__global__ __launch_bounds__(1024) void k_prior_final(const double* __restrict__ dens, int n, double lo, double up,
                                                      double from, double to, int L, double pc,
                                                      double* __restrict__ out) {
  const int tid = threadIdx.x;
  const int nu = 2 * L + 1, m = L + 1;
  double* ox = out;
  double* oy = out + m;
  double* olp = out + 2 * m;
  double* ogw = out + 3 * m;
  dd part{0.0, 0.0};
  for (int i = tid; i < m; i += blockDim.x) {
    const double v = r_seq_at(from, to, nu, L + i);
    double r;
    const double x0 = r_seq_at(lo, up, n, 0), xn = r_seq_at(lo, up, n, n - 1);
    if (v < x0 || v > xn) {
      r = NAN;
    } else {
      int a = 0, b = n - 1;
      while (a < b - 1) {
        const int ij = (a + b) / 2;
        if (v < r_seq_at(lo, up, n, ij)) b = ij;
        else a = ij;
      }
      const double xa = r_seq_at(lo, up, n, a), xb = r_seq_at(lo, up, n, b);
      if (v == xb) r = dens[b];
      else if (v == xa) r = dens[a];
      else r = dens[a] + (dens[b] - dens[a]) * ((v - xa) / (xb - xa));
    }
    if (isnan(r)) r = 0.0;
    r = r + pc;
    ox[i] = v;
    oy[i] = r;
  }
  __syncthreads();
  // fixed-order double-double sum of y (R's long-double sum())
  for (int i = tid; i < m; i += blockDim.x) part = dd_add_d(part, oy[i]);
  __shared__ double rh[1024], rl[1024];
  rh[tid] = part.hi;
  rl[tid] = part.lo;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const dd t = dd_add(dd{rh[tid], rl[tid]}, dd{rh[tid + s], rl[tid + s]});
      rh[tid] = t.hi;
      rl[tid] = t.lo;
    }
    __syncthreads();
  }
  const double tot = dd_to_d(dd{rh[0], rl[0]});
  for (int i = tid; i < m; i += blockDim.x) {
    const double yy = oy[i] / tot;
    oy[i] = yy;
    olp[i] = log(yy);
    // grid.weight = diff(10^c(x[1], x + c(diff(x)/2, 0)) - 1)
    const double xi = ox[i];
    const double e_lo = i == 0 ? ox[0] : ox[i - 1] + (xi - ox[i - 1]) / 2;
    const double e_hi = i == m - 1 ? xi + 0.0 : xi + (ox[i + 1] - xi) / 2;
    ogw[i] = (pow(10.0, e_hi) - 1) - (pow(10.0, e_lo) - 1);
  }
}

}  // namespace

hipError_t launch_prior_stats(const int* counts, long long ld, int N, int C, const double* cellp, int sq,
                              double* vout, int* occ, double* partials, int nb, double* out, hipStream_t s) {
  k_prior_occ<<<nb, kPriorBlock, 0, s>>>(counts, ld, N, C, cellp, sq, occ, partials);
  if (vout) {
    const long long e = (long long)N * C;
    k_prior_vals<<<(unsigned)((e + kPriorBlock - 1) / kPriorBlock), kPriorBlock, 0, s>>>(counts, ld, N, C, cellp, sq,
                                                                                       vout);
  }
  k_prior_stats_reduce<<<1, kPriorBlock, 0, s>>>(partials, nb, out);
  return hipGetLastError();
}

long long prior_items(int N, int C) { return (long long)((N + kPriorTile - 1) / kPriorTile) * C; }

int prior_blocks(int N, int C, int cap) {
  const long long items = (long long)((N + kPriorTile - 1) / kPriorTile) * C;
  return (int)std::max<long long>(1, std::min<long long>(items, cap));
}

// density's internal grid size for n.user = 2L + 1 points
int prior_grid_n(int L) {
  const int nu = 2 * L + 1;
  int n = std::max(nu, 512);
  if (n > 512) n = 1 << (int)std::ceil(std::log2((double)n));
  return n;
}

hipError_t launch_prior_bin(const int* counts, long long ld, int N, int C, const double* cellp, int sq,
                            const int* occ, double wsum, double max_value, double bw, int L,
                            unsigned long long* hist, int nb, hipStream_t s) {
  const int n = prior_grid_n(L);
  const double lo = -max_value - 4 * bw, up = max_value + 4 * bw;
  const double xdelta = (up - lo) / (n - 1);
  hipError_t e = hipMemsetAsync(hist, 0, sizeof(unsigned long long) * n, s);
  if (e != hipSuccess) return e;
  k_prior_bin<<<nb, kPriorBlock, sizeof(unsigned long long) * n, s>>>(counts, ld, N, C, cellp, sq, occ, wsum, lo,
                                                                      xdelta, n, hist);
  return hipGetLastError();
}

hipError_t launch_prior_tail(double tot_mass, double max_value, double bw, int L, double pc,
                             const unsigned long long* hist, double* work, double* out, hipStream_t s) {
  const int n = prior_grid_n(L);
  const double from = -max_value, to = max_value;
  const double lo = from - 4 * bw, up = to + 4 * bw;
  double* K = work;
  double* dens = work + 2 * n;
  k_prior_kords<<<(2 * n + 255) / 256, 256, 0, s>>>(n, 2 * (up - lo), bw, K);
  k_prior_conv<<<(n + 63) / 64, kPriorBlock, sizeof(double) * 3 * n, s>>>(hist, tot_mass, K, n, dens);
  k_prior_final<<<1, 1024, 0, s>>>(dens, n, lo, up, from, to, L, pc, out);
  return hipGetLastError();
}

hipError_t launch_sort_doubles(const double* in, double* out, long long n, void* work, size_t* work_bytes,
                               hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(work, *work_bytes, in, out, (int)n, 0, 64, s);
}

}  // namespace scde
