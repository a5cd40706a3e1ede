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
//   k_prior_stats  element pass: double-double sums of w (all, finite v), max of finite v,
//                  count of finite v; optionally v itself (for quantile(max.quantile < 1)).
//   k_prior_bin    element pass: C_BinDist linear binning of +-v.  Each bin term w_i (1 - fx)
//                  is rounded to a 2^-60 fixed point and summed in int64 (LDS histogram per
//                  block, one partial histogram per block): deterministic, order-independent.
//   k_prior_hist   partial histograms -> y = sum * 2^-60 * totMass.
//   k_prior_kords  dnorm(kords, sd = bw) on the 2n circular lags (nmath dnorm4).
//   k_prior_conv   the FFT cross-correlation of R, as the direct sum over the n nonzero bins.
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
constexpr int kPriorGenesPerThread = 8;
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

// Per-block partials: [S_all.hi, S_all.lo, S_fin.hi, S_fin.lo, max finite v, n finite v].
__global__ __launch_bounds__(kPriorBlock) void k_prior_stats(const int* __restrict__ counts, long long ld, int N,
                                                             int C, const double* __restrict__ cellp, int sq,
                                                             double* __restrict__ vout,
                                                             double* __restrict__ partials) {
  const int tid = threadIdx.x;
  const int ntiles = (N + kPriorTile - 1) / kPriorTile;
  const long long items = (long long)ntiles * C;
  dd sa{0.0, 0.0}, sf{0.0, 0.0};
  double vmax = -INFINITY, nfin = 0.0;
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const int c = (int)(it / ntiles), tile = (int)(it % ntiles);
    const PriorCell p = load_cell(cellp, C, c);
    const int* col = counts + (long long)c * ld;
#pragma unroll 2
    for (int k = 0; k < kPriorGenesPerThread; ++k) {
      const int g = tile * kPriorTile + k * kPriorBlock + tid;
      if (g >= N) break;
      double v, w;
      prior_elem(col[g], p, sq, v, w);
      sa = dd_add_d(sa, w);
      if (v < INFINITY) {
        sf = dd_add_d(sf, w);
        vmax = fmax(vmax, v);
        nfin += 1.0;
      }
      if (vout) vout[(long long)c * N + g] = v;
    }
  }
  __shared__ double red[6][kPriorBlock];
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
  if (tid < 6) partials[(long long)blockIdx.x * 6 + tid] = red[tid][0];
}

// One block: partials (nb x 6) -> out[0..5] = S_all, S_fin (rounded dd), max, nfinite.
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
  __shared__ double red[6][kPriorBlock];
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
  if (tid == 0) {
    out[0] = dd_to_d(dd{red[0][0], red[1][0]});
    out[1] = dd_to_d(dd{red[2][0], red[3][0]});
    out[2] = red[4][0];
    out[3] = red[5][0];
  }
}

__device__ inline void fix_add(unsigned long long* h, int i, double t) {
  const unsigned long long q = __double2ull_rn(t * kFix);
  if (q) atomicAdd(h + i, q);
}

// C_BinDist (stats/src/massdist.c) for one value; xpos outside [-1, n) contributes nothing.
__device__ inline void bin_one(double x, double wi, double lo, double xdelta, int n, unsigned long long* h) {
  if (!isfinite(x)) return;
  const double xpos = (x - lo) / xdelta;
  if (!(xpos >= -1.0 && xpos < (double)n)) return;
  const int ix = (int)floor(xpos);
  const double fx = xpos - ix;
  const int ixmax = n - 2;
  if (ix >= 0 && ix <= ixmax) {
    fix_add(h, ix, wi * (1 - fx));
    fix_add(h, ix + 1, wi * fx);
  } else if (ix == -1) {
    fix_add(h, 0, wi * fx);
  } else if (ix == ixmax + 1) {
    fix_add(h, ix, wi * (1 - fx));
  }
}

__global__ __launch_bounds__(kPriorBlock) void k_prior_bin(const int* __restrict__ counts, long long ld, int N, int C,
                                                           const double* __restrict__ cellp, int sq, double wsum,
                                                           double lo, double xdelta, int n,
                                                           unsigned long long* __restrict__ partial) {
  extern __shared__ unsigned long long hist[];
  const int tid = threadIdx.x;
  for (int j = tid; j < n; j += kPriorBlock) hist[j] = 0ull;
  __syncthreads();
  // v == 0 (every zero count) lands in the same two bins for every cell: summed in
  // registers (the same fixed-point terms, exact integer sums) instead of contended atomics
  const double xpos0 = (0.0 - lo) / xdelta;
  const int ix0 = (int)floor(xpos0);
  const double fx0 = xpos0 - ix0;
  const bool zero_mid = ix0 >= 0 && ix0 <= n - 2;
  unsigned long long z0 = 0ull, z1 = 0ull;
  const int ntiles = (N + kPriorTile - 1) / kPriorTile;
  const long long items = (long long)ntiles * C;
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const int c = (int)(it / ntiles), tile = (int)(it % ntiles);
    const PriorCell p = load_cell(cellp, C, c);
    const int* col = counts + (long long)c * ld;
    for (int k = 0; k < kPriorGenesPerThread; ++k) {
      const int g = tile * kPriorTile + k * kPriorBlock + tid;
      if (g >= N) break;
      double v, w;
      prior_elem(col[g], p, sq, v, w);
      const double wi = (w / wsum) * 0.5;  // c(wts/2, wts/2), wts = w / sum(w)
      if (v == 0.0 && zero_mid) {
        const unsigned long long a = __double2ull_rn(wi * (1 - fx0) * kFix);
        const unsigned long long b = __double2ull_rn(wi * fx0 * kFix);
        z0 += 2 * a;  // -0 and +0
        z1 += 2 * b;
        continue;
      }
      bin_one(-v, wi, lo, xdelta, n, hist);
      bin_one(v, wi, lo, xdelta, n, hist);
    }
  }
  if (zero_mid) {
    if (z0) atomicAdd(hist + ix0, z0);
    if (z1) atomicAdd(hist + ix0 + 1, z1);
  }
  __syncthreads();
  for (int j = tid; j < n; j += kPriorBlock) partial[(long long)blockIdx.x * n + j] = hist[j];
}

// y[j] = (sum over blocks of partial[b][j]) * 2^-60 * totMass   (BinDist(...) * totMass)
__global__ __launch_bounds__(kPriorBlock) void k_prior_hist(const unsigned long long* __restrict__ partial, int nb,
                                                            int n, double tot_mass, double* __restrict__ y) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;  // 4 waves split the blocks
  unsigned long long s = 0ull;
  if (j < n)
    for (int b = part; b < nb; b += 4) s += partial[(long long)b * n + j];
  __shared__ unsigned long long red[4][64];
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && j < n) {
    const unsigned long long t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    y[j] = ((double)t * kInvFix) * tot_mass;
  }
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

// Re(fft(fft(y) * Conj(fft(kords)), inverse = TRUE))[k] / (2n) = sum_a y[a] kords[(a - k) mod 2n];
// y is zero beyond n-1.  pmax(0, .)
__global__ __launch_bounds__(kPriorBlock) void k_prior_conv(const double* __restrict__ y,
                                                            const double* __restrict__ K, int n,
                                                            double* __restrict__ dens) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int mask = 2 * n - 1;
  double s = 0.0;
  for (int a = 0; a < n; ++a) s = fma(y[a], K[(a - k) & mask], s);
  dens[k] = fmax(0.0, s);
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
                              double* vout, double* partials, int nb, double* out, hipStream_t s) {
  k_prior_stats<<<nb, kPriorBlock, 0, s>>>(counts, ld, N, C, cellp, sq, vout, partials);
  k_prior_stats_reduce<<<1, kPriorBlock, 0, s>>>(partials, nb, out);
  return hipGetLastError();
}

int prior_blocks(int N, int C, int cap) {
  const long long items = (long long)((N + kPriorTile - 1) / kPriorTile) * C;
  return (int)std::max<long long>(1, std::min<long long>(items, cap));
}

hipError_t launch_prior_density(const int* counts, long long ld, int N, int C, const double* cellp, int sq,
                                double wsum, double tot_mass, double max_value, double bw, int L, double pc,
                                unsigned long long* partial, int nb, double* work, double* out, hipStream_t s) {
  const int nu = 2 * L + 1;
  int n = std::max(nu, 512);
  if (n > 512) n = 1 << (int)std::ceil(std::log2((double)n));
  const double from = -max_value, to = max_value;
  const double lo = from - 4 * bw, up = to + 4 * bw;
  const double xdelta = (up - lo) / (n - 1);
  double* y = work;
  double* K = work + n;
  double* dens = K + 2 * n;
  k_prior_bin<<<nb, kPriorBlock, sizeof(unsigned long long) * n, s>>>(counts, ld, N, C, cellp, sq, wsum, lo, xdelta,
                                                                      n, partial);
  k_prior_hist<<<(n + 63) / 64, kPriorBlock, 0, s>>>(partial, nb, n, tot_mass, y);
  k_prior_kords<<<(2 * n + 255) / 256, 256, 0, s>>>(n, 2 * (up - lo), bw, K);
  k_prior_conv<<<(n + kPriorBlock - 1) / kPriorBlock, kPriorBlock, 0, s>>>(y, K, n, dens);
  k_prior_final<<<1, 1024, 0, s>>>(dens, n, lo, up, from, to, L, pc, out);
  return hipGetLastError();
}

// density's internal grid size for n.user = 2L + 1 points
int prior_grid_n(int L) {
  const int nu = 2 * L + 1;
  int n = std::max(nu, 512);
  if (n > 512) n = 1 << (int)std::ceil(std::log2((double)n));
  return n;
}

hipError_t launch_sort_doubles(const double* in, double* out, long long n, void* work, size_t* work_bytes,
                               hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(work, *work_bytes, in, out, (int)n, 0, 64, s);
}

}  // namespace scde
