// pagoda.hip -- scde's PAGODA helper kernels (src/pagoda.cpp) for gfx950:
//   winsorizeMatrix (src/pagoda.cpp:6-31)     k_winsorize_sort / k_winsorize_select
//   matCorr         (src/pagoda.cpp:33-38)    k_colstats + k_matcorr
//   matWCorr        (src/pagoda.cpp:41-65)    k_matwcorr
//   plSemicompleteCor2 (src/pagoda.cpp:67-117) k_plcor
//   pagoda.varnorm's posterior-mode consumer (R/functions.R:1423-1450, 1466-1474):
//     k_vn_modes (jp %*% magnitudes, or the magnitude of the row maximum), k_vn_matw
//     (matw = 1 - mfp * sfp: scde.failure.probability at log(modes) times ppois(count - 1,
//     exp(fail.r), lower.tail = FALSE))
// All FP64.  Reductions run lane-parallel in a fixed tree order, so sums differ from the
// reference's sequential BLAS/Armadillo order by rounding only.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace scde {
namespace {

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// (value, index) order: ties by position (the reference's std::sort leaves them
// unspecified; the result depends on it only when the two trimmed ranges overlap)
__device__ __forceinline__ bool before(double va, int ia, double vb, int ib) {
  return va < vb || (va == vb && ia < ib);
}

// lower-triangle pair q (0-based, j > i) of an n x n matrix -> (i, j)
__device__ __forceinline__ void tri_pair(long long q, int n, int& i, int& j) {
  const double nn = (double)n;
  long long ii = (long long)(nn - 2 - floor(sqrt(-8.0 * (double)q + 4.0 * nn * (nn - 1) - 7) / 2.0 - 0.5));
  if (ii < 0) ii = 0;
  // rows before i hold (n-1) + ... + (n-i) pairs
  auto before_rows = [&](long long r) { return r * (2LL * n - r - 1) / 2; };
  while (ii > 0 && before_rows(ii) > q) --ii;
  while (ii + 1 < n && before_rows(ii + 1) <= q) ++ii;
  i = (int)ii;
  j = (int)(q - before_rows(ii) + ii + 1);
}

}  // namespace

// ---- winsorizeMatrix: one workgroup per row (rows spread so consecutive rows share an
// XCD and its L2: row = (b % 8) * ceil(k / 8) + b / 8).  The row (stride k in R's
// column-major layout) is bitonic-sorted in LDS as (value, index) pairs.
__global__ __launch_bounds__(1024) void k_winsorize_sort(const double* __restrict__ m, int k, int n, int NP, int ntr,
                                                         double* __restrict__ out) {
  extern __shared__ double sv[];  // NP values, then NP int indices
  int* si = reinterpret_cast<int*>(sv + NP);
  const int per = (k + 7) / 8;
  const int row = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (row >= k) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int j = tid; j < NP; j += nt) {
    sv[j] = j < n ? m[row + (long long)j * k] : INFINITY;
    si[j] = j;
  }
  __syncthreads();
  for (int size = 2; size <= NP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < NP / 2; t += nt) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const double va = sv[lo], vb = sv[hi];
        const int ia = si[lo], ib = si[hi];
        const bool swap = asc ? before(vb, ib, va, ia) : before(va, ia, vb, ib);
        if (swap) {
          sv[lo] = vb;
          sv[hi] = va;
          si[lo] = ib;
          si[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  const double minv = sv[ntr], maxv = sv[n - ntr - 1];
  for (int r = tid; r < n; r += nt) {
    double v = sv[r];
    if (r >= n - ntr) v = maxv;
    else if (r < ntr) v = minv;
    out[row + (long long)si[r] * k] = v;
  }
}

// Rows longer than the LDS sort (n > 8192) with ntr <= 32: the ntr + 1 smallest and
// largest (value, index) pairs by repeated block arg-extremes; everything else unchanged.
__global__ __launch_bounds__(256) void k_winsorize_select(const double* __restrict__ m, int k, int n, int ntr,
                                                          double* __restrict__ out) {
  __shared__ double rv[4];
  __shared__ int ri[4];
  __shared__ int lo_idx[33], hi_idx[33];
  __shared__ double lo_val[33], hi_val[33];
  const int row = blockIdx.x;
  if (row >= k) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int j = tid; j < n; j += 256) out[row + (long long)j * k] = m[row + (long long)j * k];
  for (int side = 0; side < 2; ++side) {
    for (int t = 0; t <= ntr; ++t) {
      // extreme (value, index) not yet taken: strictly after the previous pick in the order
      const bool have_prev = t > 0;
      const double pv = have_prev ? (side == 0 ? lo_val[t - 1] : hi_val[t - 1]) : 0.0;
      const int pi = have_prev ? (side == 0 ? lo_idx[t - 1] : hi_idx[t - 1]) : -1;
      double bv = side == 0 ? INFINITY : -INFINITY;
      int bi = side == 0 ? 0x7fffffff : -1;
      for (int j = tid; j < n; j += 256) {
        const double v = m[row + (long long)j * k];
        if (side == 0) {
          if (have_prev && !before(pv, pi, v, j)) continue;
          if (before(v, j, bv, bi)) bv = v, bi = j;
        } else {
          if (have_prev && !before(v, j, pv, pi)) continue;
          if (before(bv, bi, v, j)) bv = v, bi = j;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o);
        const int oi = __shfl_xor(bi, o);
        const bool take = side == 0 ? before(ov, oi, bv, bi) : before(bv, bi, ov, oi);
        if (take) bv = ov, bi = oi;
      }
      if (lane == 0) rv[wid] = bv, ri[wid] = bi;
      __syncthreads();
      if (tid == 0) {
        double v = rv[0];
        int ix = ri[0];
        for (int w = 1; w < 4; ++w) {
          const bool take = side == 0 ? before(rv[w], ri[w], v, ix) : before(v, ix, rv[w], ri[w]);
          if (take) v = rv[w], ix = ri[w];
        }
        if (side == 0) lo_val[t] = v, lo_idx[t] = ix;
        else hi_val[t] = v, hi_idx[t] = ix;
      }
      __syncthreads();
    }
  }
  if (tid <= ntr) {
    // ranks < ntr -> minv (sorted[ntr]); ranks >= n - ntr -> maxv (sorted[n - ntr - 1]), the later write winning
    if (tid < ntr) out[row + (long long)lo_idx[tid] * k] = lo_val[ntr];
  }
  __syncthreads();
  if (tid < ntr) out[row + (long long)hi_idx[tid] * k] = hi_val[ntr];
}

// ---- matWCorr: one wave per pair (i < j); three passes over the k rows, the weights
// jw = sqrt(w_i w_j) / sum(sqrt(w_i w_j)) recomputed per pass (same rounding each time).
__global__ __launch_bounds__(256) void k_matwcorr(const double* __restrict__ m, const double* __restrict__ w, int k,
                                                  int n, long long npairs, double* __restrict__ out) {
  const long long q = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= npairs) return;
  const int lane = threadIdx.x & 63;
  int i, j;
  tri_pair(q, n, i, j);
  const double* mi = m + (long long)i * k;
  const double* mj = m + (long long)j * k;
  const double* wi = w + (long long)i * k;
  const double* wj = w + (long long)j * k;
  double s = 0;
  for (int r = lane; r < k; r += 64) s += sqrt(wi[r] * wj[r]);
  s = wsum(s);
  double di = 0, dj = 0;
  for (int r = lane; r < k; r += 64) {
    const double jw = sqrt(wi[r] * wj[r]) / s;
    di += mi[r] * jw;
    dj += mj[r] * jw;
  }
  di = wsum(di);
  dj = wsum(dj);
  double nm = 0, ni = 0, nj = 0;
  for (int r = lane; r < k; r += 64) {
    const double jw = sqrt(wi[r] * wj[r]) / s;
    const double a = mi[r] - di, b = mj[r] - dj;
    nm += (a * b) * jw;
    ni += (a * a) * jw;
    nj += (b * b) * jw;
  }
  nm = wsum(nm);
  ni = wsum(ni);
  nj = wsum(nj);
  if (lane == 0) out[j + (long long)i * n] = nm / sqrt(ni * nj);
}

__global__ void k_eye(double* __restrict__ out, int n) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)n * n) return;
  const long long i = e / n, j = e % n;
  if (i == j) out[e] = 1.0;
  else if (j < i) out[e] = 0.0;  // upper triangle (column-major: row j < column i)
}

// ---- matCorr: per column sum and Armadillo's corrected two-pass sd (wave per column)
__global__ __launch_bounds__(256) void k_colstats(const double* __restrict__ x, int k, int ncol,
                                                  double* __restrict__ sum, double* __restrict__ sd) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncol) return;
  const int lane = threadIdx.x & 63;
  const double* xc = x + (long long)c * k;
  double s = 0;
  for (int r = lane; r < k; r += 64) s += xc[r];
  s = wsum(s);
  double var = 0;
  if (k >= 2) {
    const double mean = s / k;
    double a2 = 0, a3 = 0;
    for (int r = lane; r < k; r += 64) {
      const double t = mean - xc[r];
      a2 += t * t;
      a3 += t;
    }
    a2 = wsum(a2);
    a3 = wsum(a3);
    var = (a2 - a3 * a3 / k) / (k - 1);
  }
  if (lane == 0) {
    sum[c] = s;
    sd[c] = sqrt(var);
  }
}

// out[a, b] = (x_a . y_b - sum(x_a) sum(y_b) / k) / (k - 1) / (sd(x_a) sd(y_b)); wave per output
__global__ __launch_bounds__(256) void k_matcorr(const double* __restrict__ x, const double* __restrict__ y, int k,
                                                 int nx, int ny, const double* __restrict__ sx,
                                                 const double* __restrict__ dx, const double* __restrict__ sy,
                                                 const double* __restrict__ dy, double* __restrict__ out) {
  const long long o = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= (long long)nx * ny) return;
  const int a = (int)(o % nx), b = (int)(o / nx), lane = threadIdx.x & 63;
  const double* xa = x + (long long)a * k;
  const double* yb = y + (long long)b * k;
  double v = 0;
  for (int r = lane; r < k; r += 64) v += xa[r] * yb[r];
  v = wsum(v);
  if (lane == 0) {
    const double norm = k > 1 ? (double)(k - 1) : 1.0;
    v -= (sx[a] * sy[b]) / (double)k;
    v /= norm;
    out[o] = v / (dx[a] * dy[b]);
  }
}

// ---- plSemicompleteCor2: one thread per pair (i < j), the reference's merge join
__global__ __launch_bounds__(256) void k_plcor(int np, const long long* __restrict__ off, const int* __restrict__ idx,
                                               const double* __restrict__ val, long long npairs,
                                               double* __restrict__ r, int* __restrict__ cnt) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npairs) return;
  int i, j;
  tri_pair(q, np, i, j);
  const int* i1 = idx + off[i];
  const double* v1 = val + off[i];
  const int v1s = (int)(off[i + 1] - off[i]);
  const int* i2 = idx + off[j];
  const double* v2 = val + off[j];
  const int v2s = (int)(off[j + 1] - off[j]);
  int sgc = 0, k2 = 0;
  double l12 = 0, l11 = 0, l22 = 0;
  for (int k1 = 0; k1 < v1s && v2s > 0; ++k1) {
    const int id = i2[k2] - i1[k1];
    if (id == 0) {
      ++sgc;
      l12 += v2[k2] * v1[k1];
      l11 += v2[k2] * v2[k2];
      l22 += v1[k1] * v1[k1];
    } else if (id < 0) {
      do {
        ++k2;
      } while (k2 < v2s && i2[k2] < i1[k1]);
      if (k2 == v2s) break;
      if (i2[k2] == i1[k1]) {
        ++sgc;
        l12 += v2[k2] * v1[k1];
        l11 += v2[k2] * v2[k2];
        l22 += v1[k1] * v1[k1];
      }
    }
  }
  double cv = l11 * l22;
  if (cv > 0) cv = l12 / sqrt(cv);
  r[i + (long long)j * np] = cv;
  r[j + (long long)i * np] = cv;
  const int u = v1s + v2s - sgc;
  cnt[i + (long long)j * np] = u;
  cnt[j + (long long)i * np] = u;
}

__global__ void k_pl_diag(int np, double* __restrict__ r, int* __restrict__ cnt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  r[i + (long long)i * np] = 1.0;
  cnt[i + (long long)i * np] = 0;
}

// ------------------------------------------------------------------ launchers
// ---- pagoda.varnorm: dataset (or batch) modes from a joint posterior, R/functions.R:1426-1430.
// jp: ngenes x G, element (g, k) at jp[g * jg + k * jk].  mode 1: sum_k jp[g, k] mag[k] in k
// order, multiply then add (R's %*%, a reference-BLAS dgemv column sweep); mode 0: mag at the
// first row maximum (R's max.col breaks ties at random; ties do not occur on posterior rows).
__global__ __launch_bounds__(256) void k_vn_modes(const double* __restrict__ jp, long long jg, long long jk, int ngenes,
                                                  int G, const double* __restrict__ mag, int expected,
                                                  double* __restrict__ modes) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngenes) return;
  const double* row = jp + (long long)g * jg;
  if (expected) {
    double s = 0.0;
    for (int k = 0; k < G; ++k) s = __dadd_rn(s, __dmul_rn(row[(long long)k * jk], mag[k]));
    modes[g] = s;
  } else {
    double bv = row[0];
    int bi = 0;
    for (int k = 1; k < G; ++k) {
      const double v = row[(long long)k * jk];
      if (v > bv) {
        bv = v;
        bi = k;
      }
    }
    modes[g] = mag[bi];
  }
}

// upper Poisson tail P(X >= c), X ~ Poisson(lambda): R's ppois(c - 1, lambda, lower.tail =
// FALSE) = pgamma(lambda, c) (nmath ppois_raw).  c <= 0: 1.  Otherwise the first term
// e^-lambda lambda^c / c! times sum_j lambda^j / ((c+1)...(c+j)), summed until it stops
// changing (lambda <= c: terms fall at least geometrically); for lambda > c the complement of
// the lower sum.
__device__ double pois_upper(int c, double lambda) {
  if (c <= 0) return 1.0;
  if (!(lambda > 0.0)) return lambda == 0.0 ? 0.0 : NAN;
  if (lambda <= (double)c) {
    const double lt = -lambda + c * log(lambda) - lgamma((double)c + 1.0);
    double term = 1.0, s = 1.0;
    for (int j = 1; j < 10000; ++j) {
      term *= lambda / ((double)c + j);
      const double s1 = s + term;
      if (s1 == s) break;
      s = s1;
    }
    return exp(lt) * s;
  }
  double term = exp(-lambda), s = term;  // P(X <= c - 1)
  for (int k = 1; k < c; ++k) {
    term *= lambda / k;
    s += term;
  }
  return 1.0 - s;
}

// matw[g, j] = 1 - mfp[g, j] * sfp[g, j] for the cells j of one call (R/functions.R:1466-1474,
// and the batch columns 1490-1500 with each cell's batch modes): mfp = 1 / (exp(conc.a m (+
// conc.a2 m^2) + conc.b) + 1) at m = log(mode) (scde.failure.probability, 725-748; NaN -> 0),
// sfp = ppois(count - 1, exp(fail.r), lower.tail = FALSE).  models: ncells x 12 col-major.
// modes: per cell j, modes + mode_off[j] (the cell's batch's mode vector).
__global__ __launch_bounds__(256) void k_vn_matw(const int* __restrict__ counts, long long ld, int ngenes,
                                                 const int* __restrict__ cellidx, int ncells,
                                                 const double* __restrict__ models, int mld, int sq,
                                                 const double* __restrict__ modes, const long long* __restrict__ mode_off,
                                                 double* __restrict__ matw) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)ngenes * ncells) return;
  const int g = (int)(i % ngenes), j = (int)(i / ngenes);
  const int c = cellidx[j];
  const double conc_b = models[c], conc_a = models[c + mld], fail_r = models[c + 2LL * mld];
  const double m = log(modes[mode_off[j] + g]);
  double e = __dmul_rn(conc_a, m);
  if (sq) e = __dadd_rn(e, __dmul_rn(models[c + 11LL * mld], __dmul_rn(m, m)));
  double mfp = 1.0 / (exp(__dadd_rn(e, conc_b)) + 1.0);
  if (isnan(mfp)) mfp = 0.0;
  const double sfp = pois_upper(counts[(long long)c * ld + g], exp(fail_r));
  matw[i] = 1.0 - mfp * sfp;
}

hipError_t launch_vn_modes(const double* jp, long long jg, long long jk, int ngenes, int G, const double* mag,
                           int expected, double* modes, hipStream_t st) {
  if (ngenes <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_vn_modes, dim3((ngenes + 255) / 256), dim3(256), 0, st, jp, jg, jk, ngenes, G, mag, expected,
                     modes);
  return hipGetLastError();
}

hipError_t launch_vn_matw(const int* counts, long long ld, int ngenes, const int* cellidx, int ncells,
                          const double* models, int mld, int sq, const double* modes, const long long* mode_off,
                          double* matw, hipStream_t st) {
  const long long n = (long long)ngenes * ncells;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_vn_matw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, counts, ld, ngenes, cellidx,
                     ncells, models, mld, sq, modes, mode_off, matw);
  return hipGetLastError();
}

hipError_t launch_winsorize(const double* m, int k, int n, int ntr, double* out, hipStream_t st) {
  int NP = 1;
  while (NP < n) NP <<= 1;
  if (NP <= 8192) {
    const size_t lds = (size_t)NP * (sizeof(double) + sizeof(int));
    hipError_t e = hipFuncSetAttribute((const void*)k_winsorize_sort, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    const int per = (k + 7) / 8;
    hipLaunchKernelGGL(k_winsorize_sort, dim3(8 * per), dim3(NP >= 1024 ? 1024 : (NP < 64 ? 64 : NP)), lds, st, m,
                       k, n, NP, ntr, out);
    return hipGetLastError();
  }
  if (ntr > 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_winsorize_select, dim3(k), dim3(256), 0, st, m, k, n, ntr, out);
  return hipGetLastError();
}

hipError_t launch_matwcorr(const double* m, const double* w, int k, int n, double* out, hipStream_t st) {
  const long long nn = (long long)n * n;
  hipLaunchKernelGGL(k_eye, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st, out, n);
  const long long np = (long long)n * (n - 1) / 2;
  if (np > 0) hipLaunchKernelGGL(k_matwcorr, dim3((unsigned)((np + 3) / 4)), dim3(256), 0, st, m, w, k, n, np, out);
  return hipGetLastError();
}

hipError_t launch_matcorr(const double* x, int k, int nx, const double* y, int ny, double* stats, double* out,
                          hipStream_t st) {
  double* sx = stats;
  double* dx = stats + nx;
  double* sy = stats + 2 * nx;
  double* dy = stats + 2 * nx + ny;
  if (nx > 0) hipLaunchKernelGGL(k_colstats, dim3((nx + 3) / 4), dim3(256), 0, st, x, k, nx, sx, dx);
  if (ny > 0) hipLaunchKernelGGL(k_colstats, dim3((ny + 3) / 4), dim3(256), 0, st, y, k, ny, sy, dy);
  const long long no = (long long)nx * ny;
  if (no > 0)
    hipLaunchKernelGGL(k_matcorr, dim3((unsigned)((no + 3) / 4)), dim3(256), 0, st, x, y, k, nx, ny, sx, dx, sy, dy,
                       out);
  return hipGetLastError();
}

hipError_t launch_plcor(int np, const long long* off, const int* idx, const double* val, double* r, int* cnt,
                        hipStream_t st) {
  if (np > 0) hipLaunchKernelGGL(k_pl_diag, dim3((np + 255) / 256), dim3(256), 0, st, np, r, cnt);
  const long long npairs = (long long)np * (np - 1) / 2;
  if (npairs > 0)
    hipLaunchKernelGGL(k_plcor, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, np, off, idx, val, npairs,
                       r, cnt);
  return hipGetLastError();
}

}  // namespace scde
