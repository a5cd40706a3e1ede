// wpca.hip -- Bailey's EM weighted PCA (scde's bwpca / pagoda.pathway.wPCA secondary
// path) for gfx950: a batch of independent problems, each a column subset (a gene set)
// of one resident cells x genes matrix pair (values M, weights W).
//
// Reference: src/bwpca.cpp:59-182 (baileyWPCA), 186-322 (baileyWPCAround).
//
// One workgroup per (problem, random start) runs the whole EM loop (<= em.maxiter
// iterations) on chip:
//   * E (d x K eigenvectors) and the working coefficients C (n x K) live in LDS
//     (C in a global scratch row when it does not fit);
//   * pass B (eigenvectors): one wave per gene, lanes over cells, coalesced 8-byte loads
//     of the gene's value/weight columns, the per-gene moments reduced across lanes;
//   * pass AR (coefficients + model fit, fused): one thread per cell, loop over the
//     problem's genes (column index a scalar load), E_g broadcast from LDS; the
//     npcs x npcs normal equations solved per cell in registers (partial-pivot LU).
//     The fit of iteration i (old C, new E) and the coefficients of iteration i+1 (new E)
//     read the same elements, so they share one pass.
// A second kernel picks the best start (the reference's sequential rule) and computes
// var / totvar / scoreweights / the component column means in one pass.
//
// Numerics: FP64, -ffp-contract=off.  Deviations from the reference's arithmetic are
// rounding-order only: per-element residuals as w*(model-m)^2 (the reference squares
// (model-m)*sqrt(w)), sums reduced in a fixed tree order, the eigenvector numerators
// from moments (P_k - sum_{k'<k} Q_kk' E_k', algebraically the reference's deflated
// sum(dat % cw)).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace scde {
namespace {

constexpr int kWB = 256;  // block size: 4 waves

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

// Fixed-order block sum over 4 waves; every thread gets the total.  red: >= 4 doubles.
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ double block_max_d(double v, double* red) {
  v = wave_max_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

__device__ __forceinline__ double dlapy2(double x, double y) {
  const double xa = fabs(x), ya = fabs(y), w = fmax(xa, ya), z = fmin(xa, ya);
  if (z == 0) return w;
  return w * sqrt(1 + (z / w) * (z / w));
}

// Block-wide Householder QR of E (d x K, E[g*K+k]) -> its economical Q (LAPACK
// dgeqr2 + dorg2r, as Armadillo's qr_econ; src/bwpca.cpp:199).  tau: K doubles of LDS.
template <int K>
__device__ void block_qr(double* E, int d, double* tau, double* red) {
  const int tid = threadIdx.x;
  for (int i = 0; i < K; ++i) {
    double mx = 0;
    for (int g = i + 1 + tid; g < d; g += kWB) mx = fmax(mx, fabs(E[g * K + i]));
    mx = block_max_d(mx, red);
    double ss = 0;
    if (mx > 0)
      for (int g = i + 1 + tid; g < d; g += kWB) {
        const double t = E[g * K + i] / mx;
        ss += t * t;
      }
    ss = block_sum_d(ss, red);
    const double xnorm = mx * sqrt(ss);
    const double alpha = E[i * K + i];
    double t = 0;
    __syncthreads();
    if (d - i > 1 && xnorm != 0) {
      const double beta = -copysign(dlapy2(alpha, xnorm), alpha);
      t = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
      for (int g = i + 1 + tid; g < d; g += kWB) E[g * K + i] *= sc;
      if (tid == 0) E[i * K + i] = beta;
    }
    if (tid == 0) tau[i] = t;
    __syncthreads();
    // H(i) applied to columns i+1..K-1 (v = [1, E[i+1.., i]])
    for (int jj = i + 1; jj < K; ++jj) {
      double w = 0;
      for (int g = i + tid; g < d; g += kWB) w += E[g * K + jj] * (g == i ? 1.0 : E[g * K + i]);
      w = block_sum_d(w, red);
      const double tw = -t * w;
      if (t != 0)
        for (int g = i + tid; g < d; g += kWB) E[g * K + jj] += (g == i ? 1.0 : E[g * K + i]) * tw;
      __syncthreads();
    }
  }
  for (int i = K - 1; i >= 0; --i) {
    const double t = tau[i];
    for (int jj = i + 1; jj < K; ++jj) {
      double w = 0;
      for (int g = i + tid; g < d; g += kWB) w += E[g * K + jj] * (g == i ? 1.0 : E[g * K + i]);
      w = block_sum_d(w, red);
      const double tw = -t * w;
      if (t != 0)
        for (int g = i + tid; g < d; g += kWB) E[g * K + jj] += (g == i ? 1.0 : E[g * K + i]) * tw;
      __syncthreads();
    }
    for (int g = tid; g < d; g += kWB) {
      if (g > i) E[g * K + i] *= -t;
      else if (g == i) E[g * K + i] = 1 - t;
      else E[g * K + i] = 0;
    }
    __syncthreads();
  }
}

// solve(A, b) for the K x K normal equations (dgetrf partial pivoting with the
// reciprocal-scaled column, dgetrs).  A zero pivot -> 0 (the minimum-norm answer when
// the cell has no weight in the problem).
template <int K>
__device__ __forceinline__ void solve_small(double (&A)[K][K], double (&b)[K]) {
  if constexpr (K == 1) {
    b[0] = A[0][0] == 0 ? 0.0 : b[0] / A[0][0];
    return;
  } else {
    int piv[K];
    bool sing = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      int p = j;
      double mx = fabs(A[j][j]);
#pragma unroll
      for (int i = j + 1; i < K; ++i) {
        const double a = fabs(A[i][j]);
        if (a > mx) {
          mx = a;
          p = i;
        }
      }
      piv[j] = p;
#pragma unroll
      for (int i = j + 1; i < K; ++i)
        if (p == i) {
#pragma unroll
          for (int l = 0; l < K; ++l) {
            const double t = A[j][l];
            A[j][l] = A[i][l];
            A[i][l] = t;
          }
        }
      sing |= (A[j][j] == 0);
      const double r = 1.0 / A[j][j];
#pragma unroll
      for (int i = j + 1; i < K; ++i) A[i][j] *= r;
#pragma unroll
      for (int l = j + 1; l < K; ++l)
#pragma unroll
        for (int i = j + 1; i < K; ++i) A[i][l] -= A[i][j] * A[j][l];
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int i = j + 1; i < K; ++i)
        if (piv[j] == i) {
          const double t = b[j];
          b[j] = b[i];
          b[i] = t;
        }
#pragma unroll
    for (int l = 0; l < K; ++l)
#pragma unroll
      for (int i = l + 1; i < K; ++i) b[i] -= b[l] * A[i][l];
#pragma unroll
    for (int l = K - 1; l >= 0; --l) {
      b[l] /= A[l][l];
#pragma unroll
      for (int i = 0; i < l; ++i) b[i] -= b[l] * A[i][l];
    }
    if (sing)
#pragma unroll
      for (int i = 0; i < K; ++i) b[i] = 0;
  }
}

struct ProbView {
  int d, ns;
  const int* cols;
  const int* perm;  // d x n, or null
};

__device__ __forceinline__ long long elem(const ProbView& P, int g, int j, int col, long long ld, int n) {
  const int row = P.perm ? P.perm[(long long)g * n + j] : j;
  return (long long)col * ld + row;
}

// Pass AR: for the cells this thread owns, the fit of the current (old) C against E
// (when FIT) and the new coefficients from E.  Old C rows go to cand (global) for the
// best-model bookkeeping.  Returns this thread's residual partial.
template <int K, bool FIT>
__device__ double pass_ar(const ProbView& P, const double* __restrict__ M, const double* __restrict__ Wm,
                          long long ld, int n, const double* E, double* C, double* cand) {
  double res = 0;
  for (int j = threadIdx.x; j < n; j += kWB) {
    double A[K][K], b[K], c0[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      b[k] = 0;
      c0[k] = FIT ? C[(long long)j * K + k] : 0.0;
#pragma unroll
      for (int l = 0; l < K; ++l) A[k][l] = 0;
    }
    double r = 0;
    int g = 0;
    // 4 genes per step: 8 loads in flight per thread
    for (; g + 4 <= P.d; g += 4) {
      double mv[4], wv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int col = P.cols[g + u];
        const long long e = elem(P, g + u, j, col, ld, n);
        mv[u] = M[e];
        wv[u] = Wm[e];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double* Eg = E + (g + u) * K;
        double eg[K];
#pragma unroll
        for (int k = 0; k < K; ++k) eg[k] = Eg[k];
        if (FIT) {
          double mo = 0;
#pragma unroll
          for (int k = 0; k < K; ++k) mo += c0[k] * eg[k];
          const double dl = mo - mv[u];
          r += (dl * dl) * wv[u];
        }
        const double mw = mv[u] * wv[u];
#pragma unroll
        for (int k = 0; k < K; ++k) b[k] += mw * eg[k];
#pragma unroll
        for (int l = 0; l < K; ++l) {
          const double el = eg[l] * wv[u];
#pragma unroll
          for (int k = 0; k < K; ++k) A[k][l] += eg[k] * el;
        }
      }
    }
    for (; g < P.d; ++g) {
      const int col = P.cols[g];
      const long long e = elem(P, g, j, col, ld, n);
      const double mv = M[e], wv = Wm[e];
      double eg[K];
#pragma unroll
      for (int k = 0; k < K; ++k) eg[k] = E[g * K + k];
      if (FIT) {
        double mo = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) mo += c0[k] * eg[k];
        const double dl = mo - mv;
        r += (dl * dl) * wv;
      }
      const double mw = mv * wv;
#pragma unroll
      for (int k = 0; k < K; ++k) b[k] += mw * eg[k];
#pragma unroll
      for (int l = 0; l < K; ++l) {
        const double el = eg[l] * wv;
#pragma unroll
        for (int k = 0; k < K; ++k) A[k][l] += eg[k] * el;
      }
    }
    solve_small<K>(A, b);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (FIT) cand[(long long)j * K + k] = c0[k];
      C[(long long)j * K + k] = b[k];
    }
    res += r;
  }
  return res;
}

}  // namespace

// One block per (problem, start) entry of `blocks` (problem -1: padding).
template <int K, bool CL>
__global__ __launch_bounds__(kWB) void k_wpca_em(const double* __restrict__ M, const double* __restrict__ Wm,
                                                 long long ld, int n, const WpcaProb* __restrict__ probs,
                                                 const int2* __restrict__ blocks, const int* __restrict__ cols,
                                                 const int* __restrict__ perms, const double* __restrict__ starts,
                                                 int maxiter, double tol, const double* __restrict__ smoothc, int L,
                                                 double* __restrict__ scratch, double* __restrict__ stat) {
  extern __shared__ double lds[];
  __shared__ double red[8];
  __shared__ double tau[K];
  constexpr int NM = K + K * (K + 1) / 2;
  const int2 bs = blocks[blockIdx.x];
  if (bs.x < 0) return;
  const WpcaProb Pr = probs[bs.x];
  const int s = bs.y, d = Pr.d, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  ProbView P{d, Pr.nstarts, cols + Pr.col_off, Pr.perm_off >= 0 ? perms + Pr.perm_off : nullptr};
  double* E = lds;
  double* bestE = scratch + Pr.sE_off + (long long)s * d * K;
  double* cslot[2] = {scratch + Pr.sC_off + (long long)s * 2 * n * K,
                      scratch + Pr.sC_off + (long long)s * 2 * n * K + (long long)n * K};
  double* C = CL ? lds + (long long)d * K : scratch + Pr.sW_off + (long long)s * n * K;
  double* mom = scratch + Pr.mom_off + (long long)s * d * (NM + 1);
  double* raw = mom + (long long)d * NM;
  // random start: randu(d, K) (column-major uniforms) -> orthonormal Q
  const double* X = starts + Pr.start_off + (long long)s * d * K;
  for (int e = tid; e < d * K; e += kWB) {
    const int g = e % d, k = e / d;
    E[g * K + k] = X[e];
  }
  __syncthreads();
  block_qr<K>(E, d, tau, red);
  // coefficients for the start (iteration 0's first step)
  (void)pass_ar<K, false>(P, M, Wm, ld, n, E, C, nullptr);
  __syncthreads();
  double pres = DBL_MAX, bpres = DBL_MAX;
  int ii = 0, best = -1, cur = 0;
  while (ii < maxiter) {
    // ---- pass B: per-gene moments  P_k = sum_j (w c_k) m,  Q_kk' = sum_j (w c_k) c_k'
    for (int g = wid; g < d; g += kWB / 64) {
      double acc[NM];
#pragma unroll
      for (int q = 0; q < NM; ++q) acc[q] = 0;
      const int col = P.cols[g];
      for (int j = lane; j < n; j += 64) {
        const long long e = elem(P, g, j, col, ld, n);
        const double mv = M[e], wv = Wm[e];
        double c[K];
#pragma unroll
        for (int k = 0; k < K; ++k) c[k] = C[(long long)j * K + k];
        int q = K;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const double t = wv * c[k];
          acc[k] += mv * t;
#pragma unroll
          for (int l = 0; l <= k; ++l) acc[q++] += t * c[l];
        }
      }
#pragma unroll
      for (int q = 0; q < NM; ++q) acc[q] = wave_sum_d(acc[q]);
      if (lane == 0)
#pragma unroll
        for (int q = 0; q < NM; ++q) mom[(long long)g * NM + q] = acc[q];
    }
    __syncthreads();
    // ---- new eigenvectors, column by column (deflation by the earlier, smoothed columns)
    for (int k = 0; k < K; ++k) {
      // Q index of (k, l): K + k(k+1)/2 + l
      for (int g = tid; g < d; g += kWB) {
        const double* mg = mom + (long long)g * NM;
        double num = mg[k];
#pragma unroll
        for (int l = 0; l < K; ++l)
          if (l < k) num -= mg[K + k * (k + 1) / 2 + l] * E[g * K + l];
        const double v = num / mg[K + k * (k + 1) / 2 + k];
        if (L > 0) raw[g] = v;
        else E[g * K + k] = v;
      }
      if (L > 0) {  // conv(eigenv.col(k), smoothc) trimmed to d (src/bwpca.cpp:253-259)
        __syncthreads();
        const int np = (L - 1) / 2;
        for (int g = tid; g < d; g += kWB) {
          double sacc = 0;
          const int i = g + np;
          const int t0 = i - (L - 1) > 0 ? i - (L - 1) : 0, t1 = i < d - 1 ? i : d - 1;
          for (int t = t0; t <= t1; ++t) sacc += raw[t] * smoothc[i - t];
          E[g * K + k] = sacc;
        }
      }
      __syncthreads();
    }
    // ---- renormalise / re-orthogonalise (src/bwpca.cpp:270-277)
    for (int k = 0; k < K; ++k) {
      for (int kx = 0; kx < k; ++kx) {
        double p = 0;
        for (int g = tid; g < d; g += kWB) p += E[g * K + k] * E[g * K + kx];
        const double c = block_sum_d(p, red);
        for (int g = tid; g < d; g += kWB) E[g * K + k] -= c * E[g * K + kx];
        __syncthreads();
      }
      double p = 0;
      for (int g = tid; g < d; g += kWB) p += E[g * K + k] * E[g * K + k];
      const double nr = sqrt(block_sum_d(p, red));
      for (int g = tid; g < d; g += kWB) E[g * K + k] /= nr;
      __syncthreads();
    }
    // ---- model fit of (C, E) fused with the next coefficients
    double* cand = cslot[cur];
    const double npres = block_sum_d(pass_ar<K, true>(P, M, Wm, ld, n, E, C, cand), red);
    if (npres < bpres) {
      bpres = npres;
      best = cur;
      cur ^= 1;
      for (int e = tid; e < d * K; e += kWB) bestE[e] = E[e];
    }
    if (tol > 0 && ii > 0 && (pres - npres) / npres < tol && pres > npres) {
      pres = npres;
      break;
    }
    ++ii;
    pres = npres;
    __syncthreads();
  }
  if (tid == 0) {
    double* st = stat + (Pr.stat_off + s) * 4;
    st[0] = pres;
    st[1] = bpres;
    st[2] = (double)ii;
    st[3] = (double)best;
  }
}

// One block per problem: the best start (src/bwpca.cpp:312-319), rotation / scores
// out, and one pass for var, totvar, scoreweights, colmeans, the PC1-only residual.
template <int K>
__global__ __launch_bounds__(kWB) void k_wpca_final(const double* __restrict__ M, const double* __restrict__ Wm,
                                                    long long ld, int n, const WpcaProb* __restrict__ probs,
                                                    const int* __restrict__ kidx, const int* __restrict__ cols,
                                                    const int* __restrict__ perms,
                                                    const double* __restrict__ scratch,
                                                    const double* __restrict__ stat, double* __restrict__ out) {
  __shared__ double red[8];
  __shared__ int chosen_s;
  __shared__ int chosen_slot;
  const int p = kidx[blockIdx.x];
  const WpcaProb Pr = probs[p];
  const int d = Pr.d, tid = threadIdx.x;
  ProbView P{d, Pr.nstarts, cols + Pr.col_off, Pr.perm_off >= 0 ? perms + Pr.perm_off : nullptr};
  if (tid == 0) {
    double bestpres = -1;
    int cs = 0;
    for (int s = 0; s < Pr.nstarts; ++s) {
      const double* st = stat + (Pr.stat_off + s) * 4;
      if (s == 0 || st[0] < bestpres) {
        bestpres = st[1];
        cs = s;
      }
    }
    chosen_s = cs;
    chosen_slot = (int)stat[(Pr.stat_off + cs) * 4 + 3];
  }
  __syncthreads();
  const int s = chosen_s;
  const double* E = scratch + Pr.sE_off + (long long)s * d * K;
  const double* C = scratch + Pr.sC_off + (long long)s * 2 * n * K + (long long)(chosen_slot < 0 ? 0 : chosen_slot) * n * K;
  double* rot = out + Pr.out_rot;
  double* sco = out + Pr.out_sc;
  double* pcw = out + Pr.out_pcw;
  double* cmn = out + Pr.out_cm;
  double* sv = out + Pr.out_var;  // var[K], totvar, npres0
  for (int e = tid; e < d * K; e += kWB) rot[(e % K) * d + e / K] = E[e];  // column-major d x K
  double np[K], tot = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) np[k] = 0;
  for (int j = tid; j < n; j += kWB) {
    double c[K], pw[K], cm[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      c[k] = C[(long long)j * K + k];
      pw[k] = 0;
      cm[k] = 0;
      sco[(long long)k * n + j] = c[k];
    }
    for (int g = 0; g < d; ++g) {
      const int col = P.cols[g];
      const long long e = elem(P, g, j, col, ld, n);
      const double mv = M[e], wv = Wm[e];
      tot += (mv * mv) * wv;
      double dat = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double ek = E[g * K + k];
        dat += c[k] * ek;
        const double dl = dat - mv;
        np[k] += (dl * dl) * wv;
        pw[k] += wv * fabs(ek);
        cm[k] += mv * fabs(ek);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      pcw[(long long)k * n + j] = pw[k];
      cmn[(long long)k * n + j] = cm[k] / d;
    }
  }
  tot = block_sum_d(tot, red);
#pragma unroll
  for (int k = 0; k < K; ++k) np[k] = block_sum_d(np[k], red);
  if (tid == 0) {
    double tvarexp = 0;
    for (int k = 0; k < K; ++k) {
      sv[k] = tot - np[k] - tvarexp;
      tvarexp = tot - np[k];
    }
    sv[K] = tot;
    sv[K + 1] = np[0];
  }
}

// ------------------------------------------------------------------ launchers
namespace {
template <int K>
hipError_t launch_em_k(const WpcaLaunch& a, int nblocks, hipStream_t st) {
  const size_t need = (size_t)(a.dmax + a.n) * K * sizeof(double);
  if (need <= (size_t)a.lds_cap) {
    auto fn = k_wpca_em<K, true>;
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(nblocks), dim3(kWB), need, st, a.M, a.W, a.ld, a.n, a.probs, a.blocks, a.cols,
                       a.perms, a.starts, a.maxiter, a.tol, a.smoothc, a.L, a.scratch, a.stat);
  } else {
    const size_t ne = (size_t)a.dmax * K * sizeof(double);
    auto fn = k_wpca_em<K, false>;
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ne);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(nblocks), dim3(kWB), ne, st, a.M, a.W, a.ld, a.n, a.probs, a.blocks, a.cols,
                       a.perms, a.starts, a.maxiter, a.tol, a.smoothc, a.L, a.scratch, a.stat);
  }
  return hipGetLastError();
}
template <int K>
hipError_t launch_final_k(const WpcaLaunch& a, const int* kidx, int nprob, hipStream_t st) {
  hipLaunchKernelGGL(k_wpca_final<K>, dim3(nprob), dim3(kWB), 0, st, a.M, a.W, a.ld, a.n, a.probs, kidx, a.cols,
                     a.perms, a.scratch, a.stat, a.out);
  return hipGetLastError();
}
}  // namespace

int wpca_max_k() { return kWpcaMaxK; }

hipError_t launch_wpca_em(int K, const WpcaLaunch& a, int nblocks, hipStream_t st) {
  switch (K) {
    case 1: return launch_em_k<1>(a, nblocks, st);
    case 2: return launch_em_k<2>(a, nblocks, st);
    case 3: return launch_em_k<3>(a, nblocks, st);
    case 4: return launch_em_k<4>(a, nblocks, st);
    case 5: return launch_em_k<5>(a, nblocks, st);
    case 6: return launch_em_k<6>(a, nblocks, st);
    case 7: return launch_em_k<7>(a, nblocks, st);
    case 8: return launch_em_k<8>(a, nblocks, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_wpca_final(int K, const WpcaLaunch& a, const int* kidx, int nprob, hipStream_t st) {
  switch (K) {
    case 1: return launch_final_k<1>(a, kidx, nprob, st);
    case 2: return launch_final_k<2>(a, kidx, nprob, st);
    case 3: return launch_final_k<3>(a, kidx, nprob, st);
    case 4: return launch_final_k<4>(a, kidx, nprob, st);
    case 5: return launch_final_k<5>(a, kidx, nprob, st);
    case 6: return launch_final_k<6>(a, kidx, nprob, st);
    case 7: return launch_final_k<7>(a, kidx, nprob, st);
    case 8: return launch_final_k<8>(a, kidx, nprob, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace scde
