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

constexpr int kWB = SCDE_WPCA_BLOCK;  // block size (waves = kWB / 64)
constexpr int kNW = kWB / 64;

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

// Fixed-order block sum over NW waves; every thread gets the total.  red: NW doubles.
template <int NW = kNW>
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) t += red[w];
  return t;
}
template <int NW = kNW>
__device__ __forceinline__ double block_max_d(double v, double* red) {
  v = wave_max_d(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) t = fmax(t, red[w]);
  return t;
}

__device__ __forceinline__ double dlapy2(double x, double y) {
  const double xa = fabs(x), ya = fabs(y), w = fmax(xa, ya), z = fmin(xa, ya);
  if (z == 0) return w;
  return w * sqrt(1 + (z / w) * (z / w));
}

// Block-wide Householder QR of E (d x K, E[g*ldg+k]) -> its economical Q (LAPACK
// dgeqr2 + dorg2r, as Armadillo's qr_econ; src/bwpca.cpp:199).  tau: K doubles of LDS.
template <int K, int NT = kWB>
__device__ void block_qr(double* E, int d, int ldg, double* tau, double* red) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x;
  for (int i = 0; i < K; ++i) {
    double mx = 0;
    for (int g = i + 1 + tid; g < d; g += NT) mx = fmax(mx, fabs(E[g * ldg + i]));
    mx = block_max_d<NW>(mx, red);
    double ss = 0;
    if (mx > 0)
      for (int g = i + 1 + tid; g < d; g += NT) {
        const double t = E[g * ldg + i] / mx;
        ss += t * t;
      }
    ss = block_sum_d<NW>(ss, red);
    const double xnorm = mx * sqrt(ss);
    const double alpha = E[i * ldg + i];
    double t = 0;
    __syncthreads();
    if (d - i > 1 && xnorm != 0) {
      const double beta = -copysign(dlapy2(alpha, xnorm), alpha);
      t = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
      for (int g = i + 1 + tid; g < d; g += NT) E[g * ldg + i] *= sc;
      if (tid == 0) E[i * ldg + i] = beta;
    }
    if (tid == 0) tau[i] = t;
    __syncthreads();
    // H(i) applied to columns i+1..K-1 (v = [1, E[i+1.., i]])
    for (int jj = i + 1; jj < K; ++jj) {
      double w = 0;
      for (int g = i + tid; g < d; g += NT) w += E[g * ldg + jj] * (g == i ? 1.0 : E[g * ldg + i]);
      w = block_sum_d<NW>(w, red);
      const double tw = -t * w;
      if (t != 0)
        for (int g = i + tid; g < d; g += NT) E[g * ldg + jj] += (g == i ? 1.0 : E[g * ldg + i]) * tw;
      __syncthreads();
    }
  }
  for (int i = K - 1; i >= 0; --i) {
    const double t = tau[i];
    for (int jj = i + 1; jj < K; ++jj) {
      double w = 0;
      for (int g = i + tid; g < d; g += NT) w += E[g * ldg + jj] * (g == i ? 1.0 : E[g * ldg + i]);
      w = block_sum_d<NW>(w, red);
      const double tw = -t * w;
      if (t != 0)
        for (int g = i + tid; g < d; g += NT) E[g * ldg + jj] += (g == i ? 1.0 : E[g * ldg + i]) * tw;
      __syncthreads();
    }
    for (int g = tid; g < d; g += NT) {
      if (g > i) E[g * ldg + i] *= -t;
      else if (g == i) E[g * ldg + i] = 1 - t;
      else E[g * ldg + i] = 0;
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
  __shared__ double red[kNW];
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
  block_qr<K>(E, d, K, tau, red);
  // coefficients for the start (iteration 0's first step)
  (void)pass_ar<K, false>(P, M, Wm, ld, n, E, C, nullptr);
  __syncthreads();
  double pres = DBL_MAX, bpres = DBL_MAX;
  int ii = 0, best = -1, cur = 0;
  while (ii < maxiter) {
    // ---- pass B: per-gene moments  P_k = sum_j (w c_k) m,  Q_kk' = sum_j (w c_k) c_k'
    for (int g = wid; g < d; g += kNW) {
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
  __shared__ double red[kNW];
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

// ---- multi-start EM for npcs = 1 (pagoda's random gene sets; most of its EM work) ----
// One workgroup of 1024 threads runs SG = 5 starts of one problem together, so every
// value / weight element loaded serves 5 starts.  Thread t owns cells t + r * 1024
// (r < R) in both passes, with the 5 coefficients of each owned cell in registers:
//   * pass AR: loop over genes, E_g for the 5 starts broadcast from LDS;
//   * pass B: per gene, each thread's partial moments (P_s, Q_s over its cells) are
//     reduce-scattered across the wave on VALU (permlane swaps + DPP), the 16 waves'
//     partials combined in LDS in a fixed order, 16 genes per barrier.
// All 5 starts are computed until the last one stops; the finished ones' results are
// discarded (their best model is already saved).
constexpr int kMsNT = 1024, kMsNW = 16, kMsSG = 5, kMsGCH = 16;
#ifndef SCDE_WPCA_PREFETCH
#define SCDE_WPCA_PREFETCH 1  // k_wpca_ms1: the next gene's M / W loads issued ahead of the current gene's arithmetic
#endif

__device__ __forceinline__ void swap32d(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false,
                                                   false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false,
                                                   false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16d(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false,
                                                   false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false,
                                                   false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}

// Sum reduce-scatter of 16 values over the wave: lane l ends with the wave total of
// value (l >> 2) & 15.  Stages pair lanes by bit 5, 4 (permlane swaps), 3 (row mirror,
// lane ^ 15), 2 (half mirror, lane ^ 7), then 1, 0 (quad perms).
__device__ __forceinline__ double rs16_sum(double (&v)[16], int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    swap32d(v[j], v[j + 8]);
    v[j] = v[j] + v[j + 8];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    swap16d(v[j], v[j + 4]);
    v[j] = v[j] + v[j + 4];
  }
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const double lo = v[j], hi = v[j + 2];
      v[j] = (up ? hi : lo) + dppd<0x140>(up ? lo : hi);
    }
  }
  {
    const bool up = (lane & 4) != 0;
    const double lo = v[0], hi = v[1];
    v[0] = (up ? hi : lo) + dppd<0x141>(up ? lo : hi);
  }
  double x = v[0];
  x = x + dppd<0x4E>(x);
  x = x + dppd<0xB1>(x);
  return x;
}

template <int NW, int V>
__device__ __forceinline__ void block_sum_vec(double (&v)[V], double* red) {
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = wave_sum_d(v[i]);
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int i = 0; i < V; ++i) red[(threadIdx.x >> 6) * V + i] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < V; ++i) {
    double t = red[i];
#pragma unroll
    for (int w = 1; w < NW; ++w) t += red[w * V + i];
    v[i] = t;
  }
}

// pass AR for the SG starts: fit of the old coefficients against E (FIT) and the new ones
template <int R, bool FIT>
__device__ __forceinline__ void ms_pass_ar(const ProbView& P, const double* __restrict__ M,
                                           const double* __restrict__ Wm, long long ld, int n, const double* E,
                                           double (&c)[R][kMsSG], double (&racc)[kMsSG], double* cbase, int nc,
                                           unsigned amask, unsigned slots) {
  constexpr int SG = kMsSG;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = threadIdx.x + r * kMsNT;
    const bool in = j < n;
    const int jj = in ? j : 0;
    double A[SG], b[SG];
#pragma unroll
    for (int s = 0; s < SG; ++s) A[s] = b[s] = 0;
    int g = 0;
#if SCDE_WPCA_PREFETCH
    // the next gene pair's loads are issued before this pair's arithmetic (the pass streams M and W
    // from HBM; one pair in flight per wave left it waiting on load latency)
    double mvn[2], wvn[2];
    auto load2 = [&](int g2, double (&m)[2], double (&w)[2]) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long e = elem(P, g2 + u, jj, P.cols[g2 + u], ld, n);
        m[u] = in ? M[e] : 0.0;
        w[u] = in ? Wm[e] : 0.0;
      }
    };
    if (P.d >= 2) load2(0, mvn, wvn);
#endif
    for (; g + 2 <= P.d; g += 2) {
      double mv[2], wv[2];
#if SCDE_WPCA_PREFETCH
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        mv[u] = mvn[u];
        wv[u] = wvn[u];
      }
      if (g + 4 <= P.d) load2(g + 2, mvn, wvn);
#else
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long long e = elem(P, g + u, jj, P.cols[g + u], ld, n);
        mv[u] = in ? M[e] : 0.0;
        wv[u] = in ? Wm[e] : 0.0;
      }
#endif
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const double mw = mv[u] * wv[u];
#pragma unroll
        for (int s = 0; s < SG; ++s) {
          const double eg = E[(g + u) * SG + s];
          if (FIT) {
            const double dl = c[r][s] * eg - mv[u];
            racc[s] += (dl * dl) * wv[u];
          }
          b[s] += mw * eg;
          A[s] += eg * (eg * wv[u]);
        }
      }
    }
    for (; g < P.d; ++g) {
      const long long e = elem(P, g, jj, P.cols[g], ld, n);
      const double mv = in ? M[e] : 0.0, wv = in ? Wm[e] : 0.0;
      const double mw = mv * wv;
#pragma unroll
      for (int s = 0; s < SG; ++s) {
        const double eg = E[g * SG + s];
        if (FIT) {
          const double dl = c[r][s] * eg - mv;
          racc[s] += (dl * dl) * wv;
        }
        b[s] += mw * eg;
        A[s] += eg * (eg * wv);
      }
    }
#pragma unroll
    for (int s = 0; s < SG; ++s) {
      if (FIT && in && ((amask >> s) & 1u)) cbase[(long long)(2 * s + ((slots >> s) & 1u)) * nc + j] = c[r][s];
      c[r][s] = A[s] == 0 ? 0.0 : b[s] / A[s];
    }
  }
}

template <int R>
__global__ __launch_bounds__(kMsNT) void k_wpca_ms1(const double* __restrict__ M, const double* __restrict__ Wm,
                                                    long long ld, int n, const WpcaProb* __restrict__ probs,
                                                    const int2* __restrict__ blocks, const int* __restrict__ cols,
                                                    const int* __restrict__ perms, const double* __restrict__ starts,
                                                    int maxiter, double tol, double* __restrict__ scratch,
                                                    double* __restrict__ stat) {
  constexpr int SG = kMsSG, NW = kMsNW, NT = kMsNT, GCH = kMsGCH;
  extern __shared__ double lds[];  // E[g * SG + s]
  __shared__ double part[GCH][NW][2 * SG];
  __shared__ double red[NW * SG];
  __shared__ double tau[1];
  // per-start EM state, kept by thread 0 (the block reads it after a barrier)
  __shared__ double s_pres[SG], s_bpres[SG];
  __shared__ int s_best[SG], s_cur[SG], s_iters[SG], s_impr[SG];
  __shared__ unsigned s_amask;
  const int2 bs = blocks[blockIdx.x];
  if (bs.x < 0) return;
  const WpcaProb Pr = probs[bs.x];
  const int s0 = bs.y, d = Pr.d, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ns = Pr.nstarts - s0 < SG ? Pr.nstarts - s0 : SG;
  ProbView P{d, Pr.nstarts, cols + Pr.col_off, Pr.perm_off >= 0 ? perms + Pr.perm_off : nullptr};
  double* E = lds;
  double* mom = scratch + Pr.mom_off + (long long)s0 * d * 3;  // d x 2 x ns (fits the group's d x 3 x ns)
  double* cbase = scratch + Pr.sC_off + (long long)s0 * 2 * n;  // start s0+s, slot k: + (2 s + k) n
  double* ebase = scratch + Pr.sE_off + (long long)s0 * d;      // start s0+s: + s d
  for (int e = tid; e < d * SG; e += NT) {
    const int g = e / SG, s = e % SG;
    E[e] = s < ns ? starts[Pr.start_off + (long long)(s0 + s) * d + g] : 0.0;
  }
  if (tid < SG) {
    s_pres[tid] = s_bpres[tid] = DBL_MAX;
    s_best[tid] = -1;
    s_cur[tid] = 0;
    s_iters[tid] = 0;
  }
  if (tid == 0) s_amask = (1u << ns) - 1u;
  __syncthreads();
  for (int s = 0; s < ns; ++s) block_qr<1, NT>(E + s, d, SG, tau, red);
  double c[R][SG];
  double racc[SG];
  ms_pass_ar<R, false>(P, M, Wm, ld, n, E, c, racc, nullptr, n, 0u, 0);
  for (int it = 0; it < maxiter; ++it) {
    __syncthreads();
    const unsigned amask = s_amask;
    if (amask == 0u) break;
    // ---- pass B: moments P_s = sum_j (w c_s) m, Q_s = sum_j (w c_s) c_s, 16 genes per barrier
    for (int g0 = 0; g0 < d; g0 += GCH) {
      const int gn = d - g0 < GCH ? d - g0 : GCH;
#if SCDE_WPCA_PREFETCH
      // the next gene's loads are issued before this gene's arithmetic and reduction
      double mvn[R], wvn[R];
      auto load1 = [&](int g1, double (&m)[R], double (&w)[R]) {
        const int col1 = P.cols[g1];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = tid + r * NT;
          const long long e = elem(P, g1, j < n ? j : 0, col1, ld, n);
          m[r] = M[e];
          w[r] = Wm[e];
        }
      };
      load1(g0, mvn, wvn);
#endif
      for (int gi = 0; gi < gn; ++gi) {
        const int g = g0 + gi;
        const int col = P.cols[g];
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = 0;
#if SCDE_WPCA_PREFETCH
        double mvc[R], wvc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          mvc[r] = mvn[r];
          wvc[r] = wvn[r];
        }
        if (gi + 1 < gn) load1(g + 1, mvn, wvn);
#endif
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = tid + r * NT;
          if (j < n) {
#if SCDE_WPCA_PREFETCH
            const double mv = mvc[r], wv = wvc[r];
            (void)col;
#else
            const long long e = elem(P, g, j, col, ld, n);
            const double mv = M[e], wv = Wm[e];
#endif
#pragma unroll
            for (int s = 0; s < SG; ++s) {
              const double t = wv * c[r][s];
              v[s] += mv * t;
              v[SG + s] += t * c[r][s];
            }
          }
        }
        const double x = rs16_sum(v, lane);
        const int q = (lane >> 2) & 15;
        if ((lane & 3) == 0 && q < 2 * SG) part[gi][wid][q] = x;
      }
      __syncthreads();
      if (tid < gn * 2 * SG) {
        const int gi = tid / (2 * SG), q = tid % (2 * SG);
        double t = part[gi][0][q];
#pragma unroll
        for (int w = 1; w < NW; ++w) t += part[gi][w][q];
        const int s = q % SG;
        if (s < ns) mom[(long long)(g0 + gi) * 2 * ns + (q / SG) * ns + s] = t;
      }
      __syncthreads();
    }
    // ---- new eigenvectors E = P / Q, then unit length
    double dots[SG];
#pragma unroll
    for (int s = 0; s < SG; ++s) dots[s] = 0;
    for (int g = tid; g < d; g += NT) {
#pragma unroll
      for (int s = 0; s < SG; ++s) {
        if (s < ns) {
          const double v = mom[(long long)g * 2 * ns + s] / mom[(long long)g * 2 * ns + ns + s];
          E[g * SG + s] = v;
          dots[s] += v * v;
        }
      }
    }
    block_sum_vec<NW, SG>(dots, red);
    for (int g = tid; g < d; g += NT)
#pragma unroll
      for (int s = 0; s < SG; ++s)
        if (s < ns) E[g * SG + s] /= sqrt(dots[s]);
    __syncthreads();
    // ---- fit of (C, E) fused with the next coefficients; old C -> the start's candidate slot
#pragma unroll
    for (int s = 0; s < SG; ++s) racc[s] = 0;
    unsigned slots = 0;
#pragma unroll
    for (int s = 0; s < SG; ++s) slots |= (unsigned)(s_cur[s] & 1) << s;
    ms_pass_ar<R, true>(P, M, Wm, ld, n, E, c, racc, cbase, n, amask, slots);
    block_sum_vec<NW, SG>(racc, red);
    if (tid == 0) {
      unsigned am = amask;
      for (int s = 0; s < SG; ++s) {
        s_impr[s] = 0;
        if ((am >> s) & 1u) {
          const double npres = racc[s];
          if (npres < s_bpres[s]) {
            s_bpres[s] = npres;
            s_best[s] = s_cur[s];
            s_cur[s] ^= 1;
            s_impr[s] = 1;
          }
          if (tol > 0 && it > 0 && (s_pres[s] - npres) / npres < tol && s_pres[s] > npres) {
            s_pres[s] = npres;
            s_iters[s] = it;
            am &= ~(1u << s);
          } else {
            s_pres[s] = npres;
            s_iters[s] = it + 1;
          }
        }
      }
      s_amask = am;
    }
    __syncthreads();
    for (int e = tid; e < d * SG; e += NT) {
      const int g = e / SG, s = e % SG;
      if (s_impr[s]) ebase[(long long)s * d + g] = E[e];
    }
  }
  __syncthreads();
  if (tid < ns) {
    double* st = stat + (Pr.stat_off + s0 + tid) * 4;
    st[0] = s_pres[tid];
    st[1] = s_bpres[tid];
    st[2] = (double)s_iters[tid];
    st[3] = (double)s_best[tid];
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

int wpca_ms_group() { return kMsSG; }

// npcs = 1, no smoothing, ncells <= 4096, E for 5 starts in LDS: the multi-start kernel
bool wpca_ms_ok(int n, int dmax) {
  return n <= 4 * kMsNT && (size_t)dmax * kMsSG * sizeof(double) <= (size_t)96 * 1024;
}

hipError_t launch_wpca_ms(const WpcaLaunch& a, int nblocks, hipStream_t st) {
  const size_t need = (size_t)a.dmax * kMsSG * sizeof(double);
  const int R = (a.n + kMsNT - 1) / kMsNT;
  auto go = [&](auto fn) {
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)need);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(nblocks), dim3(kMsNT), need, st, a.M, a.W, a.ld, a.n, a.probs, a.blocks, a.cols,
                       a.perms, a.starts, a.maxiter, a.tol, a.scratch, a.stat);
    return hipGetLastError();
  };
  switch (R) {
    case 1: return go(k_wpca_ms1<1>);
    case 2: return go(k_wpca_ms1<2>);
    case 3: return go(k_wpca_ms1<3>);
    case 4: return go(k_wpca_ms1<4>);
    default: return hipErrorInvalidValue;
  }
}

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
