// Device BH: cZ = sign(Z) * qnorm(p.adjust(pnorm(|Z|, lower = FALSE), "BH"), lower = FALSE)
// (R/functions.R:5051).  p.adjust(p, "BH") (R stats): NA p-values are dropped and stay NA;
// with lp = #non-NA, i <- lp:1, o <- order(p, decreasing = TRUE), ro <- order(o),
// pmin(1, cummin(lp / i * p[o]))[ro]; lp <= 1 returns p unchanged.
//
//   k_bh_keys   p = pnorm_upper(|z|); NaN -> key -1 (sorts after every p >= 0); count lp
//   radix sort  (p, index) pairs, descending; hipCUB's radix sort is stable, so ties keep
//               index order -- R's order(..., decreasing = TRUE) (radix) does the same
//   k_bh_scale  v_r = (lp / (lp - r)) * p_(r) for the lp valid entries
//   min-scan    cummin
//   k_bh_final  adj = pmin(1, cm) scattered back; cz = sign(z) * qnorm(adj, upper)
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "device_math.h"
#include "kernels.h"

namespace scde {

// R pnorm(x, lower.tail = FALSE) (nmath pnorm.c, Cody's pnorm_both), as scde_bh_cz's host
// code; only x = |Z| >= 0 reaches it.
__device__ inline double pnorm_upper_dev(double x) {
  const double a0 = 2.2352520354606839287, a1 = 161.02823106855587881, a2 = 1067.6894854603709582,
               a3 = 18154.981253343561249, a4 = 0.065682337918207449113;
  const double b0 = 47.20258190468824187, b1 = 976.09855173777669322, b2 = 10260.932208618978205,
               b3 = 45507.789335026729956;
  const double c[9] = {0.39894151208813466764, 8.8831497943883759412, 93.506656132177855979,
                       597.27027639480026226,  2494.5375852903726711, 6848.1904505362823326,
                       11602.651437647350124,  9842.7148383839780218, 1.0765576773720192317e-8};
  const double d[8] = {22.266688044328115691, 235.38790178262499861, 1519.377599407554805,
                       6485.558298266760755,  18615.571640885098091, 34900.952721145977266,
                       38912.003286093271411, 19685.429676859990727};
  const double pp[6] = {0.21589853405795699,     0.1274011611602473639, 0.022235277870649807,
                        0.001421619193227893466, 2.9112874951168792e-5, 0.02307344176494017303};
  const double q[5] = {1.28426009614491121, 0.468238212480865118, 0.0659881378689285515,
                       0.00378239633202758244, 7.29751555083966205e-5};
  const double M_1_SQRT_2PI = 0.398942280401432677939946059934, M_SQRT_32 = 5.656854249492380195206754896838;
  if (isnan(x)) return x;
  const double y = fabs(x);
  double xnum, xden, temp, xsq, del, cum, ccum;
  if (y <= 0.67448975) {
    if (y > 1.1102230246251565e-16) {
      xsq = x * x;
      xnum = a4 * xsq;
      xden = xsq;
      xnum = (xnum + a0) * xsq;
      xden = (xden + b0) * xsq;
      xnum = (xnum + a1) * xsq;
      xden = (xden + b1) * xsq;
      xnum = (xnum + a2) * xsq;
      xden = (xden + b2) * xsq;
    } else {
      xnum = xden = 0.0;
    }
    temp = x * (xnum + a3) / (xden + b3);
    ccum = 0.5 - temp;
  } else if (y <= M_SQRT_32) {
    xnum = c[8] * y;
    xden = y;
    for (int i = 0; i < 7; ++i) {
      xnum = (xnum + c[i]) * y;
      xden = (xden + d[i]) * y;
    }
    temp = (xnum + c[7]) / (xden + d[7]);
    xsq = trunc(y * 16) / 16;
    del = (y - xsq) * (y + xsq);
    cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
    ccum = 1.0 - cum;
    if (x > 0.) ccum = cum;
  } else if (x < 37.5193) {
    xsq = 1.0 / (x * x);
    xnum = pp[5] * xsq;
    xden = xsq;
    for (int i = 0; i < 4; ++i) {
      xnum = (xnum + pp[i]) * xsq;
      xden = (xden + q[i]) * xsq;
    }
    temp = xsq * (xnum + pp[4]) / (xden + q[4]);
    temp = (M_1_SQRT_2PI - temp) / y;
    xsq = trunc(x * 16) / 16;
    del = (x - xsq) * (x + xsq);
    cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
    ccum = cum;  // x > 0 here
  } else {
    ccum = 0.0;
  }
  return ccum;
}

__global__ void k_bh_keys(const double* __restrict__ z, int n, double* __restrict__ key, int* __restrict__ idx,
                          double* __restrict__ p, int* __restrict__ count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool valid = false;
  if (i < n) {
    const double pv = pnorm_upper_dev(fabs(z[i]));
    valid = !isnan(pv);
    p[i] = pv;
    key[i] = valid ? pv : -1.0;
    idx[i] = i;
  }
  const unsigned long long b = __ballot(valid);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, __popcll(b));
}

__global__ void k_bh_scale(const double* __restrict__ skey, int n, const int* __restrict__ count,
                           double* __restrict__ v) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int lp = *count;
  if (r >= n) return;
  v[r] = (r < lp) ? ((double)lp / (double)(lp - r)) * skey[r] : INFINITY;
}

__global__ void k_bh_final(const double* __restrict__ z, const double* __restrict__ p, const int* __restrict__ sidx,
                           const double* __restrict__ cm, int n, const int* __restrict__ count,
                           double* __restrict__ cz) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int lp = *count;
  const int i = sidx[r];
  double adj;
  if (r >= lp)
    adj = NAN;  // NA p-value: stays NA
  else if (lp <= 1)
    adj = p[i];  // p.adjust: if (n <= 1) return(p0)
  else
    adj = cm[r] < 1.0 ? cm[r] : 1.0;
  const double zi = z[i];
  const double s = zi > 0 ? 1.0 : (zi < 0 ? -1.0 : (isnan(zi) ? NAN : 0.0));
  cz[i] = s * qnorm(adj, false);
}

struct MinOp {
  __device__ __host__ double operator()(double a, double b) const { return b < a ? b : a; }
};

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace layout for n entries (bytes); `work == nullptr` queries the size.
hipError_t launch_bh_cz(const double* z, int n, double* cz, void* work, size_t* work_bytes, hipStream_t s) {
  size_t sort_tmp = 0, scan_tmp = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, sort_tmp, (const double*)nullptr,
                                                              (double*)nullptr, (const int*)nullptr,
                                                              (int*)nullptr, n > 0 ? n : 1, 0, 64, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::InclusiveScan(nullptr, scan_tmp, (const double*)nullptr, (double*)nullptr, MinOp(),
                                        n > 0 ? n : 1, s);
  if (e != hipSuccess) return e;
  const size_t nd = align256(sizeof(double) * (size_t)(n > 0 ? n : 1));
  const size_t ni = align256(sizeof(int) * (size_t)(n > 0 ? n : 1));
  const size_t tmp = align256(sort_tmp > scan_tmp ? sort_tmp : scan_tmp);
  const size_t need = 4 * nd + 2 * ni + 256 + tmp;
  if (!work) {
    *work_bytes = need;
    return hipSuccess;
  }
  if (*work_bytes < need) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  char* w = static_cast<char*>(work);
  double* key = reinterpret_cast<double*>(w);
  double* skey = reinterpret_cast<double*>(w + nd);
  double* p = reinterpret_cast<double*>(w + 2 * nd);
  double* v = reinterpret_cast<double*>(w + 3 * nd);
  int* idx = reinterpret_cast<int*>(w + 4 * nd);
  int* sidx = reinterpret_cast<int*>(w + 4 * nd + ni);
  int* count = reinterpret_cast<int*>(w + 4 * nd + 2 * ni);
  void* t = w + 4 * nd + 2 * ni + 256;
  e = hipMemsetAsync(count, 0, sizeof(int), s);
  if (e != hipSuccess) return e;
  const int blk = 256, grid = (n + blk - 1) / blk;
  hipLaunchKernelGGL(k_bh_keys, dim3(grid), dim3(blk), 0, s, z, n, key, idx, p, count);
  size_t tb = sort_tmp;
  e = hipcub::DeviceRadixSort::SortPairsDescending(t, tb, key, skey, idx, sidx, n, 0, 64, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bh_scale, dim3(grid), dim3(blk), 0, s, skey, n, count, v);
  tb = scan_tmp;
  e = hipcub::DeviceScan::InclusiveScan(t, tb, v, key, MinOp(), n, s);  // key reused as cm
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bh_final, dim3(grid), dim3(blk), 0, s, z, p, sidx, key, n, count, cz);
  return hipGetLastError();
}

// Gene order for the tile bootstrap: radix sort of (key, gene) pairs on the keys' low `bits`
// bits (launch_ell forms 16-bit keys), ascending and stable.  `work == nullptr` queries the
// temporary storage size.
hipError_t launch_gene_order(const unsigned* key, const int* idx, int n, unsigned* key_out, int* order, void* work,
                             size_t* work_bytes, hipStream_t s, int bits) {
  if (bits < 1 || bits > 32) return hipErrorInvalidValue;
  if (!work) {
    return hipcub::DeviceRadixSort::SortPairs(nullptr, *work_bytes, key, key_out, idx, order, n > 0 ? n : 1, 0, bits,
                                              s);
  }
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceRadixSort::SortPairs(work, *work_bytes, key, key_out, idx, order, n, 0, bits, s);
}

}  // namespace scde
