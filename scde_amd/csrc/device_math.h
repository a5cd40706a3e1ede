// device_math.h -- FP64 device restatement of the R nmath routines the scde
// hot path calls (Rf_dnbinom / Rf_dpois at src/jpmatLogBoot.cpp:174,183,190),
// plus R's qnorm (AS241) used by the Z-score epilogue (R/functions.R:3528-3529).
//
// Everything is IEEE FP64 with inf/NaN semantics intact: the translation unit
// is compiled with -ffp-contract=off and without fast-math, because the path
// relies on exact -inf grid points and on clamping at -DBL_MAX/ncells/1.1.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>

namespace scde {

constexpr double kLn2Pi = 1.837877066409345483560659472811;
constexpr double kLnSqrt2Pi = 0.918938533204672741780329736406;
constexpr double k2Pi = 6.283185307179586476925286766559;

// Stirling-series error at n/2, n = 0..30 (exact values; R nmath stirlerr.c).
__device__ __constant__ const double kSferrHalves[31] = {
    0.0,
    0.1534264097200273452913848, 0.0810614667953272582196702,
    0.0548141210519176538961390, 0.0413406959554092940938221,
    0.03316287351993628748511048, 0.02767792568499833914878929,
    0.02374616365629749597132920, 0.02079067210376509311152277,
    0.01848845053267318523077934, 0.01664469118982119216319487,
    0.01513497322191737887351255, 0.01387612882307074799874573,
    0.01281046524292022692424986, 0.01189670994589177009505572,
    0.01110455975820691732662991, 0.010411265261972096497478567,
    0.009799416126158803298389475, 0.009255462182712732917728637,
    0.008768700134139385462952823, 0.008330563433362871256469318,
    0.007934114564314020547248100, 0.007573675487951840794972024,
    0.007244554301320383179543912, 0.006942840107209529865664152,
    0.006665247032707682442354394, 0.006408994188004207068439631,
    0.006171712263039457647532867, 0.005951370112758847735624416,
    0.005746216513010115682023589, 0.005554733551962801371038690};

__device__ inline double stirlerr(double n) {
  const double S0 = 0.083333333333333333333, S1 = 0.00277777777777777777778,
               S2 = 0.00079365079365079365079365, S3 = 0.000595238095238095238095238,
               S4 = 0.0008417508417508417508417508;
  if (n <= 15.0) {
    double nn = n + n;
    if (nn == (double)(int)nn) return kSferrHalves[(int)nn];
    return lgamma(n + 1.) - (n + 0.5) * log(n) + n - kLnSqrt2Pi;
  }
  double nn = n * n;
  if (n > 500) return (S0 - S1 / nn) / n;
  if (n > 80) return (S0 - (S1 - S2 / nn) / nn) / n;
  if (n > 35) return (S0 - (S1 - (S2 - S3 / nn) / nn) / nn) / n;
  return (S0 - (S1 - (S2 - (S3 - S4 / nn) / nn) / nn) / nn) / n;
}

// deviance term bd0(x, np) = x log(x/np) + np - x, Taylor form near x == np
#ifndef SCDE_TABLES_DIAG
#define SCDE_TABLES_DIAG 0  // timing-only builds: 1 = bd0 without its series, 2 = trivial dnbinom
#endif
__device__ inline double bd0(double x, double np) {
  if (!isfinite(x) || !isfinite(np) || np == 0.0) return NAN;
  if (!(SCDE_TABLES_DIAG & 1) && fabs(x - np) < 0.1 * (x + np)) {
    double v = (x - np) / (x + np);
    double s = (x - np) * v;
    if (fabs(s) < DBL_MIN) return s;
    double ej = 2 * x * v;
    v = v * v;
    for (int j = 1; j < 1000; j++) {
      ej *= v;
      double s1 = s + ej / ((j << 1) + 1);
      if (s1 == s) return s1;
      s = s1;
    }
  }
  return x * log(x / np) + np - x;
}

__device__ inline double dbinom_raw_log(double x, double n, double p, double q) {
  if (p == 0) return (x == 0) ? 0.0 : -INFINITY;
  if (q == 0) return (x == n) ? 0.0 : -INFINITY;
  if (x == 0) {
    if (n == 0) return 0.0;
    return (p < 0.1) ? -bd0(n, n * q) - n * p : n * log(q);
  }
  if (x == n) return (q < 0.1) ? -bd0(n, n * p) - n * q : n * log(p);
  if (x < 0 || x > n) return -INFINITY;
  double lc = stirlerr(n) - stirlerr(x) - stirlerr(n - x) - bd0(x, n * p) - bd0(n - x, n * q);
  double lf = kLn2Pi + log(x) + log1p(-x / n);
  return lc - 0.5 * lf;
}

// log dnbinom(x; size, prob)
__device__ inline double dnbinom_log(double x, double size, double prob) {
  if (isnan(x) || isnan(size) || isnan(prob)) return x + size + prob;
  if (prob <= 0 || prob > 1 || size < 0) return NAN;
  if (x < 0 || !isfinite(x)) return -INFINITY;
  if (x == 0 && size == 0) return 0.0;
  x = rint(x);
  if (!isfinite(size)) size = DBL_MAX;
  double ans = dbinom_raw_log(size, x + size, prob, 1 - prob);
  double p = size / (size + x);
  return log(p) + ans;
}

// dnbinom_log for one count x and a size (theta) that is the same at every grid point:
// the terms that depend only on (size, x) -- three stirlerr (two of them lgamma calls for
// size < 15), the log factor and log(size/(size+x)) -- are computed once per column.
// dnbinom_log_c then evaluates exactly dnbinom_log's operations in the same order, so the
// result is bit-identical.
struct NbConst {
  double x, size, n, nx, S, lf, lp;
  bool trivial;  // x == 0 && size == 0 -> 0; or non-finite inputs handled by dnbinom_log
};

__device__ inline NbConst nb_const(double x, double size) {
  NbConst c;
  c.trivial = isnan(x) || isnan(size) || size < 0 || x < 0 || !isfinite(x) || (x == 0 && size == 0);
  x = rint(x);
  if (!isfinite(size)) size = DBL_MAX;
  c.x = x;
  c.size = size;
  c.n = x + size;           // dbinom_raw's n
  c.nx = c.n - size;        // its n - x
  c.S = 0.0;
  c.lf = 0.0;
  if (!c.trivial && size != c.n && size > 0) {
    c.S = stirlerr(c.n) - stirlerr(size) - stirlerr(c.nx);
    c.lf = kLn2Pi + log(size) + log1p(-size / c.n);
  }
  c.lp = log(size / (size + x));
  return c;
}

__device__ inline double dnbinom_log_c(const NbConst& c, double x_in, double size_in, double prob) {
  if (SCDE_TABLES_DIAG & 2) return c.lp - prob * c.S;
  if (c.trivial || isnan(prob)) return dnbinom_log(x_in, size_in, prob);
  if (prob <= 0 || prob > 1) return NAN;
  const double X = c.size, n = c.n, p = prob, q = 1 - prob;
  double ans;
  if (p == 0)
    ans = (X == 0) ? 0.0 : -INFINITY;
  else if (q == 0)
    ans = (X == n) ? 0.0 : -INFINITY;
  else if (X == 0)
    ans = (n == 0) ? 0.0 : ((p < 0.1) ? -bd0(n, n * q) - n * p : n * log(q));
  else if (X == n)
    ans = (q < 0.1) ? -bd0(n, n * p) - n * q : n * log(p);
  else {
    const double lc = c.S - bd0(X, n * p) - bd0(c.nx, n * q);
    ans = lc - 0.5 * c.lf;
  }
  return c.lp + ans;
}

// log dpois(x; lambda)
__device__ inline double dpois_log(double x, double lambda) {
  if (isnan(x) || isnan(lambda)) return x + lambda;
  if (lambda < 0) return NAN;
  if (x < 0 || !isfinite(x)) return -INFINITY;
  x = rint(x);
  if (lambda == 0) return (x == 0) ? 0.0 : -INFINITY;
  if (!isfinite(lambda)) return -INFINITY;
  if (x <= lambda * DBL_MIN) return -lambda;
  if (lambda < x * DBL_MIN) return -lambda + x * log(lambda) - lgamma(x + 1);
  return -0.5 * log(k2Pi * x) + (-stirlerr(x) - bd0(x, lambda));
}

// R qnorm(p, 0, 1, lower_tail, log.p = FALSE): Wichura's AS241 (PPND16)
__device__ inline double qnorm(double p, bool lower_tail) {
  if (isnan(p)) return p;
  if (p < 0 || p > 1) return NAN;
  if (p == 0) return lower_tail ? -INFINITY : INFINITY;
  if (p == 1) return lower_tail ? INFINITY : -INFINITY;
  double p_ = lower_tail ? p : (0.5 - p + 0.5);
  double q = p_ - 0.5, r, val;
  if (fabs(q) <= .425) {
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
  r = sqrt(-log(r));
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

// exp for d in [-746, 0] (softmax and table normalisation): exp(d) = 2^(k/64) * e^r, k = rint(64 d / ln 2),
// r = d - k ln2/64 (Cody-Waite, |r| <= ln2/128), e^r - 1 by its degree-5 Taylor
// polynomial (truncation 3.5e-17), 2^(j/64) from a 64-entry LDS table, ldexp for
// 2^(k >> 6) (denormal results round once there).  exp(0) is exactly 1.  ~12 VALU
// slots against ~43 for the library exp whose degree-11 polynomial materialises
// most coefficients with v_mov; <= 2 ulp.
__device__ __constant__ const double kExp2Frac64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951};

__device__ __forceinline__ double exp_tab(double d, const double* __restrict__ tab) {
  const double kd = __builtin_rint(d * 92.33248261689366);  // 64 / ln 2
  const int k = (int)kd;
  double r = fma(kd, -0.010830424667801708, d);  // ln2/64, high 29 bits: kd * hi is exact
  r = fma(kd, -2.8447437476627285e-11, r);       // ln2/64 - hi
  const double r2 = r * r;
  double q = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  const double em1 = fma(q, r2, r);
  const double t = tab[k & 63];
  return ldexp(fma(t, em1, t), k >> 6);
}

// ---- double-double accumulation (emulates R's LDOUBLE rowSums / cumsum) ----
struct dd {
  double hi, lo;
};
__device__ inline dd two_sum(double a, double b) {
  double s = __dadd_rn(a, b);
  double bb = __dsub_rn(s, a);
  double e = __dadd_rn(__dsub_rn(a, __dsub_rn(s, bb)), __dsub_rn(b, bb));
  return {s, e};
}
__device__ inline dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  double lo = __dadd_rn(s.lo, __dadd_rn(a.lo, b.lo));
  return two_sum(s.hi, lo);
}
__device__ inline dd dd_add_d(dd a, double b) {
  dd s = two_sum(a.hi, b);
  return two_sum(s.hi, __dadd_rn(s.lo, a.lo));
}
__device__ inline double dd_to_d(dd a) { return __dadd_rn(a.hi, a.lo); }

}  // namespace scde
