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
#ifndef SCDE_BD0_SERIES_OOL
#define SCDE_BD0_SERIES_OOL 1
#endif
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

__device__ __noinline__ NbConst nb_const(double x, double size) {  // once per column, out of line
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

__device__ __noinline__ double dpois_log_cold(double x, double lambda) { return dpois_log(x, lambda); }

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

// exp_tab with the rounding of 64 d / ln 2 by the 1.5 * 2^52 shift (one fma and one add for
// rint + cvt; k is the shifted value's low word).  Study builds only (SCDE_GENE_EXP = 2).
__device__ __forceinline__ double exp_tab_m(double d, const double* __restrict__ tab) {
  const double sh = fma(d, 92.33248261689366, 0x1.8p52);
  const double kd = sh - 0x1.8p52;
  const int k = (int)(unsigned)__double_as_longlong(sh);
  double r = fma(kd, -0.010830424667801708, d);
  r = fma(kd, -2.8447437476627285e-11, r);
  const double r2 = r * r;
  double q = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  const double em1 = fma(q, r2, r);
  const double t = tab[k & 63];
  return ldexp(fma(t, em1, t), k >> 6);
}

// exp for d in [-746, 0] without a table (k_tables_lpc, where the table read's per-lane index would
// put an LDS round trip with bank conflicts in every point's chain): exp(d) = 2^n e^r, n = rint(d / ln 2),
// r = d - n ln 2 (Cody-Waite: n ln2_hi exact for |n| < 2^21), |r| <= 0.347, e^r by its degree-13
// Taylor polynomial (truncation < 5e-18 relative), ldexp for 2^n (subnormal results round once).
// exp(0) is exactly 1.  19 VALU slots, <= 2 ulp.
__device__ __forceinline__ double exp_poly(double d) {
  const double kd = __builtin_rint(d * 1.4426950408889634);
  const int n = (int)kd;
  double r = fma(kd, -6.93147180369123816490e-01, d);
  r = fma(kd, -1.90821492927058770002e-10, r);
  double p = 1.0 / 6227020800.0;
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, n);
}

// log for positive normal x (other inputs fall back to the library log): x = m 2^e with
// m in [0.75, 1.5); 97 intervals centred on c_j = 0.75 + j/128 (the one around 1 has
// c = 1 exactly, so r = m - 1 is exact there and results near 0 keep full relative
// accuracy); r = m/c_j - 1 in [-1/192, 1/192]; log1p(r) by its degree-8 Taylor
// polynomial (truncation < 1e-20); log(c_j) as a double-double.  <= 2 ulp, ~25 VALU
// slots against ~100 for the library log.  The tables are staged in LDS by the caller.
__device__ __constant__ const double kLogInvC[97] = {
    1.3333333333333333, 1.3195876288659794, 1.3061224489795917, 1.292929292929293,
    1.28, 1.2673267326732673, 1.2549019607843137, 1.2427184466019416,
    1.2307692307692308, 1.2190476190476192, 1.2075471698113207, 1.1962616822429906,
    1.1851851851851851, 1.1743119266055047, 1.1636363636363636, 1.1531531531531531,
    1.1428571428571428, 1.1327433628318584, 1.1228070175438596, 1.1130434782608696,
    1.103448275862069, 1.0940170940170941, 1.0847457627118644, 1.0756302521008403,
    1.0666666666666667, 1.0578512396694215, 1.0491803278688525, 1.0406504065040652,
    1.032258064516129, 1.024, 1.0158730158730158, 1.0078740157480315,
    1.0, 0.9922480620155039, 0.9846153846153847, 0.9770992366412213,
    0.9696969696969697, 0.9624060150375939, 0.9552238805970149, 0.9481481481481482,
    0.9411764705882353, 0.9343065693430657, 0.927536231884058, 0.920863309352518,
    0.9142857142857143, 0.9078014184397163, 0.9014084507042254, 0.8951048951048951,
    0.8888888888888888, 0.8827586206896552, 0.8767123287671232, 0.8707482993197279,
    0.8648648648648649, 0.8590604026845637, 0.8533333333333334, 0.847682119205298,
    0.8421052631578947, 0.8366013071895425, 0.8311688311688312, 0.8258064516129032,
    0.8205128205128205, 0.8152866242038217, 0.810126582278481, 0.8050314465408805,
    0.8, 0.7950310559006211, 0.7901234567901234, 0.7852760736196319,
    0.7804878048780488, 0.7757575757575758, 0.7710843373493976, 0.7664670658682635,
    0.7619047619047619, 0.757396449704142, 0.7529411764705882, 0.7485380116959064,
    0.7441860465116279, 0.7398843930635838, 0.735632183908046, 0.7314285714285714,
    0.7272727272727273, 0.7231638418079096, 0.7191011235955056, 0.7150837988826816,
    0.7111111111111111, 0.7071823204419889, 0.7032967032967034, 0.6994535519125683,
    0.6956521739130435, 0.6918918918918919, 0.6881720430107527, 0.6844919786096256,
    0.6808510638297872, 0.6772486772486772, 0.6736842105263158, 0.6701570680628273,
    0.6666666666666666};
__device__ __constant__ const double kLogCHi[97] = {
    -0.2876820724517809, -0.27731928541623435, -0.26706278524904525, -0.2569104137850272,
    -0.24686007793152578, -0.2369097470783577, -0.22705745063534608, -0.2173012756899814,
    -0.2076393647782445, -0.1980699137620938, -0.18859116980755003, -0.179201429457711,
    -0.16989903679539747, -0.16068238169047347, -0.15154989812720093, -0.14250006260728304,
    -0.13353139262452263, -0.1246424452072766, -0.1158318155251217, -0.1070981355563671,
    -0.09844007281325252, -0.08985632912186105, -0.0813456394539524, -0.07290677080808779,
    -0.06453852113757118, -0.05623971832287608, -0.048009219186360606, -0.039845908547199674,
    -0.0317486983145803, -0.023716526617316044, -0.015748356968139168, -0.007843177461025893,
    0.0, 0.007782140442054949, 0.015504186535965254, 0.02316705928153438,
    0.030771658666753687, 0.0383188643021366, 0.0458095360312942, 0.053244514518812285,
    0.06062462181643484, 0.06795066190850775, 0.07522342123758753, 0.08244366921107459,
    0.08961215868968714, 0.09672962645855111, 0.10379679368164356, 0.11081436634029011,
    0.11778303565638346, 0.12470347850095724, 0.13157635778871926, 0.13840232285911913,
    0.1451820098444979, 0.15191604202584197, 0.15860503017663857, 0.16524957289530717,
    0.17185025692665923, 0.1784076574728183, 0.184922338494012, 0.19139485299962947,
    0.19782574332991987, 0.2042155414286909, 0.21056476910734964, 0.21687393830061436,
    0.22314355131420976, 0.22937410106484582, 0.2355660713127669, 0.24171993688714516,
    0.24783616390458127, 0.25391520998096345, 0.25995752443692605, 0.26596354849713794,
    0.27193371548364176, 0.2778684510034563, 0.2837681731306446, 0.28963329258304266,
    0.2954642128938359, 0.3012613305781618, 0.3070250352949119, 0.3127557100038969,
    0.3184537311185346, 0.324119468654212, 0.329753286372468, 0.3353555419211378,
    0.3409265869705932, 0.34646676734620857, 0.3519764231571782, 0.3574558889218038,
    0.3629054936893685, 0.3683255611587076, 0.37371640979358406, 0.37907835293496944,
    0.38441169891033206, 0.3897167511400252, 0.394993808240869, 0.4002431641270127,
    0.4054651081081644};
__device__ __constant__ const double kLogCLo[97] = {
    -2.607160616442564e-17, 7.44528405583513e-18, 7.32891532732017e-18, -2.502843296152504e-17,
    -1.361743371748368e-17, -1.9682402978398164e-18, -9.551415762738488e-18, -1.6168452453763015e-18,
    -1.2053243216686129e-17, -3.742843482461439e-18, 7.432164219196925e-18, 1.0785017454858423e-17,
    4.868008764439071e-19, 3.650183553047837e-18, -5.1669593684615594e-18, 9.926388234225749e-18,
    3.664457663660085e-18, 5.808912678940971e-18, -4.338484369808096e-18, 1.73705104015906e-18,
    4.439009633675136e-18, 6.273760163689594e-19, -5.07707635593117e-18, 6.306860257532778e-18,
    6.470486661692933e-18, 3.2835149805605613e-18, -1.4390903347292205e-18, 3.129547680315208e-18,
    -3.0382263084680858e-18, 1.5774243488668215e-18, -1.0021578630528974e-18, -2.764708154124904e-19,
    0.0, -1.2819179123343845e-20, -3.278321022892429e-19, -1.1769544932063305e-18,
    1.0431732029005968e-18, -2.357996157351286e-18, 1.902959866474257e-18, -1.665575816973663e-18,
    2.6424025938726934e-18, -1.2802141240611733e-18, -5.930604196293241e-18, 5.700437773813987e-18,
    -5.4268129336647135e-18, -5.597397486289965e-19, 5.47772415726659e-18, 1.183748342825649e-18,
    -1.1971685747593677e-18, -4.6522609636496624e-18, 1.1123000879729588e-17, 4.447777301357527e-18,
    8.242418783022475e-18, 6.4838631244022194e-18, 1.1257003872182592e-17, -1.0094935622322628e-17,
    -6.0224538210113705e-18, -1.2432553788701131e-17, 3.0236614153574064e-18, -1.2129496905792884e-17,
    1.2821194372980142e-17, 2.7338281018722773e-18, -4.249405314729895e-18, 4.551026193234283e-18,
    -9.091270597324799e-18, 9.927671823978025e-18, -2.3943371495187355e-18, 8.900990022166643e-18,
    -1.2432209578702523e-17, -8.048097394424201e-18, 2.069806938978935e-17, 5.3393802761314314e-18,
    7.83319637697442e-19, -9.16018294909263e-19, -2.032665581126656e-17, 2.0535953219858174e-17,
    -2.16461086040599e-17, -9.048511144048564e-18, -1.2319916200101964e-17, -1.451808353098951e-17,
    2.7114779367326236e-17, -7.958214381893813e-18, 2.122020616196946e-18, 1.834564437059473e-17,
    1.7467136443544747e-17, 1.028583585496265e-17, -1.2953893030191963e-17, -2.5136910072413547e-17,
    -2.1492361455310972e-17, 2.690672380132659e-17, 2.1836211281198184e-17, 1.587939415338447e-17,
    -1.612149700764673e-17, 2.734172667856699e-17, -1.5113724418336168e-17, -1.1349239205188711e-17,
    -2.8811380259626426e-18};

// cold paths kept out of line so they do not inflate the hot loops' register allocation

struct LogTab {
  const double* inv;
  const double* hi;
  const double* lo;
};

__device__ __forceinline__ double log_tab_hot(double x, const LogTab& t, int eadj = 0) {  // x in [DBL_MIN, inf)
  int e;
  double m = frexp(x, &e);  // [0.5, 1)
  e -= eadj;
  if (m < 0.75) {
    m *= 2.0;
    e -= 1;
  }
  const int j = (int)((m - 0.75) * 128.0 + 0.5);
  const double r = fma(m, t.inv[j], -1.0);
  double q = fma(r, -1.0 / 8.0, 1.0 / 7.0);
  q = fma(q, r, -1.0 / 6.0);
  q = fma(q, r, 1.0 / 5.0);
  q = fma(q, r, -1.0 / 4.0);
  q = fma(q, r, 1.0 / 3.0);
  q = fma(q, r, -0.5);
  const double p = fma(q * r, r, r);  // log1p(r)
  const double ed = (double)e;
  // e*ln2_hi is exact (ln2_hi has 11 trailing zero bits)
  return (fma(ed, 0.6931471805598903, t.hi[j]) + (fma(ed, 5.497923018708371e-14, t.lo[j]) + p));
}

// Branch-free and call-free over all inputs: a subnormal x is scaled by 2^64 first (exact)
// and 64 comes off the exponent, so it takes the same table path as a normal x; zero, inf,
// negative and NaN arguments are selected in (-inf, inf, NaN, NaN as the library log).
__device__ __forceinline__ double log_tab(double x, const LogTab& t) {
  const bool sub = x > 0.0 && x < DBL_MIN;
  const double xs = sub ? x * 0x1p64 : x;
  const bool ok = xs >= DBL_MIN && xs < INFINITY;
  const double r0 = log_tab_hot(ok ? xs : 1.0, t, sub ? 64 : 0);
  const double rs = (x == 0.0) ? -INFINITY : (x == INFINITY) ? INFINITY : __builtin_nan("");
  return ok ? r0 : rs;
}

// bd0's Taylor series (|x - np| < 0.1 (x + np)), out of line
__device__ __noinline__ double bd0_series(double x, double np) {
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
  return x * log(x / np) + np - x;  // not reached for |v| < 0.1
}

// bd0 with the table log in its non-series branch
__device__ inline double bd0_t(double x, double np, const LogTab& lt) {
  if (!isfinite(x) || !isfinite(np) || np == 0.0) return NAN;
  if (SCDE_BD0_SERIES_OOL && fabs(x - np) < 0.1 * (x + np)) return bd0_series(x, np);
  if (fabs(x - np) < 0.1 * (x + np)) {
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
  return x * log_tab(x / np, lt) + np - x;
}

__device__ __noinline__ double dnbinom_log_cold(double x, double size, double prob) {
  return dnbinom_log(x, size, prob);
}

__device__ inline double dnbinom_log_ct(const NbConst& c, double x_in, double size_in, double prob, const LogTab& lt) {
  if (c.trivial || isnan(prob)) return dnbinom_log_cold(x_in, size_in, prob);
  if (prob <= 0 || prob > 1) return NAN;
  const double X = c.size, n = c.n, p = prob, q = 1 - prob;
  double ans;
  if (p == 0)
    ans = (X == 0) ? 0.0 : -INFINITY;
  else if (q == 0)
    ans = (X == n) ? 0.0 : -INFINITY;
  else if (X == 0)
    ans = (n == 0) ? 0.0 : ((p < 0.1) ? -bd0_t(n, n * q, lt) - n * p : n * log_tab(q, lt));
  else if (X == n)
    ans = (q < 0.1) ? -bd0_t(n, n * p, lt) - n * q : n * log_tab(p, lt);
  else {
    const double lc = c.S - bd0_t(X, n * p, lt) - bd0_t(c.nx, n * q, lt);
    ans = lc - 0.5 * c.lf;
  }
  return c.lp + ans;
}

// ---- fast constant-theta dnbinom (k_tables hot loop) ----
// For a constant size theta, p_k = theta / (theta + mu_k), q_k = 1 - p_k and their logs
// depend only on (cell, grid point) and are precomputed once per cell (k_cell_prep).  bd0's
// non-series branch x log(x / np) + np - x is then evaluated as x (log x - log n - log p_k)
// + np - x: no division and no log per grid point (the log of the ratio is exact to a few
// ulps of its terms; outside the series region |log(x/np)| > 0.18, so the relative error
// stays ~1e-15).  The series branch divides by the constant 2j+1 through a reciprocal
// table.  Every case the reference routes elsewhere (p or q == 0, np or nq not a positive
// finite number, x == 0 && size == 0, non-finite inputs) returns `false` and the caller
// takes the exact dnbinom_log_ct path for that lane.
__device__ __constant__ const double kInvOdd[40] = {
    1.0,       1.0 / 3,  1.0 / 5,  1.0 / 7,  1.0 / 9,  1.0 / 11, 1.0 / 13, 1.0 / 15, 1.0 / 17, 1.0 / 19,
    1.0 / 21,  1.0 / 23, 1.0 / 25, 1.0 / 27, 1.0 / 29, 1.0 / 31, 1.0 / 33, 1.0 / 35, 1.0 / 37, 1.0 / 39,
    1.0 / 41,  1.0 / 43, 1.0 / 45, 1.0 / 47, 1.0 / 49, 1.0 / 51, 1.0 / 53, 1.0 / 55, 1.0 / 57, 1.0 / 59,
    1.0 / 61,  1.0 / 63, 1.0 / 65, 1.0 / 67, 1.0 / 69, 1.0 / 71, 1.0 / 73, 1.0 / 75, 1.0 / 77, 1.0 / 79};

// bd0 series (|x - np| < 0.1 (x + np)): |v| < 0.1, so v^2 < 0.01 and the terms fall by
// 100x per step; 39 steps reach any double.
__device__ __noinline__ double bd0_series_fast(double x, double np) {
  double v = (x - np) / (x + np);
  double s = (x - np) * v;
  if (fabs(s) < DBL_MIN) return s;
  double ej = 2 * x * v;
  v = v * v;
  for (int j = 1; j < 40; j++) {
    ej *= v;
    const double s1 = s + ej * kInvOdd[j];
    if (s1 == s) return s1;
    s = s1;
  }
  return s;
}

// bd0's series as a fixed polynomial: with v = (x - np)/(x + np), |v| < 0.1, w = v^2 < 0.01,
// bd0 = (x - np) v + 2 x v sum_{j>=1} w^j / (2j + 1) (src: R nmath bd0, the loop R runs until
// the sum stops changing).  Nine terms leave a tail below 2e-17 of the first, so the result
// matches the loop to rounding, with no loop, no early exit and no divergence.
// fma as one VOP3 v_fma_f64 (the same rounding as fma()): with the coefficient held in a
// VGPR pair across the loop, the compiler's v_fmac form would first copy it into the
// accumulator (one v_mov_b64 per Horner step)
__device__ __forceinline__ double fma3(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ double bd0_poly(double x, double np) {
  const double d = x - np;
  const double v = d / (x + np);
  const double w = v * v;
  double P = fma3(1.0 / 19, w, 1.0 / 17);
  P = fma3(P, w, 1.0 / 15);
  P = fma3(P, w, 1.0 / 13);
  P = fma3(P, w, 1.0 / 11);
  P = fma3(P, w, 1.0 / 9);
  P = fma3(P, w, 1.0 / 7);
  P = fma3(P, w, 1.0 / 5);
  P = fma3(P, w, 1.0 / 3);
  P *= w;
  return fma(2.0 * x * v, P, d * v);
}

// L = log x - log np (precomputed as log x - log n - log p).  The series region is taken
// with a wave-uniform branch: only waves with a lane in it evaluate the polynomial.
#ifndef SCDE_BD0_DIAG
#define SCDE_BD0_DIAG 0  // timing-only builds: 1 = never the series (results wrong)
#endif
// bd0 in the series region from L = log(x / np) itself, with no division: x = np e^L gives
// bd0 = np psi(L), psi(L) = L e^L - e^L + 1 = sum_{k>=2} (k - 1) L^k / k!.  In the region
// |v| < 0.1, |L| < log(1.1 / 0.9) = 0.2007, and the terms through k = 12 leave a tail below
// 2.4e-17 of the first (the degree that keeps the general column's 401-point row in registers).  Its error is np |L| |dL| <= 0.2 np |dL| for an error dL of L (a
// few ulps of log x and log np), a fifth of what x L + np - x carries outside the region.
#ifndef SCDE_BD0_PSI
#define SCDE_BD0_PSI 1
#endif
__device__ __forceinline__ double bd0_psi(double np, double L) {
  double P = fma3(11.0 / 479001600.0, L, 10.0 / 39916800.0);
  P = fma3(P, L, 9.0 / 3628800.0);
  P = fma3(P, L, 8.0 / 362880.0);
  P = fma3(P, L, 7.0 / 40320.0);
  P = fma3(P, L, 6.0 / 5040.0);
  P = fma3(P, L, 5.0 / 720.0);
  P = fma3(P, L, 4.0 / 120.0);
  P = fma3(P, L, 3.0 / 24.0);
  P = fma3(P, L, 2.0 / 6.0);
  P = fma3(P, L, 0.5);
  return np * ((L * L) * P);
}
__device__ __forceinline__ double bd0_fast(double x, double np, double L) {
  const bool ser = !(SCDE_BD0_DIAG & 1) && fabs(x - np) < 0.1 * (x + np);
  double b = x * L + np - x;
  if (__builtin_amdgcn_ballot_w64(ser)) {
    const double sv = SCDE_BD0_PSI ? bd0_psi(np, L) : bd0_poly(x, np);
    b = ser ? sv : b;
  }
  return b;
}

struct NbFast {
  double X, n, nx, S, hlf, lp;  // dbinom_raw's x (= size), n, n - x; stirlerr sum; 0.5 lf; log(size/(size+x))
  double lXn, lnxn;             // log X - log n, log(n - X) - log n
  bool ok;                      // the fast path applies to this column
};

__device__ __forceinline__ NbFast nb_fast(const NbConst& c) {
  NbFast f;
  f.X = c.size;
  f.n = c.n;
  f.nx = c.nx;
  f.S = c.S;
  f.hlf = 0.5 * c.lf;
  f.lp = c.lp;
  f.ok = !c.trivial && c.size > 0 && isfinite(c.size) && c.n > 0 && isfinite(c.n);
  f.lXn = f.ok ? log(c.size) - log(c.n) : 0.0;
  f.lnxn = (f.ok && c.nx > 0) ? log(c.nx) - log(c.n) : 0.0;
  return f;
}

// Evaluated for every lane without divergent branches; `bad` marks the lanes that must take
// the exact path instead (their value here is meaningless).  The count-0 test is per column
// (wave-uniform); the q < 0.1 branch runs only in waves that have such a lane.
__device__ __forceinline__ double dnbinom_fast(const NbFast& f, double p, double q, double lp, double lq, bool& bad) {
  const double np = f.n * p, nq = f.n * q;
  bad = !(p > 0.0 && p <= 1.0 && q > 0.0 && np > 0.0 && np < INFINITY && nq > 0.0 && nq < INFINITY);
  double ans;
  if (f.X == f.n) {  // count 0: dbinom_raw's x == n branch
    const bool lowq = q < 0.1;
    ans = f.n * lp;
    if (__builtin_amdgcn_ballot_w64(lowq && !bad)) {
      const double b = -bd0_fast(f.n, np, -lp) - f.n * q;
      ans = lowq ? b : ans;
    }
  } else {
    ans = ((f.S - bd0_fast(f.X, np, f.lXn - lp)) - bd0_fast(f.nx, nq, f.lnxn - lq)) - f.hlf;
  }
  return f.lp + ans;
}

// dnbinom_fast's value without its validity flag (the caller tests validity itself)
__device__ __forceinline__ double dnbinom_fast(const NbFast& f, double p, double q, double lp, double lq) {
  bool bad;
  return dnbinom_fast(f, p, q, lp, lq, bad);
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

// int8 matrix-core helpers (k_boot_tiles bounds)
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// 4 x 4 byte transpose: p_i byte j = source j byte i.
__device__ __forceinline__ void tr4(unsigned a, unsigned b, unsigned c, unsigned d, unsigned& p0, unsigned& p1,
                                    unsigned& p2, unsigned& p3) {
  const unsigned ab02 = __builtin_amdgcn_perm(b, a, 0x06020400u);
  const unsigned ab13 = __builtin_amdgcn_perm(b, a, 0x07030501u);
  const unsigned cd02 = __builtin_amdgcn_perm(d, c, 0x06020400u);
  const unsigned cd13 = __builtin_amdgcn_perm(d, c, 0x07030501u);
  p0 = __builtin_amdgcn_perm(cd02, ab02, 0x05040100u);
  p2 = __builtin_amdgcn_perm(cd02, ab02, 0x07060302u);
  p1 = __builtin_amdgcn_perm(cd13, ab13, 0x05040100u);
  p3 = __builtin_amdgcn_perm(cd13, ab13, 0x07060302u);
}

}  // namespace scde
