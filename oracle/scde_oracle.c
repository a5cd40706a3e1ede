/*
 * scde_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A loop-for-loop CPU restatement of the slowkow/scde differential-expression
 * hot path.  It is imported only by tests/, __graft_entry__.smoke() and the
 * `cpu_baseline` leg of bench.py -- never by the product (scde_amd/).
 *
 * What it restates (file:line into the reference tree):
 *   o_logBootPosterior       src/jpmatLogBoot.cpp:100-331
 *   o_logBootBatchPosterior  src/jpmatLogBoot.cpp:343-531
 *   o_jpmatLogBoot           src/jpmatLogBoot.cpp:11-42
 *   o_jpmatLogBatchBoot      src/jpmatLogBoot.cpp:48-86
 *   o_matSlideMult           src/matSlideMult.cpp:5-23
 *   o_ratio_posterior        R/functions.R:3491-3510 (calculate.ratio.posterior)
 *   o_summary                R/functions.R:5039-5053 (quick.distribution.summary)
 *                            + R/functions.R:3514-3531 (get.ratio.posterior.Z.score)
 *   o_bh_cz                  R/functions.R:5051 (BH-adjusted cZ)
 * Third-party arithmetic restated (absent from /root/reference):
 *   glibc srand()/rand() TYPE_3 additive generator (glibc 2.x random_r.c),
 *     pinned against the live libc in tests/test_oracle.py;
 *   R nmath dnbinom / dbinom_raw / dpois_raw / stirlerr / bd0 (R 3.x-4.3
 *     "classic" forms; lgammafn replaced by C99 lgamma(), <= 1e-15 rel);
 *   R qnorm (Wichura AS241) and pnorm (Cody), pinned against mpmath;
 *   Armadillo accu()/max() two-accumulator order and R's LDOUBLE rowSums /
 *     cumsum (long double on x86-64, exactly as R does).
 *
 * Parity pin: see DESIGN.md "Oracle" -- rand() vs libc, nmath vs mpmath,
 * and the vignette known-answer table (vignettes/diffexp.md:113-119).
 *
 * All matrices are R column-major unless stated otherwise.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MIN_THETA 1.0e-2
#define MAX_THETA 1.0e+3
#define M_LN_2PI_ 1.837877066409345483560659472811
#define M_LN_SQRT_2PI_ 0.918938533204672741780329736406
#define M_2PI_ 6.283185307179586476925286766559

/* ------------------------------------------------------------------ */
/* glibc TYPE_3 rand() (srandom_r / random_r), private state            */
/* ------------------------------------------------------------------ */
#include "scde_oracle.h"

/* Generator variant, for pinning against the published vignette table:
 * 0 = glibc TYPE_3 (Linux, the default); 1 = Park-Miller "minimal standard"
 * (BSD/macOS libc rand(): x = 16807 x mod (2^31-1), returns x - 1 with
 * srand(s): x = s % 0x7ffffffe + 1).  Only the oracle has this switch. */
int o_rng_kind = 0;
void o_set_rng_kind(int k) { o_rng_kind = k; }

void o_srand(o_rng* g, unsigned int seed) {
    int32_t word;
    int i;
    if (o_rng_kind == 1) {
        g->tbl[0] = (int32_t)((seed % 0x7ffffffeu) + 1);
        return;
    }
    if (o_rng_kind == 2 || o_rng_kind == 3) {
        g->tbl[0] = (int32_t)seed;
        return;
    }
    if (seed == 0) seed = 1;
    g->tbl[0] = (int32_t)seed;
    word = (int32_t)seed;
    for (i = 1; i < 31; i++) {
        long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        g->tbl[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (i = 0; i < 310; i++) {
        uint32_t v = (uint32_t)g->tbl[g->f] + (uint32_t)g->tbl[g->r];
        g->tbl[g->f] = (int32_t)v;
        if (++g->f >= 31) g->f = 0;
        if (++g->r >= 31) g->r = 0;
    }
}

static int o_rand_pm(o_rng* g) {
    long hi = g->tbl[0] / 127773, lo = g->tbl[0] % 127773;
    long x = 16807 * lo - 2836 * hi;
    if (x < 0) x += 0x7fffffff;
    g->tbl[0] = (int32_t)x;
    return (int)(x - 1);
}

int o_rand(o_rng* g) {
    if (o_rng_kind == 1) return o_rand_pm(g);
    if (o_rng_kind == 2) { /* older BSD / Darwin: srand(s) keeps s, returns x */
        long hi = g->tbl[0] / 127773, lo = g->tbl[0] % 127773;
        long x = 16807 * lo - 2836 * hi;
        if (x < 0) x += 0x7fffffff;
        g->tbl[0] = (int32_t)x;
        return (int)x;
    }
    if (o_rng_kind == 3) { /* BSD USE_WEAK_SEEDING LCG */
        uint32_t* u = (uint32_t*)&g->tbl[0];
        unsigned long v = (unsigned long)(*u) * 1103515245ul + 12345ul;
        *u = (uint32_t)v;
        return (int)(v % 2147483648ul);
    }
    uint32_t v = (uint32_t)g->tbl[g->f] + (uint32_t)g->tbl[g->r];
    g->tbl[g->f] = (int32_t)v;
    if (++g->f >= 31) g->f = 0;
    if (++g->r >= 31) g->r = 0;
    return (int)(v >> 1);
}

/* `while(n <= (rj = rand()/(RAND_MAX/n)));`  src/jpmatLogBoot.cpp:255-257 */
static int o_draw(o_rng* g, int n) {
    int rj;
    while (n <= (rj = o_rand(g) / (2147483647 / n)))
        ;
    return rj;
}

/* export: the raw rand() stream, for pinning against libc */
void o_rand_stream(unsigned int seed, int n, int* out) {
    o_rng g;
    int i;
    o_srand(&g, seed);
    for (i = 0; i < n; i++) out[i] = o_rand(&g);
}

/* export: the draw sequence of `count` cells out of n */
void o_draw_stream(unsigned int seed, int n, int count, int* out) {
    o_rng g;
    int i;
    o_srand(&g, seed);
    for (i = 0; i < count; i++) out[i] = o_draw(&g, n);
}

/* ------------------------------------------------------------------ */
/* R nmath restatement                                                  */
/* ------------------------------------------------------------------ */
static const double sferr_halves[31] = {
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

double o_stirlerr(double n) {
    const double S0 = 0.083333333333333333333, S1 = 0.00277777777777777777778,
                 S2 = 0.00079365079365079365079365, S3 = 0.000595238095238095238095238,
                 S4 = 0.0008417508417508417508417508;
    double nn;
    if (n <= 15.0) {
        nn = n + n;
        if (nn == (int)nn) return sferr_halves[(int)nn];
        return lgamma(n + 1.) - (n + 0.5) * log(n) + n - M_LN_SQRT_2PI_;
    }
    nn = n * n;
    if (n > 500) return (S0 - S1 / nn) / n;
    if (n > 80) return (S0 - (S1 - S2 / nn) / nn) / n;
    if (n > 35) return (S0 - (S1 - (S2 - S3 / nn) / nn) / nn) / n;
    return (S0 - (S1 - (S2 - (S3 - S4 / nn) / nn) / nn) / nn) / n;
}

double o_bd0(double x, double np) {
    double ej, s, s1, v;
    int j;
    if (!isfinite(x) || !isfinite(np) || np == 0.0) return NAN;
    if (fabs(x - np) < 0.1 * (x + np)) {
        v = (x - np) / (x + np);
        s = (x - np) * v;
        if (fabs(s) < DBL_MIN) return s;
        ej = 2 * x * v;
        v = v * v;
        for (j = 1; j < 1000; j++) {
            ej *= v;
            s1 = s + ej / ((j << 1) + 1);
            if (s1 == s) return s1;
            s = s1;
        }
    }
    return x * log(x / np) + np - x;
}

/* log-scale only (give_log = TRUE everywhere on the path) */
double o_dbinom_raw_log(double x, double n, double p, double q) {
    double lf, lc;
    if (p == 0) return (x == 0) ? 0.0 : -INFINITY;
    if (q == 0) return (x == n) ? 0.0 : -INFINITY;
    if (x == 0) {
        if (n == 0) return 0.0;
        lc = (p < 0.1) ? -o_bd0(n, n * q) - n * p : n * log(q);
        return lc;
    }
    if (x == n) {
        lc = (q < 0.1) ? -o_bd0(n, n * p) - n * q : n * log(p);
        return lc;
    }
    if (x < 0 || x > n) return -INFINITY;
    lc = o_stirlerr(n) - o_stirlerr(x) - o_stirlerr(n - x) - o_bd0(x, n * p) - o_bd0(n - x, n * q);
    lf = M_LN_2PI_ + log(x) + log1p(-x / n);
    return lc - 0.5 * lf;
}

/* Rf_dnbinom(x, size, prob, TRUE)  (called at src/jpmatLogBoot.cpp:174,183) */
double o_dnbinom_log(double x, double size, double prob) {
    double ans, p;
    if (isnan(x) || isnan(size) || isnan(prob)) return x + size + prob;
    if (prob <= 0 || prob > 1 || size < 0) return NAN;
    if (x < 0 || !isfinite(x)) return -INFINITY;
    if (x == 0 && size == 0) return 0.0;
    x = nearbyint(x);
    if (!isfinite(size)) size = DBL_MAX;
    ans = o_dbinom_raw_log(size, x + size, prob, 1 - prob);
    p = size / (size + x);
    return log(p) + ans;
}

/* Rf_dpois(x, lambda, TRUE)  (src/jpmatLogBoot.cpp:190) */
double o_dpois_log(double x, double lambda) {
    if (isnan(x) || isnan(lambda)) return x + lambda;
    if (lambda < 0) return NAN;
    if (x < 0 || !isfinite(x)) return -INFINITY;
    x = nearbyint(x);
    if (lambda == 0) return (x == 0) ? 0.0 : -INFINITY;
    if (!isfinite(lambda)) return -INFINITY;
    if (x <= lambda * DBL_MIN) return -lambda;
    if (lambda < x * DBL_MIN) return -lambda + x * log(lambda) - lgamma(x + 1);
    return -0.5 * log(M_2PI_ * x) + (-o_stirlerr(x) - o_bd0(x, lambda));
}

/* Armadillo accu(): two running accumulators over even/odd elements */
static double arma_accu(const double* X, long n, long stride) {
    double v1 = 0, v2 = 0;
    long i, j;
    for (i = 0, j = 1; j < n; i += 2, j += 2) {
        v1 += X[i * stride];
        v2 += X[j * stride];
    }
    if (i < n) v1 += X[i * stride];
    return v1 + v2;
}

/* Armadillo max() with index: first maximum, strict '>' */
static double arma_max(const double* X, long n, long stride, long* idx) {
    double best = -INFINITY;
    long bi = 0, i;
    for (i = 0; i < n; i++) {
        if (X[i * stride] > best) {
            best = X[i * stride];
            bi = i;
        }
    }
    if (idx) *idx = bi;
    return best;
}

/* ------------------------------------------------------------------ */
/* Phase A: per-cell log-posterior tables  (src/jpmatLogBoot.cpp:128-211) */
/* ------------------------------------------------------------------ */
/* models: ncells x 12 col-major.  Table for cell i: G x U_i col-major.     */
static void o_cell_tables(const double* models, int ncells, int i, const int* uc, int nc,
                          const double* mag, int G, int localtheta, int squarelogit, double minlogprob,
                          int want_maxi, double* pm, int* maxi, double* work) {
#define MD(col) models[(long)i + (long)ncells * (col)]
    double* mu = work;
    double* cfp = work + G;
    double* cfpr = work + 2 * G;
    double* th = work + 3 * G;
    double* nbp = work + 4 * G;
    double maxcfp;
    int k, j;
    for (k = 0; k < G; k++) {
        mu[k] = exp(mag[k] * MD(4) + MD(3));
        double c;
        if (squarelogit) {
            c = (MD(1) + mag[k] * MD(11)) * mag[k];
        } else {
            c = mag[k] * MD(1);
        }
        c += MD(0);
        c = 1.0 / (exp(c) + 1.0);
        cfpr[k] = log(1.0 - c);
        cfp[k] = log(c);
    }
    maxcfp = arma_max(cfp, G, 1, NULL);
    if (localtheta) {
        double tb = MD(7) - MD(6);
        for (k = 0; k < G; k++) {
            double t = -1.0 * mag[k] + MD(8);
            t *= MD(9);
            t = pow(10.0, t) + 1.0;
            t = pow(t, MD(10));
            t = tb / t;
            t += MD(6);
            t = exp(-1.0 * t);
            if ((!isfinite(t)) || (t < MIN_THETA)) t = MIN_THETA;
            if (t > MAX_THETA) t = MAX_THETA;
            th[k] = t;
        }
    } else {
        for (k = 0; k < G; k++) th[k] = MD(5);
    }
    for (j = 0; j < nc; j++) {
        double x = (double)uc[j];
        double fp, maxp, s;
        for (k = 0; k < G; k++) {
            double muv = mu[k];
            if ((k < G - 1 && x > muv && x < mu[k + 1]) || (k == G - 1 && x > muv)) muv = x;
            nbp[k] = o_dnbinom_log(x, th[k], th[k] / (th[k] + muv));
        }
        for (k = 0; k < G; k++) nbp[k] += cfpr[k];
        fp = o_dpois_log(x, exp(MD(2)));
        maxp = arma_max(nbp, G, 1, NULL);
        if (maxp < (maxcfp + fp)) maxp = maxcfp + fp;
        for (k = 0; k < G; k++) nbp[k] = exp(nbp[k] - maxp) + exp(cfp[k] + fp - maxp);
        s = arma_accu(nbp, G, 1);
        for (k = 0; k < G; k++) nbp[k] = log(nbp[k] / s);
        if (want_maxi) {
            long mi;
            arma_max(nbp, G, 1, &mi);
            maxi[j] = (int)mi;
        }
        for (k = 0; k < G; k++) {
            if (nbp[k] < minlogprob) nbp[k] = minlogprob;
            pm[(long)j * G + k] = nbp[k];
        }
    }
#undef MD
}

/* Build tables for all cells.  ucl_off has ncells+1 entries; tables are laid
 * out [cell][U_i][G] contiguously at tab + G*ucl_off[i].                   */
void o_tables(const double* models, int ncells, const int* ucl, const long* ucl_off, const double* mag, int G,
              int localtheta, int squarelogit, int want_maxi, double* tab, int* maxi) {
    double minlogprob = -1 * DBL_MAX / ncells / 1.1;
    double* work = (double*)malloc(sizeof(double) * 5 * (size_t)G);
    int i;
    for (i = 0; i < ncells; i++) {
        long o = ucl_off[i];
        o_cell_tables(models, ncells, i, ucl + o, (int)(ucl_off[i + 1] - o), mag, G, localtheta, squarelogit,
                      minlogprob, want_maxi, tab + o * G, maxi ? maxi + o : NULL, work);
    }
    free(work);
}

/* column index helper: T[c](:, counti(g,c)) */
#define TCOL(c, g) (tab + ((long)ucl_off[c] + counti[(long)(g) + (long)ngenes * (c)]) * G)

/* Phase B + C of logBootPosterior (src/jpmatLogBoot.cpp:213-331).
 * jp: ngenes x G col-major (already transposed as the reference returns). */
static void o_phaseB(const double* tab, const long* ucl_off, const int* counti, int ngenes, int ncells, int G,
                     int nboot, int seed, int ensemble, const int* batch_vals, const long* batch_off,
                     const int* comp, int nbatch, double* jp) {
    double* acc = (double*)calloc((size_t)G * ngenes, sizeof(double)); /* G x ngenes (jp before .t()) */
    double* tjp = (double*)malloc(sizeof(double) * (size_t)G * ngenes);
    o_rng g;
    int b, j, k, l;
    long kk;
    o_srand(&g, (unsigned int)seed);
    if (ensemble) {
        for (j = 0; j < ncells; j++) {
            long nu = ucl_off[j + 1] - ucl_off[j];
            double* ex = (double*)malloc(sizeof(double) * G * (size_t)nu);
            long u;
            for (u = 0; u < nu; u++) {
                const double* col = tab + (ucl_off[j] + u) * G;
                double s;
                for (k = 0; k < G; k++) ex[u * G + k] = exp(col[k]);
                s = arma_accu(ex + u * G, G, 1);
                for (k = 0; k < G; k++) ex[u * G + k] /= s;
            }
            for (l = 0; l < ngenes; l++) {
                const double* col = ex + (long)counti[(long)l + (long)ngenes * j] * G;
                for (k = 0; k < G; k++) acc[(long)l * G + k] += col[k];
            }
            free(ex);
        }
        for (l = 0; l < ngenes; l++) {
            double s = arma_accu(acc + (long)l * G, G, 1);
            for (k = 0; k < G; k++) acc[(long)l * G + k] /= s;
        }
    } else if (nboot == 0 && !batch_vals) {
        for (j = 0; j < ncells; j++)
            for (l = 0; l < ngenes; l++) {
                const double* col = TCOL(j, l);
                for (k = 0; k < G; k++) acc[(long)l * G + k] += col[k];
            }
        for (l = 0; l < ngenes; l++) {
            double* a = acc + (long)l * G;
            double m = arma_max(a, G, 1, NULL), s;
            for (k = 0; k < G; k++) a[k] -= m;
            for (k = 0; k < G; k++) a[k] = exp(a[k]);
            s = arma_accu(a, G, 1);
            for (k = 0; k < G; k++) a[k] /= s;
        }
    } else {
        for (b = 0; b < nboot; b++) {
            memset(tjp, 0, sizeof(double) * (size_t)G * ngenes);
            if (!batch_vals) {
                for (j = 0; j < ncells; j++) {
                    int rj = o_draw(&g, ncells);
                    for (l = 0; l < ngenes; l++) {
                        const double* col = TCOL(rj, l);
                        double* t = tjp + (long)l * G;
                        for (k = 0; k < G; k++) t[k] += col[k];
                    }
                }
            } else {
                int bk;
                for (bk = 0; bk < nbatch; bk++) {
                    int nsamp = comp[bk];
                    if (nsamp > 0) {
                        const int* bi = batch_vals + batch_off[bk];
                        int nbc = (int)(batch_off[bk + 1] - batch_off[bk]);
                        for (j = 0; j < nsamp; j++) {
                            int rj = o_draw(&g, nbc);
                            int cell = bi[rj];
                            for (l = 0; l < ngenes; l++) {
                                const double* col = TCOL(cell, l);
                                double* t = tjp + (long)l * G;
                                for (k = 0; k < G; k++) t[k] += col[k];
                            }
                        }
                    }
                }
            }
            for (l = 0; l < ngenes; l++) {
                double* t = tjp + (long)l * G;
                double m = arma_max(t, G, 1, NULL), s;
                for (k = 0; k < G; k++) t[k] -= m;
                for (k = 0; k < G; k++) t[k] = exp(t[k]);
                s = arma_accu(t, G, 1) * nboot;
                for (k = 0; k < G; k++) t[k] /= s;
                for (k = 0; k < G; k++) acc[(long)l * G + k] += t[k];
            }
        }
    }
    /* jp = jp.t()  -> ngenes x G col-major */
    for (l = 0; l < ngenes; l++)
        for (kk = 0; kk < G; kk++) jp[(long)l + (long)ngenes * kk] = acc[(long)l * G + kk];
    free(acc);
    free(tjp);
}

static void o_phaseC(const double* tab, const long* ucl_off, const int* maxi, const int* counti, int ngenes,
                     int ncells, int G, const double* mag, int returnpost, double* modes, double* post) {
    int i, j, k;
    if ((returnpost == 1 || returnpost == 3) && modes) {
        for (i = 0; i < ncells; i++)
            for (j = 0; j < ngenes; j++)
                modes[(long)j + (long)ngenes * i] = mag[maxi[ucl_off[i] + counti[(long)j + (long)ngenes * i]]];
    }
    if ((returnpost == 2 || returnpost == 3) && post) {
        for (i = 0; i < ncells; i++) {
            double* P = post + (long)i * ngenes * G; /* ngenes x G col-major */
            for (j = 0; j < ngenes; j++) {
                const double* col = TCOL(i, j);
                for (k = 0; k < G; k++) P[(long)j + (long)ngenes * k] = col[k];
            }
        }
    }
}

/* logBootPosterior  src/jpmatLogBoot.cpp:100-331.  Returns 0. */
int o_logBootPosterior(const double* models, int ncells, const int* ucl, const long* ucl_off, const int* counti,
                       int ngenes, const double* mag, int G, int nboot, int seed, int returnpost, int localtheta,
                       int squarelogit, int ensemble, double* jp, double* modes, double* post) {
    long tot = ucl_off[ncells];
    double* tab = (double*)malloc(sizeof(double) * (size_t)tot * G);
    int want_maxi = (returnpost == 1 || returnpost == 3);
    int* maxi = want_maxi ? (int*)malloc(sizeof(int) * (size_t)tot) : NULL;
    o_tables(models, ncells, ucl, ucl_off, mag, G, localtheta, squarelogit, want_maxi, tab, maxi);
    o_phaseB(tab, ucl_off, counti, ngenes, ncells, G, nboot, seed, ensemble, NULL, NULL, NULL, 0, jp);
    o_phaseC(tab, ucl_off, maxi, counti, ngenes, ncells, G, mag, returnpost, modes, post);
    free(tab);
    free(maxi);
    return 0;
}

/* logBootBatchPosterior  src/jpmatLogBoot.cpp:343-531 */
int o_logBootBatchPosterior(const double* models, int ncells, const int* ucl, const long* ucl_off,
                            const int* counti, int ngenes, const double* mag, int G, const int* batch_vals,
                            const long* batch_off, const int* comp, int nbatch, int nboot, int seed, int returnpost,
                            int localtheta, int squarelogit, double* jp, double* modes, double* post) {
    long tot = ucl_off[ncells];
    double* tab = (double*)malloc(sizeof(double) * (size_t)tot * G);
    int want_maxi = (returnpost == 1);
    int* maxi = want_maxi ? (int*)malloc(sizeof(int) * (size_t)tot) : NULL;
    o_tables(models, ncells, ucl, ucl_off, mag, G, localtheta, squarelogit, want_maxi, tab, maxi);
    o_phaseB(tab, ucl_off, counti, ngenes, ncells, G, nboot, seed, 0, batch_vals, batch_off, comp, nbatch, jp);
    o_phaseC(tab, ucl_off, maxi, counti, ngenes, ncells, G, mag, returnpost == 1 ? 1 : (returnpost == 2 ? 2 : 0),
             modes, post);
    free(tab);
    free(maxi);
    return 0;
}

/* row-wise softmax, jpmatLogBoot flavour (src/jpmatLogBoot.cpp:33-38) */
static void o_rowsoftmax_add(double* tjp, int nrows, int ncols, double* jp) {
    int r, c;
    for (r = 0; r < nrows; r++) {
        double m = arma_max(tjp + r, ncols, nrows, NULL), s;
        for (c = 0; c < ncols; c++) tjp[r + (long)nrows * c] -= m;
        for (c = 0; c < ncols; c++) tjp[r + (long)nrows * c] = exp(tjp[r + (long)nrows * c]);
        /* sum(tjp, 1): Armadillo accumulates row sums column by column */
        s = 0;
        for (c = 0; c < ncols; c++) s += tjp[r + (long)nrows * c];
        for (c = 0; c < ncols; c++) tjp[r + (long)nrows * c] /= s;
    }
    for (r = 0; r < nrows * ncols; r++) jp[r] += tjp[r];
}

/* jpmatLogBoot  src/jpmatLogBoot.cpp:11-42.  mats: nmat pointers to nrows x ncols col-major */
int o_jpmatLogBoot(const double* const* mats, int nmat, int nrows, int ncols, int nboot, int seed, double* jp) {
    long n = (long)nrows * ncols, e;
    double* tjp = (double*)malloc(sizeof(double) * n);
    o_rng g;
    int b, j;
    memset(jp, 0, sizeof(double) * n);
    o_srand(&g, (unsigned int)seed);
    for (b = 0; b < nboot; b++) {
        memset(tjp, 0, sizeof(double) * n);
        for (j = 0; j < nmat; j++) {
            int rj = o_draw(&g, nmat);
            for (e = 0; e < n; e++) tjp[e] += mats[rj][e];
        }
        o_rowsoftmax_add(tjp, nrows, ncols, jp);
    }
    free(tjp);
    return 0;
}

/* jpmatLogBatchBoot  src/jpmatLogBoot.cpp:48-86.  type k owns mats[type_off[k] .. type_off[k+1]) */
int o_jpmatLogBatchBoot(const double* const* mats, const int* type_off, const int* comp, int ntypes, int nrows,
                        int ncols, int nboot, int seed, double* jp) {
    long n = (long)nrows * ncols, e;
    double* tjp = (double*)malloc(sizeof(double) * n);
    o_rng g;
    int b, j, k;
    memset(jp, 0, sizeof(double) * n);
    o_srand(&g, (unsigned int)seed);
    for (b = 0; b < nboot; b++) {
        memset(tjp, 0, sizeof(double) * n);
        for (k = 0; k < ntypes; k++) {
            int nsamp = comp[k];
            if (nsamp > 0) {
                int nmat = type_off[k + 1] - type_off[k];
                for (j = 0; j < nsamp; j++) {
                    int rj = o_draw(&g, nmat);
                    const double* m = mats[type_off[k] + rj];
                    for (e = 0; e < n; e++) tjp[e] += m[e];
                }
            }
        }
        o_rowsoftmax_add(tjp, nrows, ncols, jp);
    }
    free(tjp);
    return 0;
}

/* matSlideMult  src/matSlideMult.cpp:5-23 ; out: nrows x (2n-1) col-major */
int o_matSlideMult(const double* m1, const double* m2, int nrows, int n, double* rm) {
    int i, r, t;
    /* left half: rm.col(n-i) = sum(m1.cols(0,n-i) % m2.cols(i-1,n-1), 1), i = n..2 */
    for (i = n; i > 1; i--) {
        int o = n - i, len = n - i + 1;
        for (r = 0; r < nrows; r++) {
            double s = 0;
            for (t = 0; t < len; t++) {
                double p = m1[r + (long)nrows * t] * m2[r + (long)nrows * (t + i - 1)];
                s += p;
            }
            rm[r + (long)nrows * o] = s;
        }
    }
    /* right half: rm.col(n-2+i) = sum(m1.cols(i-1,n-1) % m2.cols(0,n-i), 1), i = 1..n */
    for (i = 1; i <= n; i++) {
        int o = n - 2 + i, len = n - i + 1;
        for (r = 0; r < nrows; r++) {
            double s = 0;
            for (t = 0; t < len; t++) {
                double p = m1[r + (long)nrows * (t + i - 1)] * m2[r + (long)nrows * t];
                s += p;
            }
            rm[r + (long)nrows * o] = s;
        }
    }
    return 0;
}

/* calculate.ratio.posterior  R/functions.R:3491-3510 (n.cores = 1 form).
 * pmat1/pmat2 nrows x n col-major; prior_y (length n) or NULL to skip the
 * prior adjustment.  out: nrows x (2n-1), rows normalised by LDOUBLE rowSums. */
int o_ratio_posterior(const double* pmat1, const double* pmat2, const double* prior_y, int nrows, int n,
                      double* out) {
    long N = (long)nrows * n;
    double* a = (double*)malloc(sizeof(double) * N);
    double* b = (double*)malloc(sizeof(double) * N);
    long e;
    int r, c, m = 2 * n - 1;
    for (e = 0; e < N; e++) {
        int col = (int)(e / nrows);
        a[e] = prior_y ? pmat1[e] * prior_y[col] : pmat1[e];
        b[e] = prior_y ? pmat2[e] * prior_y[col] : pmat2[e];
    }
    o_matSlideMult(a, b, nrows, n, out);
    for (r = 0; r < nrows; r++) {
        long double s = 0;
        double sd;
        for (c = 0; c < m; c++) s += out[r + (long)nrows * c];
        sd = (double)s;
        for (c = 0; c < m; c++) out[r + (long)nrows * c] /= sd;
    }
    free(a);
    free(b);
    return 0;
}

/* ------------------------------------------------------------------ */
/* R qnorm (AS241) / pnorm (Cody), upper-tail, non-log                   */
/* ------------------------------------------------------------------ */
double o_qnorm(double p, int lower_tail) {
    double p_, q, r, val;
    if (isnan(p)) return p;
    if (p < 0 || p > 1) return NAN;
    if (p == 0) return lower_tail ? -INFINITY : INFINITY;
    if (p == 1) return lower_tail ? INFINITY : -INFINITY;
    p_ = lower_tail ? p : (0.5 - p + 0.5);
    q = p_ - 0.5;
    if (fabs(q) <= .425) {
        r = .180625 - q * q;
        val = q *
              (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
                   45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
                133.14166789178437745) * r + 3.387132872796366608) /
              (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
                   21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
                42.313330701600911252) * r + 1.);
        return val;
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

/* Cody's pnorm_both, returning the requested tail (R nmath pnorm.c) */
double o_pnorm(double x, int lower_tail) {
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
    static const double p[6] = {0.21589853405795699,     0.1274011611602473639, 0.022235277870649807,
                                0.001421619193227893466, 2.9112874951168792e-5, 0.02307344176494017303};
    static const double q[5] = {1.28426009614491121, 0.468238212480865118, 0.0659881378689285515,
                                0.00378239633202758244, 7.29751555083966205e-5};
    const double SIXTEN = 16, M_SQRT_32 = 5.656854249492380195206754896838, M_1_SQRT_2PI = 0.398942280401432677939946059934;
    double xden, xnum, temp, del, eps, xsq, y, cum, ccum;
    int i;
    if (isnan(x)) return x;
    eps = DBL_EPSILON * 0.5;
    y = fabs(x);
    if (y <= 0.67448975) {
        if (y > eps) {
            xsq = x * x;
            xnum = a[4] * xsq;
            xden = xsq;
            for (i = 0; i < 3; ++i) {
                xnum = (xnum + a[i]) * xsq;
                xden = (xden + b[i]) * xsq;
            }
        } else
            xnum = xden = 0.0;
        temp = x * (xnum + a[3]) / (xden + b[3]);
        cum = 0.5 + temp;
        ccum = 0.5 - temp;
    } else if (y <= M_SQRT_32) {
        xnum = c[8] * y;
        xden = y;
        for (i = 0; i < 7; ++i) {
            xnum = (xnum + c[i]) * y;
            xden = (xden + d[i]) * y;
        }
        temp = (xnum + c[7]) / (xden + d[7]);
        xsq = trunc(y * SIXTEN) / SIXTEN;
        del = (y - xsq) * (y + xsq);
        cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        ccum = 1.0 - cum;
        if (x > 0.) {
            temp = cum;
            cum = ccum;
            ccum = temp;
        }
    } else if ((-37.5193 < x && x < 8.2924) || (-8.2924 < x && x < 37.5193)) {
        xsq = 1.0 / (x * x);
        xnum = p[5] * xsq;
        xden = xsq;
        for (i = 0; i < 4; ++i) {
            xnum = (xnum + p[i]) * xsq;
            xden = (xden + q[i]) * xsq;
        }
        temp = xsq * (xnum + p[4]) / (xden + q[4]);
        temp = (M_1_SQRT_2PI - temp) / y;
        xsq = trunc(x * SIXTEN) / SIXTEN;
        del = (x - xsq) * (x + xsq);
        cum = exp(-xsq * xsq * 0.5) * exp(-del * 0.5) * temp;
        ccum = 1.0 - cum;
        if (x > 0.) {
            temp = cum;
            cum = ccum;
            ccum = temp;
        }
    } else {
        if (x > 0) {
            cum = 1.;
            ccum = 0.;
        } else {
            cum = 0.;
            ccum = 1.;
        }
    }
    return lower_tail ? cum : ccum;
}

/* quick.distribution.summary + get.ratio.posterior.Z.score
 * (R/functions.R:5039-5050, 3514-3531), scalar expectation.
 * rpost: nrows x m col-major (rows sum to 1); diffv: as.numeric(colnames).
 * out: nrows x 5 col-major  (lb, mle, ub, ce, Z).                          */
int o_summary(const double* rpost, int nrows, int m, const double* diffv, double expectation, double* out) {
    const double l10_2 = 0.30102999566398119521; /* log10(2) */
    /* quick.distribution.summary passes expectation/log2(10) (R/functions.R:5050) */
    double target = expectation / 3.32192809488736234787, best = INFINITY;
    int zi = 0, r, c;
    for (c = 0; c < m; c++) {
        double d = fabs(diffv[c] - target);
        if (d < best) {
            best = d;
            zi = c;
        }
    }
    for (r = 0; r < nrows; r++) {
        long double cs = 0;
        int mle = 0, lbi = 0, ubi = m - 1, found_ub = 0;
        double mx = -INFINITY, lb, ub, mlev, ce;
        long double tot = 0, gs = 0;
        double rs, zv, gsd, zl, zg, z;
        for (c = 0; c < m; c++) {
            double v = rpost[r + (long)nrows * c];
            double csd;
            if (v > mx) {
                mx = v;
                mle = c;
            }
            cs += v;
            csd = (double)cs;
            if (csd < 0.025) lbi = c;
            if (!found_ub && csd > (1 - 0.025)) {
                ubi = c;
                found_ub = 1;
            }
        }
        lb = diffv[lbi] / l10_2;
        mlev = diffv[mle] / l10_2;
        ub = diffv[ubi] / l10_2;
        ce = 0;
        if (lb > 0) ce = lb;
        if (ub < 0) ce = ub;
        /* Z score: rpost + min.p, renormalised by LDOUBLE rowSums */
        for (c = 0; c < m; c++) tot += (long double)(rpost[r + (long)nrows * c] + 1e-15);
        rs = (double)tot;
        /* rpost[, 1:(zi-1)]; for zi == 1 R's 1:0 selects column 1 */
        if (zi == 0)
            gs = (long double)((rpost[r] + 1e-15) / rs);
        for (c = 0; c < zi; c++) gs += (long double)((rpost[r + (long)nrows * c] + 1e-15) / rs);
        gsd = (double)gs;
        zv = (rpost[r + (long)nrows * zi] + 1e-15) / rs;
        zl = o_qnorm(gsd, 0);
        if (zl > 0) zl = 0;
        zg = o_qnorm(gsd + zv, 0);
        if (zg < 0) zg = 0;
        z = (fabs(zl) > fabs(zg)) ? zl : zg;
        out[r] = lb;
        out[r + (long)nrows] = mlev;
        out[r + 2L * nrows] = ub;
        out[r + 3L * nrows] = ce;
        out[r + 4L * nrows] = z;
    }
    return 0;
}

/* cZ = sign(Z) * qnorm(p.adjust(pnorm(|Z|, lower=F), "BH"), lower=F)   (R/functions.R:5051) */
static const double* cmp_p;
static int cmp_desc(const void* a, const void* b) {
    int i = *(const int*)a, j = *(const int*)b;
    double pi = cmp_p[i], pj = cmp_p[j];
    if (pi > pj) return -1;
    if (pi < pj) return 1;
    return (i < j) ? -1 : (i > j);
}
int o_bh_cz(const double* z, int n, double* cz) {
    /* p.adjust (R stats): NA p-values are dropped (p <- p[nna]) and stay NA; the default
     * n = length(p) is a promise forced after that subsetting, so n = lp = #non-NA;
     * `if (n <= 1) return(p0)` returns the unadjusted p (NAs included). */
    double* p = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    int* o = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    double* adj = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    double cm = INFINITY;
    int i, lp = 0;
    for (i = 0; i < n; i++) {
        p[i] = o_pnorm(fabs(z[i]), 0);
        adj[i] = p[i];
        if (!isnan(p[i])) o[lp++] = i;
    }
    cmp_p = p;
    qsort(o, lp, sizeof(int), cmp_desc); /* ties by index: R's order(decreasing=TRUE) is stable */
    if (lp > 1) {
        /* i <- lp:1L ; o <- order(p, decreasing = TRUE); pmin(1, cummin(n/i * p[o]))[ro] */
        for (i = 0; i < lp; i++) {
            double rank = (double)(lp - i);
            double v = ((double)lp / rank) * p[o[i]];
            if (v < cm) cm = v;
            adj[o[i]] = cm < 1 ? cm : 1;
        }
    }
    for (i = 0; i < n; i++) {
        double s = (z[i] > 0) ? 1.0 : (z[i] < 0 ? -1.0 : (isnan(z[i]) ? NAN : 0.0));
        cz[i] = s * o_qnorm(adj[i], 0);
    }
    free(p);
    free(o);
    free(adj);
    return 0;
}
