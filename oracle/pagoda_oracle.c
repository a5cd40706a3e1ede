/*
 * pagoda_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker).
 *
 * Loop-for-loop CPU restatement of scde's PAGODA helper kernels (src/pagoda.cpp), the
 * remaining .Call symbols of the package.  Imported only by tests/, never by the
 * product (scde_amd/).
 *
 *   o_winsorizeMatrix       src/pagoda.cpp:6-31
 *   o_matCorr               src/pagoda.cpp:33-38  (arma::cor(x, y))
 *   o_matWCorr              src/pagoda.cpp:41-65
 *   o_plSemicompleteCor2    src/pagoda.cpp:67-117
 *
 * Third-party arithmetic restated (absent from /root/reference; versions unpinned,
 * RcppArmadillo >= 0.5.400.2.0): Armadillo sort_index (ties are ordered by position
 * here; the reference's std::sort leaves them unspecified -- the result only depends on
 * it when trim > 1/2), dot (2 accumulators for n <= 32, reference-BLAS ddot above),
 * accu / sum (2 accumulators), cor (X'Y - sum(X)' sum(Y) / N, / (N - 1), / sd' sd) and
 * stddev (Armadillo's corrected two-pass variance).
 *
 * Matrices are R column-major.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double acc2(const double* x, long n) {
    double v1 = 0, v2 = 0;
    long i, j;
    for (i = 0, j = 1; j < n; i += 2, j += 2) {
        v1 += x[i];
        v2 += x[j];
    }
    if (i < n) v1 += x[i];
    return v1 + v2;
}

static double pdot(const double* a, const double* b, long n) {
    long i;
    if (n <= 32) {
        double v1 = 0, v2 = 0;
        long j;
        for (i = 0, j = 1; j < n; i += 2, j += 2) {
            v1 += a[i] * b[i];
            v2 += a[j] * b[j];
        }
        if (i < n) v1 += a[i] * b[i];
        return v1 + v2;
    } else {
        double t = 0;
        long m = n % 5;
        for (i = 0; i < m; i++) t += a[i] * b[i];
        for (i = m; i < n; i += 5)
            t = t + a[i] * b[i] + a[i + 1] * b[i + 1] + a[i + 2] * b[i + 2] + a[i + 3] * b[i + 3] +
                a[i + 4] * b[i + 4];
        return t;
    }
}

/* ---------------------------------------------------------------- winsorize */
static const double* g_row;
static int cmp_idx(const void* a, const void* b) {
    const int i = *(const int*)a, j = *(const int*)b;
    if (g_row[i] < g_row[j]) return -1;
    if (g_row[i] > g_row[j]) return 1;
    return (i > j) - (i < j);
}

/* mat: k rows x n cols.  ntr = round(n * trim) from each side of every row. */
void o_winsorizeMatrix(const double* mat, int k, int n, double trim, double* out) {
    const int ntr = (int)round(n * trim);
    int i, j;
    double* z = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
    int* o = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    memcpy(out, mat, sizeof(double) * (size_t)k * n);
    if (ntr == 0) {
        free(z);
        free(o);
        return;
    }
    for (i = 0; i < k; i++) {
        double minv, maxv;
        for (j = 0; j < n; j++) {
            z[j] = mat[i + (long)j * k];
            o[j] = j;
        }
        g_row = z;
        qsort(o, n, sizeof(int), cmp_idx);
        minv = z[o[ntr]];
        maxv = z[o[n - ntr - 1]];
        for (j = 0; j < ntr; j++) z[o[j]] = minv;
        for (j = n - ntr; j < n; j++) z[o[j]] = maxv;
        for (j = 0; j < n; j++) out[i + (long)j * k] = z[j];
    }
    free(z);
    free(o);
}

/* ---------------------------------------------------------------- matWCorr */
/* mat, w: k x n; out: n x n, identity with c(j, i) for j > i (upper triangle 0). */
void o_matWCorr(const double* mat, const double* w, int k, int n, double* out) {
    double* ic = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
    double* jc = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
    double* jw = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
    double* t = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
    int i, j, r;
    memset(out, 0, sizeof(double) * (size_t)n * n);
    for (i = 0; i < n; i++) out[i + (long)i * n] = 1.0;
    for (i = 0; i < n - 1; i++) {
        for (j = i + 1; j < n; j++) {
            const double* mi = mat + (long)i * k;
            const double* mj = mat + (long)j * k;
            const double* wi = w + (long)i * k;
            const double* wj = w + (long)j * k;
            double s, di, dj, nm, dn;
            for (r = 0; r < k; r++) {
                jw[r] = sqrt(wi[r] * wj[r]);
                ic[r] = mi[r];
                jc[r] = mj[r];
            }
            s = acc2(jw, k);
            for (r = 0; r < k; r++) jw[r] /= s;
            di = pdot(ic, jw, k);
            dj = pdot(jc, jw, k);
            for (r = 0; r < k; r++) {
                ic[r] -= di;
                jc[r] -= dj;
            }
            for (r = 0; r < k; r++) t[r] = ic[r] * jc[r];
            nm = pdot(t, jw, k);
            for (r = 0; r < k; r++) {
                ic[r] *= ic[r];
                jc[r] *= jc[r];
            }
            dn = pdot(ic, jw, k);
            dn *= pdot(jc, jw, k);
            out[j + (long)i * n] = nm / sqrt(dn);
        }
    }
    free(ic);
    free(jc);
    free(jw);
    free(t);
}

/* ---------------------------------------------------------------- matCorr */
/* Armadillo op_var::direct_var (norm_type 0): corrected two-pass */
static double arma_var(const double* x, long n) {
    long i;
    double mean, acc2v = 0, acc3 = 0;
    if (n < 2) return 0.0;
    mean = acc2(x, n) / (double)n;
    for (i = 0; i < n; i++) {
        const double tmp = mean - x[i];
        acc2v += tmp * tmp;
        acc3 += tmp;
    }
    return (acc2v - acc3 * acc3 / (double)n) / (double)(n - 1);
}

/* x: k x nx, y: k x ny -> out nx x ny = arma::cor(x, y) */
void o_matCorr(const double* x, int k, int nx, const double* y, int ny, double* out) {
    double* sx = (double*)malloc(sizeof(double) * (nx > 0 ? nx : 1));
    double* sy = (double*)malloc(sizeof(double) * (ny > 0 ? ny : 1));
    double* dx = (double*)malloc(sizeof(double) * (nx > 0 ? nx : 1));
    double* dy = (double*)malloc(sizeof(double) * (ny > 0 ? ny : 1));
    const double norm = k > 1 ? (double)(k - 1) : 1.0;
    int a, b;
    for (a = 0; a < nx; a++) {
        sx[a] = acc2(x + (long)a * k, k);
        dx[a] = sqrt(arma_var(x + (long)a * k, k));
    }
    for (b = 0; b < ny; b++) {
        sy[b] = acc2(y + (long)b * k, k);
        dy[b] = sqrt(arma_var(y + (long)b * k, k));
    }
    for (b = 0; b < ny; b++)
        for (a = 0; a < nx; a++) {
            double v = 0;
            long r;
            for (r = 0; r < k; r++) v += x[r + (long)a * k] * y[r + (long)b * k];
            v -= (sx[a] * sy[b]) / (double)k;
            v /= norm;
            out[a + (long)b * nx] = v / (dx[a] * dy[b]);
        }
    free(sx);
    free(sy);
    free(dx);
    free(dy);
}

/* ---------------------------------------------------------------- plSemicompleteCor2 */
/* list element p: idx[off[p] .. off[p+1]) (increasing gene indices), val (same range).
 * r: np x np (identity diagonal), n: np x np (0 diagonal). */
void o_plSemicompleteCor2(int np, const int64_t* off, const int* idx, const double* val, double* r, int* n) {
    int i, j;
    for (i = 0; i < np; i++)
        for (j = 0; j < np; j++) {
            r[i + (long)j * np] = i == j ? 1.0 : 0.0;
            n[i + (long)j * np] = 0;
        }
    for (i = 0; i < np; i++) {
        const int* i1 = idx + off[i];
        const double* v1 = val + off[i];
        const int v1s = (int)(off[i + 1] - off[i]);
        for (j = i + 1; j < np; j++) {
            const int* i2 = idx + off[j];
            const double* v2 = val + off[j];
            const int v2s = (int)(off[j + 1] - off[j]);
            int sgc = 0, k1, k2 = 0;
            double l12 = 0, l11 = 0, l22 = 0, cv;
            for (k1 = 0; k1 < v1s && v2s > 0; k1++) {
                const int id = i2[k2] - i1[k1];
                if (id == 0) {
                    sgc++;
                    l12 += v2[k2] * v1[k1];
                    l11 += v2[k2] * v2[k2];
                    l22 += v1[k1] * v1[k1];
                } else if (id < 0) {
                    do {
                        k2++;
                    } while (k2 < v2s && i2[k2] < i1[k1]);
                    if (k2 == v2s) break;
                    if (i2[k2] == i1[k1]) {
                        sgc++;
                        l12 += v2[k2] * v1[k1];
                        l11 += v2[k2] * v2[k2];
                        l22 += v1[k1] * v1[k1];
                    }
                }
            }
            cv = l11 * l22;
            if (cv > 0) cv = l12 / sqrt(cv);
            r[i + (long)j * np] = cv;
            r[j + (long)i * np] = cv;
            sgc = v1s + v2s - sgc;
            n[i + (long)j * np] = sgc;
            n[j + (long)i * np] = sgc;
        }
    }
}
