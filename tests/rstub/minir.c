/* TEST INFRASTRUCTURE: a minimal stand-in for the R C API the .Call shim
 * (R/src/scde_hip_shim.c) uses, so the tests can run the shim's entry points the way R's
 * .Call would -- on R-shaped objects (column-major matrices with dims, lists, integer and
 * logical scalars, named result lists) -- without R, which is absent from this image.
 * It implements only the semantics the shim relies on: allocation (never freed; the test
 * process is short), coercion between INTSXP / LGLSXP / REALSXP (NaN -> NA_integer_),
 * as.integer / as.numeric of scalars, dims, names, and Rf_error as a longjmp back to
 * minir_call, which reports the message.  Not product code; never loaded by it.
 * unif_rand draws R's Mersenne-Twister through the library's own restatement
 * (scde_r_set_seed / scde_r_unif_rand), seeded by minir_set_seed. */
#include <math.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "Rinternals.h"
#include "scde_hip.h"

#define NILSXP 0
#define SYMSXP 1
#define CHARSXP 9
#define LGLSXP 10

struct SEXPREC {
  SEXPTYPE type;
  R_xlen_t len;
  int nrow, ncol; /* -1: no dim attribute */
  void *data;
  SEXP names;
  char *str; /* CHARSXP */
};

static struct SEXPREC nil_obj = {NILSXP, 0, -1, -1, NULL, NULL, NULL};
static struct SEXPREC names_sym = {SYMSXP, 0, -1, -1, NULL, NULL, NULL};
SEXP R_NilValue = &nil_obj;
SEXP R_NamesSymbol = &names_sym;

static jmp_buf err_jmp;
static int err_armed = 0;
static char err_msg[2048];
static int protect_depth = 0;

void Rf_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err_msg, sizeof(err_msg), fmt, ap);
  va_end(ap);
  if (err_armed) longjmp(err_jmp, 1);
  fprintf(stderr, "minir: Rf_error outside minir_call: %s\n", err_msg);
  abort();
}

static size_t elt_size(SEXPTYPE t) {
  switch (t) {
    case INTSXP:
    case LGLSXP:
      return sizeof(int);
    case REALSXP:
      return sizeof(double);
    case STRSXP:
    case VECSXP:
      return sizeof(SEXP);
    default:
      return 1;
  }
}

SEXP Rf_allocVector(SEXPTYPE t, R_xlen_t n) {
  SEXP x = (SEXP)calloc(1, sizeof(struct SEXPREC));
  x->type = t;
  x->len = n;
  x->nrow = x->ncol = -1;
  x->data = calloc(n > 0 ? (size_t)n : 1, elt_size(t));
  if (t == STRSXP || t == VECSXP)
    for (R_xlen_t i = 0; i < n; i++) ((SEXP *)x->data)[i] = R_NilValue;
  x->names = R_NilValue;
  return x;
}

SEXP Rf_allocMatrix(SEXPTYPE t, int nr, int nc) {
  SEXP x = Rf_allocVector(t, (R_xlen_t)nr * nc);
  x->nrow = nr;
  x->ncol = nc;
  return x;
}

R_xlen_t XLENGTH(SEXP x) { return x->len; }
int *INTEGER(SEXP x) {
  if (x->type != INTSXP && x->type != LGLSXP) Rf_error("INTEGER() on a non-integer object (type %u)", x->type);
  return (int *)x->data;
}
double *REAL(SEXP x) {
  if (x->type != REALSXP) Rf_error("REAL() on a non-double object (type %u)", x->type);
  return (double *)x->data;
}
SEXP VECTOR_ELT(SEXP x, R_xlen_t i) {
  if (x->type != VECSXP || i < 0 || i >= x->len) Rf_error("VECTOR_ELT out of range");
  return ((SEXP *)x->data)[i];
}
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != VECSXP || i < 0 || i >= x->len) Rf_error("SET_VECTOR_ELT out of range");
  ((SEXP *)x->data)[i] = v;
  return v;
}
SEXP Rf_mkChar(const char *s) {
  SEXP x = Rf_allocVector(CHARSXP, 0);
  x->str = strdup(s);
  return x;
}
void SET_STRING_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != STRSXP || i < 0 || i >= x->len) Rf_error("SET_STRING_ELT out of range");
  ((SEXP *)x->data)[i] = v;
}
SEXP Rf_setAttrib(SEXP x, SEXP sym, SEXP v) {
  if (sym == R_NamesSymbol) x->names = v;
  return v;
}
int Rf_nrows(SEXP x) { return x->nrow >= 0 ? x->nrow : (int)x->len; }
int Rf_ncols(SEXP x) { return x->ncol >= 0 ? x->ncol : 1; }
SEXP Rf_protect(SEXP x) {
  protect_depth++;
  return x;
}
void Rf_unprotect(int n) { protect_depth -= n; }
char *R_alloc(size_t n, int size) { return (char *)calloc(n > 0 ? n : 1, (size_t)size); }

SEXP Rf_coerceVector(SEXP x, SEXPTYPE t) {
  if (x->type == t || (t == INTSXP && x->type == LGLSXP)) {
    if (x->type == t) return x;
  }
  if (x->type == NILSXP) return Rf_allocVector(t, 0);
  SEXP y = Rf_allocVector(t, x->len);
  y->nrow = x->nrow;
  y->ncol = x->ncol;
  y->names = x->names;
  for (R_xlen_t i = 0; i < x->len; i++) {
    if (t == REALSXP) {
      const int v = ((int *)x->data)[i];
      ((double *)y->data)[i] = (v == NA_INTEGER) ? NAN : (double)v;
    } else if (t == INTSXP) {
      if (x->type == REALSXP) {
        const double v = ((double *)x->data)[i];
        ((int *)y->data)[i] = (isnan(v) || fabs(v) >= 2147483648.0) ? NA_INTEGER : (int)v;
      } else {
        ((int *)y->data)[i] = ((int *)x->data)[i];
      }
    } else {
      Rf_error("minir: coercion to type %u not supported", t);
    }
  }
  return y;
}

int Rf_asInteger(SEXP x) {
  if (x->len < 1) return NA_INTEGER;
  if (x->type == INTSXP || x->type == LGLSXP) return ((int *)x->data)[0];
  if (x->type == REALSXP) {
    const double v = ((double *)x->data)[0];
    return isnan(v) ? NA_INTEGER : (int)v;
  }
  return NA_INTEGER;
}
double Rf_asReal(SEXP x) {
  if (x->len < 1) return NAN;
  if (x->type == REALSXP) return ((double *)x->data)[0];
  if (x->type == INTSXP || x->type == LGLSXP) {
    const int v = ((int *)x->data)[0];
    return v == NA_INTEGER ? NAN : (double)v;
  }
  return NAN;
}

SEXP Rf_mkNamed(SEXPTYPE t, const char **names) {
  int n = 0;
  while (names[n][0]) n++;
  SEXP x = Rf_allocVector(t, n);
  SEXP nm = Rf_allocVector(STRSXP, n);
  for (int i = 0; i < n; i++) SET_STRING_ELT(nm, i, Rf_mkChar(names[i]));
  x->names = nm;
  return x;
}

/* R's unif_rand through the library's restatement of R's Mersenne-Twister */
static uint32_t mt_state[625];
void minir_set_seed(unsigned seed) { (void)scde_r_set_seed(seed, mt_state); }
double unif_rand(void) {
  double u = 0.0;
  (void)scde_r_unif_rand(mt_state, 1, &u);
  return u;
}

/* ---- helpers for the Python side (ctypes) ---- */
SEXP minir_nil(void) { return R_NilValue; }
SEXP minir_real(R_xlen_t n, const double *v) {
  SEXP x = Rf_allocVector(REALSXP, n);
  if (n) memcpy(x->data, v, sizeof(double) * (size_t)n);
  return x;
}
SEXP minir_int(R_xlen_t n, const int *v) {
  SEXP x = Rf_allocVector(INTSXP, n);
  if (n) memcpy(x->data, v, sizeof(int) * (size_t)n);
  return x;
}
SEXP minir_lgl(int v) {
  SEXP x = Rf_allocVector(LGLSXP, 1);
  ((int *)x->data)[0] = v;
  return x;
}
SEXP minir_real_matrix(int nr, int nc, const double *v) {
  SEXP x = Rf_allocMatrix(REALSXP, nr, nc);
  if (nr > 0 && nc > 0) memcpy(x->data, v, sizeof(double) * (size_t)nr * nc);
  return x;
}
SEXP minir_int_matrix(int nr, int nc, const int *v) {
  SEXP x = Rf_allocMatrix(INTSXP, nr, nc);
  if (nr > 0 && nc > 0) memcpy(x->data, v, sizeof(int) * (size_t)nr * nc);
  return x;
}
SEXP minir_list(R_xlen_t n) { return Rf_allocVector(VECSXP, n); }
void minir_set(SEXP l, R_xlen_t i, SEXP v) { SET_VECTOR_ELT(l, i, v); }
int minir_type(SEXP x) { return (int)x->type; }
R_xlen_t minir_length(SEXP x) { return x->len; }
int minir_nrow(SEXP x) { return x->nrow; }
int minir_ncol(SEXP x) { return x->ncol; }
void *minir_data(SEXP x) { return x->data; }
SEXP minir_elt(SEXP x, R_xlen_t i) { return VECTOR_ELT(x, i); }
const char *minir_name(SEXP x, R_xlen_t i) {
  if (x->names == R_NilValue || i >= x->names->len) return "";
  return ((SEXP *)x->names->data)[i]->str;
}
const char *minir_error(void) { return err_msg; }
int minir_protect_depth(void) { return protect_depth; }

/* .Call(f, args...): the entry on SEXP arguments; NULL (with minir_error()) after Rf_error */
typedef SEXP (*sexpfn)();
SEXP minir_call(void *fp, int nargs, SEXP *a) {
  sexpfn f = (sexpfn)fp;
  err_msg[0] = 0;
  if (setjmp(err_jmp)) {
    err_armed = 0;
    return NULL;
  }
  err_armed = 1;
  SEXP r = NULL;
  switch (nargs) {
    case 1: r = f(a[0]); break;
    case 2: r = f(a[0], a[1]); break;
    case 3: r = f(a[0], a[1], a[2]); break;
    case 4: r = f(a[0], a[1], a[2], a[3]); break;
    case 5: r = f(a[0], a[1], a[2], a[3], a[4]); break;
    case 6: r = f(a[0], a[1], a[2], a[3], a[4], a[5]); break;
    case 7: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6]); break;
    case 8: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]); break;
    case 9: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8]); break;
    case 10: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9]); break;
    case 11: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10]); break;
    case 12: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11]); break;
    case 13: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12]); break;
    case 14: r = f(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9], a[10], a[11], a[12], a[13]); break;
    default: err_armed = 0; Rf_error("minir_call: %d arguments", nargs);
  }
  err_armed = 0;
  return r;
}
