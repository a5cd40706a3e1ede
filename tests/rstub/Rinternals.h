/* TEST INFRASTRUCTURE: declarations of the R C API the shim uses, so that
 * tests/test_abi.py can syntax-check R/src/scde_hip_shim.c in a container without R.
 * Declarations only (no definitions); the real headers come with R. */
#ifndef SCDE_TEST_RINTERNALS_H
#define SCDE_TEST_RINTERNALS_H
#include <stddef.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
#define NA_INTEGER (-2147483647 - 1)
extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;
void Rf_error(const char*, ...);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
R_xlen_t XLENGTH(SEXP);
char* R_alloc(size_t, int);
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
SEXP Rf_coerceVector(SEXP, SEXPTYPE);
int* INTEGER(SEXP);
double* REAL(SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
SEXP Rf_allocVector(SEXPTYPE, R_xlen_t);
SEXP Rf_allocMatrix(SEXPTYPE, int, int);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP Rf_mkChar(const char*);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
SEXP Rf_mkNamed(SEXPTYPE, const char**);
#endif
