/*
 * scde_hip_shim.c -- the .Call shim that makes libscde_hip.so a drop-in for scde's native
 * code (NAMESPACE:29 useDynLib(scde); symbols resolved by name, no R_registerRoutines).
 *
 * Layer 1 (same symbol names and argument lists as the reference, so R/functions.R runs
 * unchanged):
 *   logBootPosterior       src/jpmatLogBoot.cpp:100 (decl src/jpmatLogBoot.h:8)
 *   logBootBatchPosterior  src/jpmatLogBoot.cpp:343 (decl .h:9)
 *   jpmatLogBoot           src/jpmatLogBoot.cpp:11  (decl .h:6)
 *   jpmatLogBatchBoot      src/jpmatLogBoot.cpp:48  (decl .h:7)
 *   matSlideMult           src/matSlideMult.cpp:5   (decl src/matSlideMult.h:6)
 *   baileyWPCA             src/bwpca.cpp:59         (decl src/bwpca.h:8)
 *   winsorizeMatrix, matWCorr, plSemicompleteCor2, matCorr  src/pagoda.cpp (decl src/pagoda.h:5-8)
 * Layer 2 (the fused device path behind R/scde_hip.R's wrappers):
 *   scde_hip_expression_difference, scde_hip_expression_difference_batch, scde_hip_posteriors,
 *   scde_hip_varnorm_weights
 *
 * Build: src/Makevars adds -I$(SCDE_HIP_HOME)/include and -lscde_hip.
 * Errors from the library become Rf_error; there is no CPU fallback.
 */
#include <R.h>
#include <Rmath.h> /* unif_rand */
#include <Rinternals.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "scde_hip.h"

static void chk(int rc) { if (rc != SCDE_OK) Rf_error("scde_hip: %s", scde_last_error()); }
static int as_int(SEXP x) { return Rf_asInteger(x); }   /* numeric or logical scalars, like Rcpp::as<int> */

/* VECSXP of integer (or double) vectors -> concatenated int values + offsets[n+1] */
static void flatten_ilist(SEXP l, int **vals, int64_t **off) {
  R_xlen_t n = XLENGTH(l), tot = 0;
  *off = (int64_t *) R_alloc(n + 1, sizeof(int64_t));
  (*off)[0] = 0;
  for (R_xlen_t i = 0; i < n; i++) { tot += XLENGTH(VECTOR_ELT(l, i)); (*off)[i + 1] = tot; }
  *vals = (int *) R_alloc(tot > 0 ? tot : 1, sizeof(int));
  for (R_xlen_t i = 0; i < n; i++) {
    if (XLENGTH(VECTOR_ELT(l, i)) == 0) continue;  /* tapply's NULL for an empty level */
    SEXP v = PROTECT(Rf_coerceVector(VECTOR_ELT(l, i), INTSXP));
    memcpy(*vals + (*off)[i], INTEGER(v), sizeof(int) * XLENGTH(v));
    UNPROTECT(1);
  }
}

/* CountsI arrives as a REALSXP (match(...) - 1); the reference coerces it to int. */
static int *as_int_matrix(SEXP m) {
  SEXP v = PROTECT(Rf_coerceVector(m, INTSXP));
  int *out = (int *) R_alloc(XLENGTH(v) > 0 ? XLENGTH(v) : 1, sizeof(int));
  memcpy(out, INTEGER(v), sizeof(int) * XLENGTH(v));
  UNPROTECT(1);
  return out;
}

/* list(jp=, modes=, post=) exactly as src/jpmatLogBoot.cpp:287-288, 302-303, 325-327 */
static SEXP pack(SEXP jp, SEXP modes, SEXP post, int postflag) {
  if (postflag == 0) return jp;
  int n = 1 + (modes != R_NilValue) + (post != R_NilValue);
  SEXP out = PROTECT(Rf_allocVector(VECSXP, n)), nm = PROTECT(Rf_allocVector(STRSXP, n));
  int i = 0;
  SET_VECTOR_ELT(out, i, jp); SET_STRING_ELT(nm, i++, Rf_mkChar("jp"));
  if (modes != R_NilValue) { SET_VECTOR_ELT(out, i, modes); SET_STRING_ELT(nm, i++, Rf_mkChar("modes")); }
  if (post != R_NilValue) { SET_VECTOR_ELT(out, i, post); SET_STRING_ELT(nm, i++, Rf_mkChar("post")); }
  Rf_setAttrib(out, R_NamesSymbol, nm);
  UNPROTECT(2);
  return out;
}

static SEXP alloc_post(int ncells, int ngenes, int ngrid, double **buf) {
  /* the library writes ncells consecutive ngenes x ngrid blocks; R wants a list of matrices */
  *buf = (double *) R_alloc((size_t) ncells * ngenes * ngrid > 0 ? (size_t) ncells * ngenes * ngrid : 1,
                            sizeof(double));
  return Rf_allocVector(VECSXP, ncells);
}
static void fill_post(SEXP post, const double *buf, int ncells, int ngenes, int ngrid) {
  for (int c = 0; c < ncells; c++) {
    SEXP m = Rf_allocMatrix(REALSXP, ngenes, ngrid);
    SET_VECTOR_ELT(post, c, m);
    memcpy(REAL(m), buf + (size_t) c * ngenes * ngrid, sizeof(double) * (size_t) ngenes * ngrid);
  }
}

SEXP logBootPosterior(SEXP Models, SEXP Ucl, SEXP CountsI, SEXP Magnitudes, SEXP Nboot, SEXP Seed,
                      SEXP ReturnIndividualPosteriors, SEXP LocalThetaFit, SEXP SquareLogitConc,
                      SEXP EnsembleProbability) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), mag = PROTECT(Rf_coerceVector(Magnitudes, REALSXP));
  int ncells = Rf_nrows(Models), ngenes = Rf_nrows(CountsI), ngrid = XLENGTH(mag);
  int postflag = as_int(ReturnIndividualPosteriors);
  int *uv; int64_t *uo; flatten_ilist(Ucl, &uv, &uo);
  int *ci = as_int_matrix(CountsI);
  SEXP jp = PROTECT(Rf_allocMatrix(REALSXP, ngenes, ngrid));
  SEXP modes = R_NilValue, post = R_NilValue; double *pbuf = NULL;
  if (postflag == 1 || postflag == 3) modes = Rf_allocMatrix(REALSXP, ngenes, ncells);
  PROTECT(modes);
  if (postflag == 2 || postflag == 3) post = alloc_post(ncells, ngenes, ngrid, &pbuf);
  PROTECT(post);
  chk(scde_logBootPosterior(REAL(mm), ncells, uv, uo, ci, ngenes, REAL(mag), ngrid, as_int(Nboot), as_int(Seed),
                            postflag, as_int(LocalThetaFit), as_int(SquareLogitConc), as_int(EnsembleProbability),
                            REAL(jp), modes == R_NilValue ? NULL : REAL(modes), pbuf));
  if (post != R_NilValue) fill_post(post, pbuf, ncells, ngenes, ngrid);
  SEXP out = pack(jp, modes, post, postflag);
  UNPROTECT(5);
  return out;
}

SEXP logBootBatchPosterior(SEXP Models, SEXP Ucl, SEXP CountsI, SEXP Magnitudes, SEXP BatchIL, SEXP Composition,
                           SEXP Nboot, SEXP Seed, SEXP ReturnIndividualPosteriors, SEXP LocalThetaFit,
                           SEXP SquareLogitConc) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), mag = PROTECT(Rf_coerceVector(Magnitudes, REALSXP));
  SEXP comp = PROTECT(Rf_coerceVector(Composition, INTSXP));
  int ncells = Rf_nrows(Models), ngenes = Rf_nrows(CountsI), ngrid = XLENGTH(mag);
  int postflag = as_int(ReturnIndividualPosteriors);
  int *uv, *bv; int64_t *uo, *bo;
  flatten_ilist(Ucl, &uv, &uo);
  flatten_ilist(BatchIL, &bv, &bo);
  int *ci = as_int_matrix(CountsI);
  SEXP jp = PROTECT(Rf_allocMatrix(REALSXP, ngenes, ngrid));
  /* the reference handles postflag 1 and 2 only (src/jpmatLogBoot.cpp:499-530) */
  SEXP modes = R_NilValue, post = R_NilValue; double *pbuf = NULL;
  if (postflag == 1) modes = Rf_allocMatrix(REALSXP, ngenes, ncells);
  PROTECT(modes);
  if (postflag == 2) post = alloc_post(ncells, ngenes, ngrid, &pbuf);
  PROTECT(post);
  chk(scde_logBootBatchPosterior(REAL(mm), ncells, uv, uo, ci, ngenes, REAL(mag), ngrid, bv, bo, INTEGER(comp),
                                 XLENGTH(comp), as_int(Nboot), as_int(Seed), postflag, as_int(LocalThetaFit),
                                 as_int(SquareLogitConc), REAL(jp), modes == R_NilValue ? NULL : REAL(modes), pbuf));
  if (post != R_NilValue) fill_post(post, pbuf, ncells, ngenes, ngrid);
  SEXP out = pack(jp, modes, post, (postflag == 1 || postflag == 2) ? postflag : 0);
  UNPROTECT(6);
  return out;
}

SEXP jpmatLogBoot(SEXP Matl, SEXP Nboot, SEXP Seed) {
  int nmat = XLENGTH(Matl);
  if (nmat == 0) Rf_error("jpmatLogBoot: empty list");
  const double **mats = (const double **) R_alloc(nmat, sizeof(double *));
  int nr = Rf_nrows(VECTOR_ELT(Matl, 0)), nc = Rf_ncols(VECTOR_ELT(Matl, 0));
  for (int i = 0; i < nmat; i++) mats[i] = REAL(VECTOR_ELT(Matl, i));
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, nr, nc));
  chk(scde_jpmatLogBoot(mats, nmat, nr, nc, as_int(Nboot), as_int(Seed), REAL(out)));
  UNPROTECT(1);
  return out;
}

SEXP jpmatLogBatchBoot(SEXP Matll, SEXP Comp, SEXP Nboot, SEXP Seed) {
  int nt = XLENGTH(Matll), tot = 0;
  int *off = (int *) R_alloc(nt + 1, sizeof(int));
  off[0] = 0;
  for (int k = 0; k < nt; k++) { tot += XLENGTH(VECTOR_ELT(Matll, k)); off[k + 1] = tot; }
  if (tot == 0) Rf_error("jpmatLogBatchBoot: empty list");
  const double **mats = (const double **) R_alloc(tot, sizeof(double *));
  for (int k = 0; k < nt; k++)
    for (int j = 0; j < off[k + 1] - off[k]; j++) mats[off[k] + j] = REAL(VECTOR_ELT(VECTOR_ELT(Matll, k), j));
  SEXP comp = PROTECT(Rf_coerceVector(Comp, INTSXP));
  /* the output shape comes from the first non-empty sublist (tot > 0: one exists) */
  int k0 = 0;
  while (off[k0 + 1] == off[k0]) k0++;
  SEXP m0 = VECTOR_ELT(VECTOR_ELT(Matll, k0), 0);
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, Rf_nrows(m0), Rf_ncols(m0)));
  chk(scde_jpmatLogBatchBoot(mats, off, INTEGER(comp), nt, Rf_nrows(m0), Rf_ncols(m0), as_int(Nboot),
                             as_int(Seed), REAL(out)));
  UNPROTECT(2);
  return out;
}

SEXP matSlideMult(SEXP Mat1, SEXP Mat2) {
  int nr = Rf_nrows(Mat1), nc = Rf_ncols(Mat1);
  if (Rf_nrows(Mat2) != nr || Rf_ncols(Mat2) != nc) Rf_error("matSlideMult: shapes differ");
  SEXP a = PROTECT(Rf_coerceVector(Mat1, REALSXP)), b = PROTECT(Rf_coerceVector(Mat2, REALSXP));
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, nr, 2 * nc - 1));
  chk(scde_matSlideMult(REAL(a), REAL(b), nr, nc, REAL(out)));
  UNPROTECT(3);
  return out;
}

/* ---------------------------------------------------------------- weighted PCA */
SEXP baileyWPCA(SEXP Mat, SEXP Matw, SEXP Npcs, SEXP Nstarts, SEXP Smooth, SEXP EMtol, SEXP EMmaxiter,
                SEXP Seed, SEXP Nshuffles) {
  SEXP m = PROTECT(Rf_coerceVector(Mat, REALSXP)), w = PROTECT(Rf_coerceVector(Matw, REALSXP));
  const int n = Rf_nrows(m), d = Rf_ncols(m);
  if (Rf_nrows(w) != n || Rf_ncols(w) != d) Rf_error("baileyWPCA: Mat and Matw differ in shape");
  int npcs = as_int(Npcs); if (npcs > d) npcs = d;            /* bwpca.cpp:77 */
  const int nstarts = as_int(Nstarts), nsh = as_int(Nshuffles);
  (void) Seed;                                                /* arma_rng::set_seed: no-op */
  const R_xlen_t nu = (R_xlen_t)(1 + nsh) * nstarts * d * npcs;
  double *starts = (double *) R_alloc(nu, sizeof(double));
  for (R_xlen_t i = 0; i < nu; i++) starts[i] = unif_rand();  /* randu's draw order */
  int *perms = NULL;
  if (nsh > 0) {                                              /* set_random_matrices */
    perms = (int *) R_alloc((R_xlen_t) nsh * d * n, sizeof(int));
    int *ind = (int *) R_alloc(n, sizeof(int));
    for (int s = 0; s < nsh; s++) {
      for (int i = 0; i < n; i++) ind[i] = i;
      for (int c = 0; c < d; c++) {
        for (int i = 1; i < n; i++) { int j = rand() % (i + 1); if (i != j) { int t = ind[i]; ind[i] = ind[j]; ind[j] = t; } }
        memcpy(perms + ((R_xlen_t) s * d + c) * n, ind, sizeof(int) * n);
      }
    }
  }
  SEXP rot = PROTECT(Rf_allocMatrix(REALSXP, d, npcs)), sco = PROTECT(Rf_allocMatrix(REALSXP, n, npcs));
  SEXP pcw = PROTECT(Rf_allocMatrix(REALSXP, n, npcs)), var = PROTECT(Rf_allocVector(REALSXP, npcs));
  SEXP tot = PROTECT(Rf_allocVector(REALSXP, 1)), rv = PROTECT(Rf_allocVector(REALSXP, nsh > 0 ? nsh : 0));
  chk(scde_baileyWPCA(REAL(m), REAL(w), n, d, npcs, nstarts, as_int(Smooth), Rf_asReal(EMtol), as_int(EMmaxiter),
                      starts, nsh, perms, REAL(rot), REAL(sco), REAL(pcw), REAL(var), REAL(tot),
                      nsh > 0 ? REAL(rv) : NULL));
  const char *nm[] = {"rotation", "scores", "scoreweights", "var", "totvar", "randvar", ""};
  if (nsh == 0) nm[5] = "";
  SEXP out = PROTECT(Rf_mkNamed(VECSXP, nm));
  SET_VECTOR_ELT(out, 0, rot); SET_VECTOR_ELT(out, 1, sco); SET_VECTOR_ELT(out, 2, pcw);
  SET_VECTOR_ELT(out, 3, var); SET_VECTOR_ELT(out, 4, tot);
  if (nsh > 0) SET_VECTOR_ELT(out, 5, rv);
  UNPROTECT(9);
  return out;
}

/* ---------------------------------------------------------------- PAGODA helpers */
SEXP winsorizeMatrix(SEXP Mat, SEXP Trim) {
  SEXP m = PROTECT(Rf_coerceVector(Mat, REALSXP));
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, Rf_nrows(m), Rf_ncols(m)));
  chk(scde_winsorizeMatrix(REAL(m), Rf_nrows(m), Rf_ncols(m), Rf_asReal(Trim), REAL(out)));
  UNPROTECT(2);
  return out;
}

SEXP matWCorr(SEXP Mat, SEXP Matw) {
  SEXP m = PROTECT(Rf_coerceVector(Mat, REALSXP)), w = PROTECT(Rf_coerceVector(Matw, REALSXP));
  const int k = Rf_nrows(m), n = Rf_ncols(m);
  if (Rf_nrows(w) != k || Rf_ncols(w) != n) Rf_error("matWCorr: Mat and Matw differ in shape");
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, n, n));
  chk(scde_matWCorr(REAL(m), REAL(w), k, n, REAL(out)));
  UNPROTECT(3);
  return out;
}

SEXP matCorr(SEXP X, SEXP Y) {
  SEXP x = PROTECT(Rf_coerceVector(X, REALSXP)), y = PROTECT(Rf_coerceVector(Y, REALSXP));
  if (Rf_nrows(x) != Rf_nrows(y)) Rf_error("matCorr: row counts differ");
  SEXP out = PROTECT(Rf_allocMatrix(REALSXP, Rf_ncols(x), Rf_ncols(y)));
  chk(scde_matCorr(REAL(x), Rf_nrows(x), Rf_ncols(x), REAL(y), Rf_ncols(y), REAL(out)));
  UNPROTECT(3);
  return out;
}

SEXP plSemicompleteCor2(SEXP Pl) {   /* list of list(i = <numeric>, v = <numeric>) */
  const int np = (int) XLENGTH(Pl);
  int64_t *off = (int64_t *) R_alloc(np + 1, sizeof(int64_t));
  off[0] = 0;
  for (int p = 0; p < np; p++) off[p + 1] = off[p] + XLENGTH(VECTOR_ELT(VECTOR_ELT(Pl, p), 1));
  int *idx = (int *) R_alloc(off[np] > 0 ? off[np] : 1, sizeof(int));
  double *val = (double *) R_alloc(off[np] > 0 ? off[np] : 1, sizeof(double));
  for (int p = 0; p < np; p++) {
    SEXP i = PROTECT(Rf_coerceVector(VECTOR_ELT(VECTOR_ELT(Pl, p), 0), REALSXP));
    SEXP v = PROTECT(Rf_coerceVector(VECTOR_ELT(VECTOR_ELT(Pl, p), 1), REALSXP));
    for (int64_t e = 0; e < off[p + 1] - off[p]; e++) { idx[off[p] + e] = (int) REAL(i)[e]; val[off[p] + e] = REAL(v)[e]; }
    UNPROTECT(2);
  }
  SEXP r = PROTECT(Rf_allocMatrix(REALSXP, np, np)), n = PROTECT(Rf_allocMatrix(INTSXP, np, np));
  chk(scde_plSemicompleteCor2(np, off, idx, val, REAL(r), INTEGER(n)));
  const char *nm[] = {"r", "n", ""};
  SEXP out = PROTECT(Rf_mkNamed(VECSXP, nm));
  SET_VECTOR_ELT(out, 0, r); SET_VECTOR_ELT(out, 1, n);
  UNPROTECT(3);
  return out;
}

/* ---------------------------------------------------------------- layer 2: fused device path */
/* models: the R `mm` matrix (ncells x 12, NA where absent, R/functions.R:601-604); counts: the
 * integer genes x cells matrix with columns in model-row order. */
SEXP scde_hip_expression_difference(SEXP Models, SEXP Counts, SEXP PriorX, SEXP PriorY, SEXP Groups,
                                    SEXP Nboot, SEXP NCores, SEXP LocalTheta, SEXP SquareLogitConc,
                                    SEXP Expectation, SEXP ReturnPosteriors) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), px = PROTECT(Rf_coerceVector(PriorX, REALSXP));
  SEXP py = PROTECT(Rf_coerceVector(PriorY, REALSXP)), gr = PROTECT(Rf_coerceVector(Groups, INTSXP));
  SEXP ci = PROTECT(Rf_coerceVector(Counts, INTSXP));
  const int *counts = INTEGER(ci);
  const int ngenes = Rf_nrows(Counts), ncells = Rf_ncols(Counts), G = XLENGTH(px);
  int *codes = (int *) R_alloc(ncells, sizeof(int));
  for (int c = 0; c < ncells; c++) codes[c] = INTEGER(gr)[c] == NA_INTEGER ? -1 : INTEGER(gr)[c] - 1;  /* factor codes */
  scde_de_params p;
  memset(&p, 0, sizeof(p));
  p.ncells = ncells; p.models = REAL(mm); p.local_theta = as_int(LocalTheta); p.square_logit_conc = as_int(SquareLogitConc);
  p.groups = codes; p.prior_x = REAL(px); p.prior_y = REAL(py); p.ngrid = G; p.nboot = as_int(Nboot);
  p.n_cores = as_int(NCores); p.gene_offset = 0; p.ngenes_total = ngenes; p.expectation = Rf_asReal(Expectation);
  p.rand_kind = scde_get_rand_kind(); p.compute_cz = 1;
  const int rp = as_int(ReturnPosteriors);
  SEXP res = PROTECT(Rf_allocMatrix(REALSXP, ngenes, 6));
  SEXP jp1 = rp ? Rf_allocMatrix(REALSXP, ngenes, G) : R_NilValue;
  PROTECT(jp1);
  SEXP jp2 = rp ? Rf_allocMatrix(REALSXP, ngenes, G) : R_NilValue;
  PROTECT(jp2);
  SEXP ratio = rp ? Rf_allocMatrix(REALSXP, ngenes, 2 * G - 1) : R_NilValue;
  PROTECT(ratio);
  chk(scde_expression_difference_host(NULL, counts, ngenes, ngenes, &p, REAL(res), rp ? REAL(jp1) : NULL,
                                      rp ? REAL(jp2) : NULL, rp ? REAL(ratio) : NULL));
  const char *nm[] = {"results", "jp1", "jp2", "ratio", ""};
  SEXP out = PROTECT(Rf_mkNamed(VECSXP, nm));
  SET_VECTOR_ELT(out, 0, res); SET_VECTOR_ELT(out, 1, jp1); SET_VECTOR_ELT(out, 2, jp2); SET_VECTOR_ELT(out, 3, ratio);
  UNPROTECT(10);
  return out;
}

/* Batch-corrected scde.expression.difference (R/functions.R:321-399) in one call.  Groups and
 * Batch are factor codes by model row (1-based, NA allowed: such cells join no group / no batch
 * level, as tapply and table drop them); NBatch = nlevels(batch).  Returns the three N x 6
 * summaries (batch.adjusted, results, batch.effect) and, with ReturnPosteriors, the group
 * difference posterior (N x 2G-1), the batch-adjusted one (N x 4G-3) and both joint posteriors. */
SEXP scde_hip_expression_difference_batch(SEXP Models, SEXP BatchModels, SEXP Counts, SEXP PriorX, SEXP PriorY,
                                          SEXP Groups, SEXP Batch, SEXP NBatch, SEXP Nboot, SEXP NCores,
                                          SEXP LocalTheta, SEXP SquareLogitConc, SEXP Expectation,
                                          SEXP ReturnPosteriors) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), bmm = PROTECT(Rf_coerceVector(BatchModels, REALSXP));
  SEXP px = PROTECT(Rf_coerceVector(PriorX, REALSXP)), py = PROTECT(Rf_coerceVector(PriorY, REALSXP));
  SEXP gr = PROTECT(Rf_coerceVector(Groups, INTSXP)), bt = PROTECT(Rf_coerceVector(Batch, INTSXP));
  SEXP ci = PROTECT(Rf_coerceVector(Counts, INTSXP));
  const int ngenes = Rf_nrows(Counts), ncells = Rf_ncols(Counts), G = XLENGTH(px), nb = as_int(NBatch);
  if (XLENGTH(gr) != ncells || XLENGTH(bt) != ncells) Rf_error("scde_hip: groups/batch length differs from the cell count");
  if (Rf_nrows(mm) != ncells || Rf_nrows(bmm) != ncells) Rf_error("scde_hip: model rows differ from the cell count");
  int *codes = (int *) R_alloc(ncells, sizeof(int)), *bcodes = (int *) R_alloc(ncells, sizeof(int));
  for (int c = 0; c < ncells; c++) {
    codes[c] = INTEGER(gr)[c] == NA_INTEGER ? -1 : INTEGER(gr)[c] - 1;
    bcodes[c] = INTEGER(bt)[c] == NA_INTEGER ? -1 : INTEGER(bt)[c] - 1;
  }
  scde_de_params p;
  memset(&p, 0, sizeof(p));
  p.ncells = ncells; p.models = REAL(mm); p.local_theta = as_int(LocalTheta); p.square_logit_conc = as_int(SquareLogitConc);
  p.groups = codes; p.prior_x = REAL(px); p.prior_y = REAL(py); p.ngrid = G; p.nboot = as_int(Nboot);
  p.n_cores = as_int(NCores); p.gene_offset = 0; p.ngenes_total = ngenes; p.expectation = Rf_asReal(Expectation);
  p.rand_kind = scde_get_rand_kind(); p.compute_cz = 1;
  const int rp = as_int(ReturnPosteriors), m = 2 * G - 1;
  double *res = (double *) R_alloc((size_t) 18 * ngenes > 0 ? (size_t) 18 * ngenes : 1, sizeof(double));
  SEXP jp1 = PROTECT(rp ? Rf_allocMatrix(REALSXP, ngenes, G) : R_NilValue);
  SEXP jp2 = PROTECT(rp ? Rf_allocMatrix(REALSXP, ngenes, G) : R_NilValue);
  SEXP ratio = PROTECT(rp ? Rf_allocMatrix(REALSXP, ngenes, m) : R_NilValue);
  SEXP aratio = PROTECT(rp ? Rf_allocMatrix(REALSXP, ngenes, 2 * m - 1) : R_NilValue);
  chk(scde_expression_difference_batch_host(NULL, INTEGER(ci), ngenes, ngenes, &p, REAL(bmm), bcodes, nb, res,
                                            rp ? REAL(jp1) : NULL, rp ? REAL(jp2) : NULL, rp ? REAL(ratio) : NULL,
                                            rp ? REAL(aratio) : NULL, NULL));
  SEXP tabs[3];
  for (int t = 0; t < 3; t++) {
    tabs[t] = PROTECT(Rf_allocMatrix(REALSXP, ngenes, 6));
    memcpy(REAL(tabs[t]), res + (size_t) t * 6 * ngenes, sizeof(double) * 6 * (size_t) ngenes);
  }
  const char *nm[] = {"batch.adjusted", "results", "batch.effect", "jp1", "jp2", "ratio", "adj.ratio", ""};
  SEXP out = PROTECT(Rf_mkNamed(VECSXP, nm));
  for (int t = 0; t < 3; t++) SET_VECTOR_ELT(out, t, tabs[t]);
  SET_VECTOR_ELT(out, 3, jp1); SET_VECTOR_ELT(out, 4, jp2); SET_VECTOR_ELT(out, 5, ratio); SET_VECTOR_ELT(out, 6, aratio);
  UNPROTECT(15);
  return out;
}

/* scde.posteriors (R/functions.R:566-669) in one call.  BatchIL / Composition: R_NilValue, or the
 * reference's batchil <- tapply(c(1:nrow(models)) - 1, batch, I) (0-based model rows per batch
 * level, R/functions.R:570) and the composition vector (draws per boot per level, 568-569), as
 * the reference passes them to logBootBatchPosterior (613, 635).  As there, a batch call returns
 * modes for postflag 1 and the individual posteriors for postflag 2 only (src/jpmatLogBoot.cpp:
 * 499-530); postflag 3 returns jp. */
SEXP scde_hip_posteriors(SEXP Models, SEXP Counts, SEXP PriorX, SEXP Nboot, SEXP NCores, SEXP LocalTheta,
                         SEXP SquareLogitConc, SEXP PostFlag, SEXP Ensemble, SEXP BatchIL, SEXP Composition) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), px = PROTECT(Rf_coerceVector(PriorX, REALSXP));
  SEXP ci = PROTECT(Rf_coerceVector(Counts, INTSXP));
  const int *counts = INTEGER(ci);
  const int ngenes = Rf_nrows(Counts), ncells = Rf_ncols(Counts), G = XLENGTH(px);
  const int postflag = as_int(PostFlag);
  const int batch = BatchIL != R_NilValue;
  int *bv = NULL, nbatch = 0; int64_t *bo = NULL;
  SEXP comp = PROTECT(batch ? Rf_coerceVector(Composition, INTSXP) : R_NilValue);
  if (batch) {
    nbatch = (int) XLENGTH(comp);
    if (XLENGTH(BatchIL) != nbatch) Rf_error("scde_hip: composition has %d levels, batch %d", nbatch, (int) XLENGTH(BatchIL));
    flatten_ilist(BatchIL, &bv, &bo);
  }
  int *cellidx = (int *) R_alloc(ncells, sizeof(int));
  for (int c = 0; c < ncells; c++) cellidx[c] = c;
  const int want_modes = batch ? postflag == 1 : (postflag == 1 || postflag == 3);
  const int want_post = batch ? postflag == 2 : (postflag == 2 || postflag == 3);
  SEXP jp = PROTECT(Rf_allocMatrix(REALSXP, ngenes, G));
  SEXP modes = want_modes ? Rf_allocMatrix(REALSXP, ngenes, ncells) : R_NilValue;
  PROTECT(modes);
  SEXP post = R_NilValue; double *pbuf = NULL;
  if (want_post) post = alloc_post(ncells, ngenes, G, &pbuf);
  PROTECT(post);
  chk(scde_posteriors_host(NULL, counts, ngenes, ngenes, ncells, cellidx, ncells, REAL(mm), as_int(LocalTheta),
                           as_int(SquareLogitConc), REAL(px), G, as_int(Nboot), as_int(NCores), 0, ngenes, postflag,
                           as_int(Ensemble), bv, bo, batch ? INTEGER(comp) : NULL, nbatch, REAL(jp),
                           modes == R_NilValue ? NULL : REAL(modes), pbuf));
  if (post != R_NilValue) fill_post(post, pbuf, ncells, ngenes, G);
  SEXP out = pack(jp, modes, post, batch ? ((postflag == 1 || postflag == 2) ? postflag : 0) : postflag);
  UNPROTECT(7);
  return out;
}

SEXP scde_hip_varnorm_weights(SEXP Models, SEXP Counts, SEXP PriorX, SEXP Nboot, SEXP NCores, SEXP LocalTheta,
                              SEXP SquareLogitConc, SEXP BatchCodes, SEXP NBatch, SEXP UseExpectedValue) {
  SEXP mm = PROTECT(Rf_coerceVector(Models, REALSXP)), px = PROTECT(Rf_coerceVector(PriorX, REALSXP));
  SEXP ci = PROTECT(Rf_coerceVector(Counts, INTSXP));
  const int *counts = INTEGER(ci);
  const int ngenes = Rf_nrows(Counts), ncells = Rf_ncols(Counts), G = XLENGTH(px), nb = as_int(NBatch);
  int *codes = NULL;
  if (nb > 1) {
    SEXP bc = PROTECT(Rf_coerceVector(BatchCodes, INTSXP));
    codes = (int *) R_alloc(ncells, sizeof(int));
    for (int c = 0; c < ncells; c++) codes[c] = INTEGER(bc)[c] - 1;  /* factor codes */
    UNPROTECT(1);
  }
  const int nm_ = nb > 1 ? 1 + nb : 1;
  SEXP modes = PROTECT(Rf_allocMatrix(REALSXP, ngenes, nm_));
  SEXP matw = PROTECT(Rf_allocMatrix(REALSXP, ngenes, ncells));
  SEXP bmatw = nb > 1 ? Rf_allocMatrix(REALSXP, ngenes, ncells) : R_NilValue;
  PROTECT(bmatw);
  double *mbuf = (double *) R_alloc((size_t) nm_ * ngenes > 0 ? (size_t) nm_ * ngenes : 1, sizeof(double));
  chk(scde_pagoda_varnorm_weights_host(NULL, counts, ngenes, ngenes, ncells, REAL(mm), as_int(LocalTheta),
                                       as_int(SquareLogitConc), REAL(px), G, as_int(Nboot), as_int(NCores), codes,
                                       nb > 1 ? nb : 0, as_int(UseExpectedValue), mbuf, REAL(matw),
                                       nb > 1 ? REAL(bmatw) : NULL));
  /* library: level-major (level x gene); R: one column per level */
  for (int m = 0; m < nm_; m++) memcpy(REAL(modes) + (size_t) m * ngenes, mbuf + (size_t) m * ngenes, sizeof(double) * ngenes);
  const char *nm[] = {"modes", "matw", "bmatw", ""};
  SEXP out = PROTECT(Rf_mkNamed(VECSXP, nm));
  SET_VECTOR_ELT(out, 0, modes); SET_VECTOR_ELT(out, 1, matw); SET_VECTOR_ELT(out, 2, bmatw);
  UNPROTECT(7);
  return out;
}
