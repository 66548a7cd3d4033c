/* FitOCTLib's .Call shim over libfitoct.  Replaces the
 * rstan::sampling / rstan::optimizing / rstan::vb calls inside FitOCTLib::fitExpGP and
 * FitOCTLib::fitMonoExp; the R-level signatures (FitOCT.R:95,110-124, priPost.R:2-16,
 * server.R:341-343,408-426) are unchanged, see R/fitExpGP.R.  Compiled by R CMD
 * INSTALL (src/Makevars); R is not part of this repository's image, so the R-free half
 * (fitoct_drive.c) carries the logic -- sampling with progress and interrupts, the
 * Stan CSV files, the optimum with its generated quantities, the ADVI CSV -- and is
 * what tests/test_rshim_driver.py exercises.  This file only converts R objects.
 *
 * Threading: everything runs on the R main thread.  The poll loop asks R for a user
 * interrupt through R_ToplevelExec, so R_CheckUserInterrupt's longjmp never unwinds
 * through library code; the interrupt is re-raised only after the plan is destroyed.
 * Errors: Rf_error(fitoct_last_error()) after every library resource is released
 * (host buffers here are R_alloc'ed or R vectors, reclaimed by R).
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <R_ext/Utils.h>
#include <string.h>

#include "fitoct_drive.h"

/* ---- R lists -> ABI structs ------------------------------------------------- */
static SEXP elt(SEXP list, const char* name) {
  SEXP names = Rf_getAttrib(list, R_NamesSymbol);
  for (R_xlen_t i = 0; i < XLENGTH(list); ++i)
    if (strcmp(CHAR(STRING_ELT(names, i)), name) == 0) return VECTOR_ELT(list, i);
  Rf_error("fitoct: argument list has no element '%s'", name);
  return R_NilValue;
}
static double num(SEXP list, const char* name) { return Rf_asReal(elt(list, name)); }
static int inum(SEXP list, const char* name) { return Rf_asInteger(elt(list, name)); }

/* prob: list(x, y, uy, dataType, Nn, gridType, rho, theta0, Sigma0, prior, lambda_rate,
 *            lambda_scale, nu, prior_PD) as built by fitoct_problem() in R/fitExpGP.R */
static void to_problem(SEXP prob, fitoct_problem* p) {
  fitoct_default_problem(p);
  SEXP x = elt(prob, "x"), y = elt(prob, "y"), uy = elt(prob, "uy");
  SEXP th = elt(prob, "theta0"), S0 = elt(prob, "Sigma0");
  if (TYPEOF(x) != REALSXP || TYPEOF(y) != REALSXP || TYPEOF(uy) != REALSXP ||
      TYPEOF(th) != REALSXP || TYPEOF(S0) != REALSXP)
    Rf_error("fitoct: x, y, uy, theta0 and Sigma0 must be double vectors");
  if (XLENGTH(y) != XLENGTH(x) || XLENGTH(uy) != XLENGTH(x))
    Rf_error("fitoct: x, y and uy must have the same length");
  if (XLENGTH(x) > FITOCT_MAX_BINS) Rf_error("fitoct: too many depth bins");
  if (XLENGTH(th) != 3 || XLENGTH(S0) != 9) Rf_error("fitoct: theta0 must have 3 values, Sigma0 9");
  p->N = (int32_t)XLENGTH(x);
  p->x = REAL(x);
  p->y = REAL(y);
  p->uy = REAL(uy);
  p->data_type = inum(prob, "dataType");
  p->Nn = inum(prob, "Nn");
  p->grid_type = strcmp(CHAR(Rf_asChar(elt(prob, "gridType"))), "internal") ? FITOCT_GRID_EXTREMAL
                                                                            : FITOCT_GRID_INTERNAL;
  p->rho = num(prob, "rho");
  for (int k = 0; k < 3; ++k) p->theta0[k] = REAL(th)[k];
  for (int k = 0; k < 9; ++k) p->Sigma0[k] = REAL(S0)[k];   /* symmetric: order-free */
  p->prior_type = inum(prob, "prior");                      /* 0 normal 1 lasso 2 horseshoe 3 mono */
  p->lambda_rate = num(prob, "lambda_rate");
  p->lambda_scale = num(prob, "lambda_scale");
  p->nu = num(prob, "nu");
  p->prior_PD = inum(prob, "prior_PD");
}

/* ---- progress and interrupts ------------------------------------------------- */
static void check_interrupt(void* unused) {
  (void)unused;
  R_CheckUserInterrupt();
}
static int32_t r_interrupted(void* ctx) {
  (void)ctx;
  return R_ToplevelExec(check_interrupt, NULL) == FALSE;
}
/* rstan-format lines on R's stdout, whatever open_progress is: the Shiny server sinks
 * stdout to stan.log and parses them (server.R:391-393,457-484) */
static void r_line(void* ctx, const char* line) {
  (void)ctx;
  Rprintf("%s\n", line);
  R_FlushConsole();
}

static void stop_on(int32_t rc) {
  if (rc == FITOCT_E_CANCELLED) {
    R_CheckUserInterrupt();                 /* re-raise the user's interrupt */
    Rf_error("fitoct: sampling cancelled");
  }
  if (rc != FITOCT_OK) Rf_error("fitoct: %s", fitoct_last_error());
}

/* .Call(fitoct_R_sample, prob, ctrl, files): ctrl = list(chains, warmup, samples, seed,
 * adapt_delta, max_treedepth, devices); one Stan CSV per chain at files[].  devices: the
 * integer device list (fitExpGP(n_gpus = k, device = d) passes d, ..., d + k - 1): the
 * library splits the chains into contiguous blocks, one host thread per GPU, and still
 * returns only on the R main thread (SURVEY.md §8b threading) */
SEXP fitoct_R_sample(SEXP prob, SEXP ctrl, SEXP files) {
  fitoct_problem p;
  fitoct_config c;
  to_problem(prob, &p);
  fitoct_default_config(&c);
  c.chains = inum(ctrl, "chains");
  c.warmup = inum(ctrl, "warmup");
  c.samples = inum(ctrl, "samples");
  c.seed = (uint64_t)num(ctrl, "seed");
  c.adapt_delta = num(ctrl, "adapt_delta");
  c.max_treedepth = inum(ctrl, "max_treedepth");
  SEXP devs = elt(ctrl, "devices");
  if (TYPEOF(devs) != INTSXP || XLENGTH(devs) < 1 || XLENGTH(devs) > FITOCT_MAX_DEVICES)
    Rf_error("fitoct: devices must be an integer vector of 1 to %d device ordinals",
             FITOCT_MAX_DEVICES);
  c.device = INTEGER(devs)[0];
  c.n_devices = (int32_t)XLENGTH(devs);
  for (int i = 0; i < c.n_devices; ++i) c.devices[i] = INTEGER(devs)[i];
  if (TYPEOF(files) != STRSXP || XLENGTH(files) != c.chains)
    Rf_error("fitoct: one output file per chain is required");
  const char** paths = (const char**)R_alloc((size_t)c.chains, sizeof(char*));
  for (int i = 0; i < c.chains; ++i) paths[i] = Rf_translateCharFP(STRING_ELT(files, i));
  /* the library owns nothing of ours after this returns, and has freed its own */
  stop_on(fitoct_drive_sample_csv(&p, &c, paths, 50, r_line, r_interrupted, NULL));
  return R_NilValue;
}

/* .Call(fitoct_R_sample_bulk, prob, ctrl): the same run as fitoct_R_sample for many chains
 * (R/fitExpGP.R uses it above 64 chains), returned as R vectors instead of one CSV per chain:
 * list(draws = array(dim = c(rows, 7 + n_params, chains), dimnames = list(NULL, columns,
 * NULL)), stepsize [chains], inv_metric [D, chains] matrix, elapsed [2, chains] matrix).
 * fitoct_drive_sample_bulk writes straight into the R vectors (no copy). */
SEXP fitoct_R_sample_bulk(SEXP prob, SEXP ctrl) {
  fitoct_problem p;
  fitoct_config c;
  to_problem(prob, &p);
  fitoct_default_config(&c);
  c.chains = inum(ctrl, "chains");
  c.warmup = inum(ctrl, "warmup");
  c.samples = inum(ctrl, "samples");
  c.seed = (uint64_t)num(ctrl, "seed");
  c.adapt_delta = num(ctrl, "adapt_delta");
  c.max_treedepth = inum(ctrl, "max_treedepth");
  SEXP devs = elt(ctrl, "devices");
  if (TYPEOF(devs) != INTSXP || XLENGTH(devs) < 1 || XLENGTH(devs) > FITOCT_MAX_DEVICES)
    Rf_error("fitoct: devices must be an integer vector of 1 to %d device ordinals",
             FITOCT_MAX_DEVICES);
  c.device = INTEGER(devs)[0];
  c.n_devices = (int32_t)XLENGTH(devs);
  for (int i = 0; i < c.n_devices; ++i) c.devices[i] = INTEGER(devs)[i];
  const int P = fitoct_output_n_params(&p), D = fitoct_dim(p.prior_type, p.Nn);
  if (P <= 0 || D <= 0 || c.chains < 1 || c.samples < 1 || c.warmup < 0)
    Rf_error("fitoct: invalid model or chain / iteration counts");
  const int n_out = 7 + P;
  const R_xlen_t rows = c.save_warmup ? (R_xlen_t)c.warmup + c.samples : c.samples;
  SEXP draws = PROTECT(Rf_allocVector(REALSXP, rows * n_out * (R_xlen_t)c.chains));
  SEXP eps = PROTECT(Rf_allocVector(REALSXP, c.chains));
  SEXP minv = PROTECT(Rf_allocMatrix(REALSXP, D, c.chains));
  SEXP el = PROTECT(Rf_allocMatrix(REALSXP, 2, c.chains));
  const int32_t rc = fitoct_drive_sample_bulk(&p, &c, REAL(draws), (int64_t)XLENGTH(draws),
                                              REAL(eps), REAL(minv), REAL(el), 50, r_line,
                                              r_interrupted, NULL);
  if (rc != FITOCT_OK) {
    UNPROTECT(4);
    stop_on(rc);
  }
  SEXP dim = PROTECT(Rf_allocVector(INTSXP, 3));
  INTEGER(dim)[0] = (int)rows;
  INTEGER(dim)[1] = n_out;
  INTEGER(dim)[2] = c.chains;
  Rf_setAttrib(draws, R_DimSymbol, dim);
  char buf[64];
  SEXP cn = PROTECT(Rf_allocVector(STRSXP, n_out));
  static const char* lead[7] = {"lp__", "accept_stat__", "stepsize__", "treedepth__",
                                "n_leapfrog__", "divergent__", "energy__"};
  for (int j = 0; j < 7; ++j) SET_STRING_ELT(cn, j, Rf_mkChar(lead[j]));
  for (int j = 0; j < P; ++j) {
    fitoct_output_param_name(&p, j, buf, (int32_t)sizeof buf);
    SET_STRING_ELT(cn, 7 + j, Rf_mkChar(buf));
  }
  SEXP dn = PROTECT(Rf_allocVector(VECSXP, 3));
  SET_VECTOR_ELT(dn, 1, cn);
  Rf_setAttrib(draws, R_DimNamesSymbol, dn);
  const char* names[] = {"draws", "stepsize", "inv_metric", "elapsed"};
  SEXP out = PROTECT(Rf_allocVector(VECSXP, 4));
  SEXP on = PROTECT(Rf_allocVector(STRSXP, 4));
  SET_VECTOR_ELT(out, 0, draws);
  SET_VECTOR_ELT(out, 1, eps);
  SET_VECTOR_ELT(out, 2, minv);
  SET_VECTOR_ELT(out, 3, el);
  for (int i = 0; i < 4; ++i) SET_STRING_ELT(on, i, Rf_mkChar(names[i]));
  Rf_setAttrib(out, R_NamesSymbol, on);
  UNPROTECT(9);
  return out;
}

/* .Call(fitoct_R_optimize, prob, ctrl): ctrl = list(device, hessian) ->
 * list(par (named, output layout), value, return_code, hessian (D x D, dimnames),
 *      dL, m, resid) -- rstan::optimizing(as_vector = FALSE) after R/fitExpGP.R regroups par */
SEXP fitoct_R_optimize(SEXP prob, SEXP ctrl) {
  fitoct_problem p;
  fitoct_optim_config oc;
  to_problem(prob, &p);
  fitoct_default_optim_config(&oc);
  oc.device = inum(ctrl, "device");
  oc.hessian = Rf_asLogical(elt(ctrl, "hessian")) == TRUE;
  const int D = fitoct_dim(p.prior_type, p.Nn), P = fitoct_output_n_params(&p);
  if (D <= 0 || P <= 0) Rf_error("fitoct: %s", fitoct_last_error());
  SEXP par = PROTECT(Rf_allocVector(REALSXP, P));
  SEXP H = PROTECT(Rf_allocMatrix(REALSXP, D, D));
  SEXP dL = PROTECT(Rf_allocVector(REALSXP, p.N));
  SEXP m = PROTECT(Rf_allocVector(REALSXP, p.N));
  SEXP resid = PROTECT(Rf_allocVector(REALSXP, p.N));
  double value = 0.0;
  int32_t return_code = 0;
  const int32_t rc = fitoct_drive_optimize(&p, &oc, NULL, REAL(par), oc.hessian ? REAL(H) : NULL,
                                           p.prior_type == FITOCT_MODEL_MONOEXP ? NULL : REAL(dL),
                                           REAL(m), REAL(resid), &value, &return_code);
  if (rc != FITOCT_OK) {
    UNPROTECT(5);
    stop_on(rc);
  }
  char buf[64];
  SEXP pn = PROTECT(Rf_allocVector(STRSXP, P));
  for (int i = 0; i < P; ++i) {
    fitoct_output_param_name(&p, i, buf, (int32_t)sizeof buf);
    SET_STRING_ELT(pn, i, Rf_mkChar(buf));
  }
  Rf_setAttrib(par, R_NamesSymbol, pn);
  SEXP hn = PROTECT(Rf_allocVector(STRSXP, D));   /* unconstrained parameters, draw names */
  for (int j = 0; j < D; ++j) {
    fitoct_column_name(p.prior_type, p.Nn, 7 + j, buf, (int32_t)sizeof buf);
    SET_STRING_ELT(hn, j, Rf_mkChar(buf));
  }
  SEXP dn = PROTECT(Rf_allocVector(VECSXP, 2));
  SET_VECTOR_ELT(dn, 0, hn);
  SET_VECTOR_ELT(dn, 1, hn);
  Rf_setAttrib(H, R_DimNamesSymbol, dn);           /* symmetric: row/column order-free */
  const char* names[] = {"par", "value", "return_code", "hessian", "dL", "m", "resid"};
  SEXP out = PROTECT(Rf_allocVector(VECSXP, 7));
  SEXP on = PROTECT(Rf_allocVector(STRSXP, 7));
  SET_VECTOR_ELT(out, 0, par);
  SET_VECTOR_ELT(out, 1, Rf_ScalarReal(value));
  SET_VECTOR_ELT(out, 2, Rf_ScalarInteger(return_code));
  SET_VECTOR_ELT(out, 3, oc.hessian ? H : R_NilValue);
  SET_VECTOR_ELT(out, 4, p.prior_type == FITOCT_MODEL_MONOEXP ? R_NilValue : dL);
  SET_VECTOR_ELT(out, 5, m);
  SET_VECTOR_ELT(out, 6, resid);
  for (int i = 0; i < 7; ++i) SET_STRING_ELT(on, i, Rf_mkChar(names[i]));
  Rf_setAttrib(out, R_NamesSymbol, on);
  UNPROTECT(10);
  return out;
}

/* .Call(fitoct_R_vb, prob, ctrl, file): ctrl = list(seed, device); CmdStan variational CSV */
SEXP fitoct_R_vb(SEXP prob, SEXP ctrl, SEXP file) {
  fitoct_problem p;
  fitoct_vb_config vc;
  to_problem(prob, &p);
  fitoct_default_vb_config(&vc);
  vc.seed = (uint64_t)num(ctrl, "seed");
  vc.device = inum(ctrl, "device");
  stop_on(fitoct_drive_vb_csv(&p, &vc, NULL, Rf_translateCharFP(Rf_asChar(file))));
  return R_NilValue;
}

/* .Call(fitoct_R_mono_theta0, x, y, dataType): fitMonoExp's starting point */
SEXP fitoct_R_mono_theta0(SEXP x, SEXP y, SEXP dataType) {
  if (TYPEOF(x) != REALSXP || TYPEOF(y) != REALSXP || XLENGTH(x) != XLENGTH(y) ||
      XLENGTH(x) > FITOCT_MAX_BINS)
    Rf_error("fitoct: x and y must be double vectors of the same length");
  SEXP out = PROTECT(Rf_allocVector(REALSXP, 3));
  const int32_t rc = fitoct_mono_initial_theta((int32_t)XLENGTH(x), REAL(x), REAL(y),
                                               Rf_asInteger(dataType), REAL(out));
  UNPROTECT(1);
  stop_on(rc);
  return out;
}

SEXP fitoct_R_device_count(void) { return Rf_ScalarInteger(fitoct_device_count()); }

static const R_CallMethodDef call_methods[] = {
    {"fitoct_R_sample", (DL_FUNC)&fitoct_R_sample, 3},
    {"fitoct_R_sample_bulk", (DL_FUNC)&fitoct_R_sample_bulk, 2},
    {"fitoct_R_optimize", (DL_FUNC)&fitoct_R_optimize, 2},
    {"fitoct_R_vb", (DL_FUNC)&fitoct_R_vb, 3},
    {"fitoct_R_mono_theta0", (DL_FUNC)&fitoct_R_mono_theta0, 3},
    {"fitoct_R_device_count", (DL_FUNC)&fitoct_R_device_count, 0},
    {NULL, NULL, 0}};

void R_init_FitOCTLibHIP(DllInfo* dll) {
  R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
