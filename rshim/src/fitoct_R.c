/* FitOCTLib's .Call shim over libfitoct.  Replaces the
 * rstan::sampling(ExpGP, ...) call inside FitOCTLib::fitExpGP; the R-level signature
 * (FitOCT.R:110-124, priPost.R:2-16, server.R:408-426) is unchanged, see
 * R/fitExpGP.R.  Compiled by R CMD INSTALL (src/Makevars); R is not part of this
 * repository's image, so the R-free half (fitoct_drive.c) carries the logic and is
 * what tests/test_rshim_driver.py exercises.
 *
 * Threading: everything runs on the R main thread.  The poll loop asks R for a user
 * interrupt through R_ToplevelExec, so R_CheckUserInterrupt's longjmp never unwinds
 * through library code; the interrupt is re-raised only after the plan is destroyed.
 * Errors: Rf_error(fitoct_last_error()) after every resource is released.
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <R_ext/Utils.h>
#include <string.h>

#include "fitoct_drive.h"

static void check_interrupt(void* unused) {
  (void)unused;
  R_CheckUserInterrupt();
}

typedef struct {
  int open_progress;
  int64_t next_report;
} drive_ctx;

static int32_t r_interrupted(void* ctx) {
  (void)ctx;
  return R_ToplevelExec(check_interrupt, NULL) == FALSE;
}

/* rstan-style progress lines (what open_progress = TRUE showed via stan.log) */
static void r_progress(void* vctx, int64_t done, int64_t total) {
  drive_ctx* c = (drive_ctx*)vctx;
  if (!c->open_progress || total <= 0) return;
  if (done >= c->next_report || done == total) {
    Rprintf("fitoct: transitions %lld / %lld [%3d%%]\n", (long long)done, (long long)total,
            (int)(100 * done / total));
    c->next_report = done + (total + 9) / 10;
  }
}

/* .Call("fitoct_R_sample", x, y, uy, dataType, Nn, gridType, rho, theta0, Sigma0, prior,
 *       hyper = c(lambda_rate, lambda_scale, nu), prior_PD, chains, warmup, samples, seed,
 *       adapt_delta, max_treedepth, open_progress, device)
 * -> list(draws [chains*iters*ncols, C order], names, stepsize [chains], inv_metric) */
SEXP fitoct_R_sample(SEXP x, SEXP y, SEXP uy, SEXP dataType, SEXP Nn, SEXP gridType,
                     SEXP rho, SEXP theta0, SEXP Sigma0, SEXP prior, SEXP hyper,
                     SEXP priorPD, SEXP chains, SEXP warmup, SEXP samples, SEXP seed,
                     SEXP adaptDelta, SEXP maxDepth, SEXP openProgress, SEXP device) {
  fitoct_problem p;
  fitoct_config c;
  fitoct_default_problem(&p);
  fitoct_default_config(&c);
  if (LENGTH(y) != LENGTH(x) || LENGTH(uy) != LENGTH(x))
    Rf_error("fitoct: x, y and uy must have the same length");
  if (LENGTH(theta0) != 3 || LENGTH(Sigma0) != 9 || LENGTH(hyper) != 3)
    Rf_error("fitoct: theta0 must have 3 values, Sigma0 9, hyper 3");
  p.N = LENGTH(x);
  p.x = REAL(x);
  p.y = REAL(y);
  p.uy = REAL(uy);
  p.data_type = asInteger(dataType);
  p.Nn = asInteger(Nn);
  p.grid_type = strcmp(CHAR(asChar(gridType)), "internal") ? FITOCT_GRID_EXTREMAL
                                                           : FITOCT_GRID_INTERNAL;
  p.rho = asReal(rho);
  for (int k = 0; k < 3; ++k) p.theta0[k] = REAL(theta0)[k];
  for (int k = 0; k < 9; ++k) p.Sigma0[k] = REAL(Sigma0)[k];   /* symmetric: order-free */
  p.prior_type = asInteger(prior);                              /* 0 normal, 1 lasso, 2 horseshoe */
  p.lambda_rate = REAL(hyper)[0];
  p.lambda_scale = REAL(hyper)[1];
  p.nu = REAL(hyper)[2];
  p.prior_PD = asInteger(priorPD);
  c.chains = asInteger(chains);
  c.warmup = asInteger(warmup);
  c.samples = asInteger(samples);
  c.seed = (uint64_t)asReal(seed);
  c.adapt_delta = asReal(adaptDelta);
  c.max_treedepth = asInteger(maxDepth);
  c.device = asInteger(device);
  if (c.chains <= 0 || c.warmup < 0 || c.samples <= 0) Rf_error("fitoct: bad chains / iterations");

  const int ncols = fitoct_n_cols(p.prior_type, p.Nn), D = fitoct_dim(p.prior_type, p.Nn);
  if (ncols <= 0 || D <= 0) Rf_error("fitoct: unsupported prior_type / Nn");
  const R_xlen_t iters = (R_xlen_t)c.warmup + c.samples;   /* save_warmup = 1 */
  SEXP draws = PROTECT(allocVector(REALSXP, (R_xlen_t)c.chains * iters * ncols));
  SEXP eps = PROTECT(allocVector(REALSXP, c.chains));
  SEXP minv = PROTECT(allocVector(REALSXP, (R_xlen_t)c.chains * D));
  fitoct_result r;
  memset(&r, 0, sizeof r);
  r.draws = REAL(draws);
  r.draws_capacity = XLENGTH(draws);
  r.stepsize = REAL(eps);
  r.inv_metric = REAL(minv);
  drive_ctx ctx = {asLogical(openProgress) == TRUE, 0};
  /* the library owns nothing of ours after this returns, and has freed its own */
  const int32_t rc = fitoct_drive_sample(&p, &c, &r, 50, r_progress, r_interrupted, &ctx);
  if (rc == FITOCT_E_CANCELLED) {
    UNPROTECT(3);
    R_CheckUserInterrupt();                 /* re-raise the user's interrupt */
    Rf_error("fitoct: sampling cancelled");
  }
  if (rc != FITOCT_OK) {
    UNPROTECT(3);
    Rf_error("fitoct: %s", fitoct_last_error());
  }
  SEXP names = PROTECT(allocVector(STRSXP, ncols));
  char buf[64];
  for (int i = 0; i < ncols; ++i) {
    fitoct_column_name(p.prior_type, p.Nn, i, buf, (int32_t)sizeof buf);
    SET_STRING_ELT(names, i, mkChar(buf));
  }
  SEXP out = PROTECT(allocVector(VECSXP, 4));
  SET_VECTOR_ELT(out, 0, draws);
  SET_VECTOR_ELT(out, 1, names);
  SET_VECTOR_ELT(out, 2, eps);
  SET_VECTOR_ELT(out, 3, minv);
  UNPROTECT(5);
  return out;
}

SEXP fitoct_R_device_count(void) { return ScalarInteger(fitoct_device_count()); }

static const R_CallMethodDef call_methods[] = {
    {"fitoct_R_sample", (DL_FUNC)&fitoct_R_sample, 20},
    {"fitoct_R_device_count", (DL_FUNC)&fitoct_R_device_count, 0},
    {NULL, NULL, 0}};

void R_init_FitOCTLibHIP(DllInfo* dll) {
  R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
