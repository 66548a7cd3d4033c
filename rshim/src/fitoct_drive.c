/* See fitoct_drive.h.  Plain C99 over the C ABI of include/fitoct.h. */
#define _POSIX_C_SOURCE 199309L
#include "fitoct_drive.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static void sleep_ms(int32_t ms) {
  struct timespec ts;
  ts.tv_sec = ms / 1000;
  ts.tv_nsec = (long)(ms % 1000) * 1000000L;
  nanosleep(&ts, NULL);
}

int32_t fitoct_drive_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res, int32_t poll_ms, fitoct_progress_fn progress,
                            fitoct_interrupt_fn interrupted, void* ctx) {
  fitoct_plan* plan = NULL;
  int32_t rc = fitoct_plan_create(prob, cfg, &plan);
  if (rc != FITOCT_OK) return rc;            /* nothing allocated */
  rc = fitoct_plan_launch(plan, NULL, NULL);
  int cancelled = 0;
  if (rc == FITOCT_OK) {
    int64_t done = 0, total = 0, last = -1;
    int32_t fin = 0;
    if (poll_ms <= 0) poll_ms = 50;
    for (;;) {
      rc = fitoct_plan_poll(plan, &done, &total, &fin);
      if (rc != FITOCT_OK || fin) break;
      if (!cancelled && interrupted && interrupted(ctx)) {
        rc = fitoct_plan_cancel(plan);       /* chains stop at their next 8th transition */
        if (rc != FITOCT_OK) break;
        cancelled = 1;
      }
      if (progress && !cancelled && done != last) {
        progress(ctx, done, total);
        last = done;
      }
      sleep_ms(poll_ms);
    }
    /* always drain the launch before the plan's buffers go away */
    const int32_t rw = fitoct_plan_wait(plan);
    if (rc == FITOCT_OK) rc = rw;
    if (rc == FITOCT_OK) rc = fitoct_plan_download(plan, res);
    if (rc == FITOCT_OK && progress) progress(ctx, total, total);
  }
  fitoct_plan_destroy(plan);
  if (cancelled && (rc == FITOCT_OK || rc == FITOCT_E_CANCELLED)) rc = FITOCT_E_CANCELLED;
  return rc;
}

/* ---- method = 'sample' -> progress lines + Stan CSV per chain ---------------- */
typedef struct {
  fitoct_line_fn line;
  fitoct_interrupt_fn interrupted;
  void* ctx;
  int32_t warmup, samples;
  int32_t last_pct;
} csv_ctx;

static void csv_progress(void* vc, int64_t done, int64_t total) {
  csv_ctx* c = (csv_ctx*)vc;
  char buf[160];
  const int32_t pct = fitoct_progress_line(done, total, c->warmup, c->samples, buf, sizeof buf);
  if (pct < 0 || pct == c->last_pct) return;
  c->last_pct = pct;
  if (c->line) c->line(c->ctx, buf);
}

static int32_t csv_interrupted(void* vc) {
  csv_ctx* c = (csv_ctx*)vc;
  return c->interrupted ? c->interrupted(c->ctx) : 0;
}

int32_t fitoct_drive_sample_csv(const fitoct_problem* prob, const fitoct_config* cfg,
                                const char* const* paths, int32_t poll_ms, fitoct_line_fn line,
                                fitoct_interrupt_fn interrupted, void* ctx) {
  if (!prob || !cfg || !paths) return FITOCT_E_ARG;
  const int32_t ncols = fitoct_n_cols(prob->prior_type, prob->Nn);
  const int32_t D = fitoct_dim(prob->prior_type, prob->Nn);
  if (cfg->chains < 1 || cfg->warmup < 0 || cfg->samples < 1 || ncols <= 0 || D <= 0) {
    /* the library's own argument check sets the message; nothing is allocated */
    fitoct_plan* plan = NULL;
    const int32_t rc = fitoct_plan_create(prob, cfg, &plan);
    fitoct_plan_destroy(plan);
    return rc != FITOCT_OK ? rc : FITOCT_E_ARG;
  }
  const int64_t rows = cfg->save_warmup ? (int64_t)cfg->warmup + cfg->samples : cfg->samples;
  const size_t n_draws = (size_t)cfg->chains * (size_t)rows * (size_t)ncols;
  double* draws = (double*)malloc(sizeof(double) * n_draws);
  double* eps = (double*)malloc(sizeof(double) * (size_t)cfg->chains);
  double* minv = (double*)malloc(sizeof(double) * (size_t)cfg->chains * (size_t)D);
  int32_t rc = FITOCT_OK;
  if (!draws || !eps || !minv) {
    rc = FITOCT_E_INTERNAL;
  } else {
    fitoct_result r;
    memset(&r, 0, sizeof r);
    r.draws = draws;
    r.draws_capacity = (int64_t)n_draws;
    r.stepsize = eps;
    r.inv_metric = minv;
    csv_ctx c = {line, interrupted, ctx, cfg->warmup, cfg->samples, -1};
    rc = fitoct_drive_sample(prob, cfg, &r, poll_ms, csv_progress, csv_interrupted, &c);
    const int64_t wrows = cfg->save_warmup ? cfg->warmup : 0;
    for (int32_t ch = 0; rc == FITOCT_OK && ch < cfg->chains; ++ch) {
      const double* d = draws + (size_t)ch * (size_t)rows * (size_t)ncols;
      double lw = 0.0, ls = 0.0;       /* n_leapfrog__ (column 4) per phase */
      for (int64_t i = 0; i < rows; ++i) {
        const double v = d[(size_t)i * ncols + 4];
        if (i < wrows) lw += v;
        else ls += v;
      }
      const double t = r.kernel_ms / 1e3;
      const double tw = (lw + ls > 0.0) ? t * lw / (lw + ls) : 0.0;
      rc = fitoct_write_stan_csv(paths[ch], prob, cfg, ch, d, eps[ch], minv + (size_t)ch * D, tw,
                                 t - tw);
    }
  }
  free(draws);
  free(eps);
  free(minv);
  return rc;
}

/* ---- method = 'sample', many chains -> binary arrays for R ----------------------- */
int32_t fitoct_drive_bulk_layout(const fitoct_problem* prob, int32_t chains, int64_t rows,
                                 const double* raw, double* out) {
  if (!prob || !raw || !out || chains < 1 || rows < 1) return FITOCT_E_ARG;
  const int32_t ncols = fitoct_n_cols(prob->prior_type, prob->Nn);
  const int32_t P = fitoct_output_n_params(prob);
  if (ncols <= 0 || P <= 0) return FITOCT_E_ARG;
  const int32_t n_out = 7 + P;
  /* one chain's rows in the output layout, then transposed to column runs */
  const int64_t blk = rows < 256 ? rows : 256;
  double* tmp = (double*)malloc(sizeof(double) * (size_t)blk * (size_t)n_out);
  if (!tmp) return FITOCT_E_INTERNAL;
  int32_t rc = FITOCT_OK;
  for (int32_t ch = 0; rc == FITOCT_OK && ch < chains; ++ch) {
    const double* src = raw + (size_t)ch * (size_t)rows * (size_t)ncols;
    double* dst = out + (size_t)ch * (size_t)n_out * (size_t)rows;
    for (int64_t r0 = 0; rc == FITOCT_OK && r0 < rows; r0 += blk) {
      const int64_t nr = rows - r0 < blk ? rows - r0 : blk;
      rc = fitoct_output_rows(prob, 7, nr, src + (size_t)r0 * (size_t)ncols, tmp);
      for (int64_t i = 0; rc == FITOCT_OK && i < nr; ++i)
        for (int32_t j = 0; j < n_out; ++j)
          dst[(size_t)j * (size_t)rows + (size_t)(r0 + i)] = tmp[(size_t)i * (size_t)n_out + j];
    }
  }
  free(tmp);
  return rc;
}

int32_t fitoct_drive_sample_bulk(const fitoct_problem* prob, const fitoct_config* cfg,
                                 double* draws, int64_t draws_capacity, double* stepsize,
                                 double* inv_metric, double* elapsed, int32_t poll_ms,
                                 fitoct_line_fn line, fitoct_interrupt_fn interrupted, void* ctx) {
  if (!prob || !cfg || !draws) return FITOCT_E_ARG;
  const int32_t ncols = fitoct_n_cols(prob->prior_type, prob->Nn);
  const int32_t P = fitoct_output_n_params(prob);
  if (cfg->chains < 1 || cfg->warmup < 0 || cfg->samples < 1 || ncols <= 0 || P <= 0) {
    fitoct_plan* plan = NULL;   /* the library's own argument check sets the message */
    const int32_t rc = fitoct_plan_create(prob, cfg, &plan);
    fitoct_plan_destroy(plan);
    return rc != FITOCT_OK ? rc : FITOCT_E_ARG;
  }
  const int64_t rows = cfg->save_warmup ? (int64_t)cfg->warmup + cfg->samples : cfg->samples;
  if (draws_capacity < (int64_t)cfg->chains * (7 + P) * rows) return FITOCT_E_ARG;
  const size_t n_raw = (size_t)cfg->chains * (size_t)rows * (size_t)ncols;
  double* raw = (double*)malloc(sizeof(double) * n_raw);
  if (!raw) return FITOCT_E_INTERNAL;
  fitoct_result r;
  memset(&r, 0, sizeof r);
  r.draws = raw;
  r.draws_capacity = (int64_t)n_raw;
  r.stepsize = stepsize;
  r.inv_metric = inv_metric;
  csv_ctx c = {line, interrupted, ctx, cfg->warmup, cfg->samples, -1};
  int32_t rc = fitoct_drive_sample(prob, cfg, &r, poll_ms, csv_progress, csv_interrupted, &c);
  if (rc == FITOCT_OK && elapsed) {
    const int64_t wrows = cfg->save_warmup ? cfg->warmup : 0;
    const double t = r.kernel_ms / 1e3;
    for (int32_t ch = 0; ch < cfg->chains; ++ch) {
      const double* d = raw + (size_t)ch * (size_t)rows * (size_t)ncols;
      double lw = 0.0, ls = 0.0;       /* n_leapfrog__ (column 4) per phase */
      for (int64_t i = 0; i < rows; ++i) {
        const double v = d[(size_t)i * ncols + 4];
        if (i < wrows) lw += v;
        else ls += v;
      }
      elapsed[2 * ch] = (lw + ls > 0.0) ? t * lw / (lw + ls) : 0.0;
      elapsed[2 * ch + 1] = t - elapsed[2 * ch];
    }
  }
  if (rc == FITOCT_OK) rc = fitoct_drive_bulk_layout(prob, cfg->chains, rows, raw, draws);
  free(raw);
  return rc;
}

/* ---- method = 'optim' ---------------------------------------------------------- */
/* theta and yGP of an output-layout row (yGP found by name: a parameter of the normal
 * and lasso families, a transformed parameter of the horseshoe) */
static int32_t theta_ygp(const fitoct_problem* prob, const double* par, double* theta,
                         double* ygp) {
  const int32_t P = fitoct_output_n_params(prob);
  char name[64];
  int32_t first_y = -1;
  for (int32_t i = 0; i < P && first_y < 0; ++i) {
    const int32_t rc = fitoct_output_param_name(prob, i, name, sizeof name);
    if (rc != FITOCT_OK) return rc;
    if (strcmp(name, "yGP.1") == 0) first_y = i;
  }
  for (int k = 0; k < 3; ++k) theta[k] = par[k];
  if (prob->prior_type == FITOCT_MODEL_MONOEXP) return FITOCT_OK;
  if (first_y < 0) return FITOCT_E_INTERNAL;
  for (int k = 0; k < prob->Nn; ++k) ygp[k] = par[first_y + k];
  return FITOCT_OK;
}

int32_t fitoct_drive_optimize(const fitoct_problem* prob, const fitoct_optim_config* cfg,
                              const double* init_q, double* par_out, double* hessian_out,
                              double* dL, double* m, double* resid, double* value,
                              int32_t* return_code) {
  if (!prob || !cfg || !par_out) return FITOCT_E_ARG;
  const int32_t D = fitoct_dim(prob->prior_type, prob->Nn);
  if (D <= 0) return FITOCT_E_ARG;
  double* q = (double*)malloc(sizeof(double) * (size_t)(2 * D + 1));
  double* ygp = (double*)malloc(sizeof(double) * (size_t)(prob->Nn > 0 ? prob->Nn : 1));
  if (!q || !ygp) {
    free(q);
    free(ygp);
    return FITOCT_E_INTERNAL;
  }
  fitoct_optim_result r;
  memset(&r, 0, sizeof r);
  r.par = q;
  r.hessian = hessian_out;
  fitoct_optim_config c = *cfg;
  if (!hessian_out) c.hessian = 0;
  int32_t rc = fitoct_optimize(prob, &c, init_q, &r);
  if (rc == FITOCT_OK) {
    /* constrained optimum + br -> output layout */
    double* raw = q + D;               /* [D + 1]: constrained parameters, br */
    rc = fitoct_constrain(prob->prior_type, prob->Nn, 1, q, raw);
    if (rc == FITOCT_OK) {
      raw[D] = r.sumr2 / prob->N;
      rc = fitoct_output_rows(prob, 0, 1, raw, par_out);
    }
    double theta[3];
    if (rc == FITOCT_OK) rc = theta_ygp(prob, par_out, theta, ygp);
    if (rc == FITOCT_OK && (dL || m || resid))
      rc = fitoct_expgp_curves(prob, 1, theta, ygp, dL, m, resid, NULL);
    if (value) *value = r.value;
    if (return_code) *return_code = r.return_code;
  }
  free(q);
  free(ygp);
  return rc;
}

/* ---- method = 'vb' ------------------------------------------------------------- */
int32_t fitoct_drive_vb_csv(const fitoct_problem* prob, const fitoct_vb_config* cfg,
                            const double* init_q, const char* path) {
  if (!prob || !cfg || !path) return FITOCT_E_ARG;
  const int32_t D = fitoct_dim(prob->prior_type, prob->Nn);
  const int32_t S = cfg->output_samples > 0 ? cfg->output_samples : 0;
  const int32_t P = fitoct_output_n_params(prob);
  if (D <= 0 || P <= 0) return FITOCT_E_ARG;
  const size_t nq = (size_t)S * D;
  double* buf = (double*)malloc(sizeof(double) * (2 * (size_t)D + nq + 3 * (size_t)S +
                                                  2 * (size_t)D + 2 + (size_t)P + 24));
  if (!buf) return FITOCT_E_INTERNAL;
  double* mu = buf;
  double* om = mu + D;
  double* q = om + D;
  double* lp = q + nq;
  double* lg = lp + S;
  double* s2 = lg + S;
  double* raw = s2 + S;                /* [D + 1] */
  double* par = raw + D + 1;           /* [P] */
  double* ygp = par + P;               /* [<= 24] */
  fitoct_vb_result r;
  memset(&r, 0, sizeof r);
  r.mu = mu;
  r.omega = om;
  r.draws = S ? q : NULL;
  r.log_p = S ? lp : NULL;
  r.log_g = S ? lg : NULL;
  r.sumr2 = S ? s2 : NULL;
  int32_t rc = fitoct_vb(prob, cfg, init_q, &r);
  double mean_s2 = NAN;
  if (rc == FITOCT_OK) {   /* br of the mean row: residuals at the constrained mean */
    rc = fitoct_constrain(prob->prior_type, prob->Nn, 1, mu, raw);
    raw[D] = NAN;
    if (rc == FITOCT_OK) rc = fitoct_output_rows(prob, 0, 1, raw, par);
    double theta[3], br = NAN;
    if (rc == FITOCT_OK) rc = theta_ygp(prob, par, theta, ygp);
    if (rc == FITOCT_OK) rc = fitoct_expgp_curves(prob, 1, theta, ygp, NULL, NULL, NULL, &br);
    mean_s2 = br * prob->N;
  }
  if (rc == FITOCT_OK)
    rc = fitoct_write_vb_csv(path, prob, cfg, mu, mean_s2, S, q, lp, lg, s2, r.eta);
  free(buf);
  return rc;
}
