// Stan-format output of libfitoct (host only): the column layout the reference's
// consumers read, generated quantities per bin, and the one Stan-CSV writer that
// both bindings (the R .Call shim and the Python ctypes mirror) use.
//
// Consumers (SURVEY.md §8b "R return value"): plotExpGP.R:9,41-43 and
// server.R:88-237 ask for pars = c('theta','yGP','lambda','sigma','br','lp__')
// through print(fit, pars), as.matrix(fit, pars), traceplot(inc_warmup=TRUE),
// pairs(fit, pars) and rstan::summary(fit, pars)$summary; every family must
// therefore expose each of those names.  rstan::read_stan_csv turns the CSV
// written here into a real stanfit.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"

namespace fitoct {
namespace {

// One output parameter column: where its value comes from.
enum Src { S_RAW = 0, S_LAMBDA_DATA, S_TAU, S_HS_LAMBDA, S_HS_YGP };
struct OutCol {
  std::string name;
  int src;
  int k;   // S_RAW: raw parameter index (0..D, D = br); S_HS_*: control point
};

// Output parameter layout after the leading columns (Stan's order: parameters,
// transformed parameters, generated quantities).
std::vector<OutCol> out_layout(const fitoct_problem* p) {
  std::vector<OutCol> v;
  const int fam = p->prior_type, Nn = p->Nn, D = model_dim(fam, Nn);
  char b[64];
  for (int j = 0; j < D; ++j) v.push_back({column_name(fam, Nn, 7 + j), S_RAW, j});
  if (fam == FITOCT_PRIOR_LASSO) {
    // ⚑ lassoPrior.stan has no lambda parameter: its penalty lambda_s is data
    // (lassoPrior.stan:4).  It is exposed as the constant column `lambda` so that
    // the consumers' pars list resolves (plotExpGP.R:41); rstan reports Rhat NaN for it.
    v.push_back({"lambda", S_LAMBDA_DATA, 0});
  } else if (fam == FITOCT_PRIOR_HORSESHOE) {
    // transformed parameters of horseShoePrior.stan:25-33, in declaration order
    v.push_back({"tau", S_TAU, 0});
    for (int k = 0; k < Nn; ++k) {
      snprintf(b, sizeof b, "lambda.%d", k + 1);
      v.push_back({b, S_HS_LAMBDA, k});
    }
    for (int k = 0; k < Nn; ++k) {
      snprintf(b, sizeof b, "yGP.%d", k + 1);
      v.push_back({b, S_HS_YGP, k});
    }
  }
  if (!p->prior_PD) v.push_back({"br", S_RAW, D});   // plotExpGP.R:42-43: no br in a prior run
  return v;
}

// constrained raw parameters r[0..D-1], br r[D]  ->  output values
void fill_row(const fitoct_problem* p, const std::vector<OutCol>& lay, const double* r, double* o) {
  const int Nn = p->Nn;
  const bool hs = p->prior_type == FITOCT_PRIOR_HORSESHOE;
  // horseshoe raw order: theta[3] z[Nn] r1_global r2_global r1_local[Nn] r2_local[Nn] sigma
  const double* z = r + 3;
  const double* r1l = r + 5 + Nn;
  const double* r2l = r + 5 + 2 * Nn;
  const double tau = hs ? r[3 + Nn] * sqrt(r[4 + Nn]) : 0.0;
  for (size_t i = 0; i < lay.size(); ++i) {
    const OutCol& c = lay[i];
    switch (c.src) {
      case S_RAW: o[i] = r[c.k]; break;
      case S_LAMBDA_DATA: o[i] = p->lambda_scale; break;
      case S_TAU: o[i] = tau; break;
      case S_HS_LAMBDA: o[i] = r1l[c.k] * sqrt(r2l[c.k]); break;
      case S_HS_YGP: o[i] = z[c.k] * (r1l[c.k] * sqrt(r2l[c.k])) * tau; break;
    }
  }
}

int check_layout_problem(const fitoct_problem* p) {
  if (!p) return fail(FITOCT_E_ARG, "problem is NULL");
  if (model_dim(p->prior_type, p->Nn) < 0) return fail(FITOCT_E_ARG, "unknown prior_type");
  if (p->prior_type != FITOCT_MODEL_MONOEXP && (p->Nn < 2 || p->Nn > 24))
    return fail(FITOCT_E_ARG, "Nn must be in [2, 24]");
  return FITOCT_OK;
}

const char* kSampler[7] = {"lp__", "accept_stat__", "stepsize__", "treedepth__",
                           "n_leapfrog__", "divergent__", "energy__"};
const char* kVbLead[3] = {"lp__", "log_p__", "log_g__"};

// numbers as R's read.csv / scan reads them back exactly (NaN, Inf, -Inf)
void put_num(FILE* f, double v) {
  if (isnan(v)) fputs("NaN", f);
  else if (isinf(v)) fputs(v > 0 ? "Inf" : "-Inf", f);
  else fprintf(f, "%.17g", v);
}

const char* family_name(int fam) {
  switch (fam) {
    case FITOCT_PRIOR_NORMAL: return "ExpGP_normal";
    case FITOCT_PRIOR_LASSO: return "ExpGP_lasso";
    case FITOCT_PRIOR_HORSESHOE: return "ExpGP_horseshoe";
    default: return "MonoExp";
  }
}

void write_header_common(FILE* f, const fitoct_problem* p) {
  // key = value lines as CmdStan writes them; rstan's parser strips '#', blanks and
  // "(Default)" and splits on '=', so no value below contains '='
  fputs("# stan_version_major = 2\n# stan_version_minor = 32\n# stan_version_patch = 2\n", f);
  fprintf(f, "# model = %s_model\n", family_name(p->prior_type));
}

void write_header_tail(FILE* f, const fitoct_problem* p, long long id, unsigned long long seed,
                       const char* path) {
  fprintf(f, "# id = %lld\n", id);
  fputs("# data\n", f);
  fprintf(f, "#   file = fitoct_problem (N %d, Nn %d, prior_PD %d)\n", p->N, p->Nn, p->prior_PD);
  fputs("# init = fitoct (jittered around the prior centre, DESIGN.md §1)\n", f);
  fputs("# random\n", f);
  fprintf(f, "#   seed = %llu\n", seed);
  fputs("# output\n", f);
  fprintf(f, "#   file = %s\n", path);
  fputs("#   diagnostic_file =  (Default)\n#   refresh = 100 (Default)\n", f);
  fprintf(f, "# engine = libfitoct ABI %d (MI355X HIP)\n", FITOCT_ABI_VERSION);
}

}  // namespace
}  // namespace fitoct

using namespace fitoct;

extern "C" {

int32_t fitoct_output_n_params(const fitoct_problem* prob) {
  return guarded(__func__, [&]() -> int32_t {
    if (check_layout_problem(prob)) return -1;
    return (int32_t)out_layout(prob).size();
  });
}

int32_t fitoct_output_param_name(const fitoct_problem* prob, int32_t i, char* buf, int32_t buflen) {
  return guarded(__func__, [&]() -> int32_t {
    int rc = check_layout_problem(prob);
    if (rc) return rc;
    const std::vector<OutCol> lay = out_layout(prob);
    if (i < 0 || i >= (int32_t)lay.size()) return fail(FITOCT_E_ARG, "output column index out of range");
    const std::string& s = lay[i].name;
    if (!buf || buflen < (int32_t)s.size() + 1) return fail(FITOCT_E_ARG, "buffer too small");
    memcpy(buf, s.c_str(), s.size() + 1);
    return FITOCT_OK;
  });
}

int32_t fitoct_output_rows(const fitoct_problem* prob, int32_t n_lead, int64_t n_rows,
                           const double* raw, double* out) {
  return guarded(__func__, [&]() -> int32_t {
    int rc = check_layout_problem(prob);
    if (rc) return rc;
    if (n_lead < 0 || n_rows < 0 || (n_rows > 0 && (!raw || !out)))
      return fail(FITOCT_E_ARG, "bad buffers");
    const std::vector<OutCol> lay = out_layout(prob);
    const int D = model_dim(prob->prior_type, prob->Nn);
    const int64_t w_in = n_lead + D + 1, w_out = n_lead + (int64_t)lay.size();
    for (int64_t r = 0; r < n_rows; ++r) {
      const double* src = raw + r * w_in;
      double* dst = out + r * w_out;
      for (int j = 0; j < n_lead; ++j) dst[j] = src[j];
      fill_row(prob, lay, src + n_lead, dst + n_lead);
    }
    return FITOCT_OK;
  });
}

int32_t fitoct_write_stan_csv(const char* path, const fitoct_problem* prob,
                              const fitoct_config* cfg, int32_t chain, const double* raw,
                              double stepsize, const double* inv_metric, double warmup_s,
                              double sampling_s) {
  try {
    int rc = check_layout_problem(prob);
    if (rc) return rc;
    if (!path || !cfg || !raw) return fail(FITOCT_E_ARG, "NULL argument");
    if (chain < 0 || chain >= cfg->chains) return fail(FITOCT_E_ARG, "chain index out of range");
    const int D = model_dim(prob->prior_type, prob->Nn), ncols = D + 8;
    const int W = cfg->warmup, S = cfg->samples;
    const int rows = cfg->save_warmup ? W + S : S;
    const std::vector<OutCol> lay = out_layout(prob);
    FILE* f = fopen(path, "w");
    if (!f) return fail(FITOCT_E_ARG, std::string("cannot open ") + path + " for writing");
    write_header_common(f, prob);
    fputs("# method = sample (Default)\n#   sample\n", f);
    fprintf(f, "#     num_samples = %d\n#     num_warmup = %d\n#     save_warmup = %d\n", S, W,
            cfg->save_warmup ? 1 : 0);
    fputs("#     thin = 1 (Default)\n#     adapt\n", f);
    fprintf(f, "#       engaged = %d\n#       gamma = %g\n#       delta = %g\n", cfg->adapt_engaged ? 1 : 0,
            cfg->gamma, cfg->adapt_delta);
    fprintf(f, "#       kappa = %g\n#       t0 = %g\n#       init_buffer = %d\n", cfg->kappa, cfg->t0,
            cfg->init_buffer);
    fprintf(f, "#       term_buffer = %d\n#       window = %d\n", cfg->term_buffer, cfg->window);
    fputs("#     algorithm = hmc (Default)\n#       hmc\n#         engine = nuts (Default)\n"
          "#           nuts\n", f);
    fprintf(f, "#             max_depth = %d\n", cfg->max_treedepth);
    fputs("#         metric = diag_e (Default)\n#         metric_file =  (Default)\n", f);
    fprintf(f, "#         stepsize = %g\n#         stepsize_jitter = 0 (Default)\n", cfg->stepsize);
    write_header_tail(f, prob, (long long)cfg->chain_offset + chain + 1,
                      (unsigned long long)cfg->seed, path);
    for (int j = 0; j < 7; ++j) fprintf(f, "%s,", kSampler[j]);
    for (size_t j = 0; j < lay.size(); ++j)
      fprintf(f, "%s%s", lay[j].name.c_str(), j + 1 < lay.size() ? "," : "\n");
    std::vector<double> o(7 + lay.size());
    auto put_row = [&](const double* r) {
      for (int j = 0; j < 7; ++j) o[j] = r[j];
      fill_row(prob, lay, r + 7, o.data() + 7);
      for (size_t j = 0; j < o.size(); ++j) {
        put_num(f, o[j]);
        fputc(j + 1 < o.size() ? ',' : '\n', f);
      }
    };
    const int wrows = cfg->save_warmup ? W : 0;
    for (int i = 0; i < wrows; ++i) put_row(raw + (size_t)i * ncols);
    // CmdStan prints the adaptation block between the warmup and sampling draws
    if (cfg->adapt_engaged && W > 0) {
      fputs("# Adaptation terminated\n# Step size = ", f);
      put_num(f, stepsize);
      fputs("\n# Diagonal elements of inverse mass matrix:\n# ", f);
      for (int j = 0; j < D; ++j) {
        put_num(f, inv_metric ? inv_metric[j] : 1.0);
        fputs(j + 1 < D ? ", " : "\n", f);
      }
    }
    for (int i = wrows; i < rows; ++i) put_row(raw + (size_t)i * ncols);
    fputs("# \n", f);
    // fixed-point, as CmdStan prints it (rstan reads the numbers before "seconds")
    fprintf(f, "#  Elapsed Time: %.6f seconds (Warm-up)\n", warmup_s);
    fprintf(f, "#                %.6f seconds (Sampling)\n", sampling_s);
    fprintf(f, "#                %.6f seconds (Total)\n# \n", warmup_s + sampling_s);
    const bool ok = !ferror(f);
    if (fclose(f) != 0 || !ok) return fail(FITOCT_E_ARG, std::string("write error on ") + path);
    return FITOCT_OK;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "fitoct_write_stan_csv: out of memory");
  }
}

int32_t fitoct_write_vb_csv(const char* path, const fitoct_problem* prob,
                            const fitoct_vb_config* cfg, const double* mu, double mean_sumr2,
                            int32_t n, const double* q, const double* log_p, const double* log_g,
                            const double* sumr2, double eta) {
  try {
    int rc = check_layout_problem(prob);
    if (rc) return rc;
    if (!path || !cfg || !mu || n < 0 || (n > 0 && (!q || !log_p || !log_g)))
      return fail(FITOCT_E_ARG, "NULL argument");
    const int fam = prob->prior_type, Nn = prob->Nn, D = model_dim(fam, Nn);
    const std::vector<OutCol> lay = out_layout(prob);
    FILE* f = fopen(path, "w");
    if (!f) return fail(FITOCT_E_ARG, std::string("cannot open ") + path + " for writing");
    write_header_common(f, prob);
    fputs("# method = variational\n#   variational\n#     algorithm = meanfield (Default)\n"
          "#       meanfield\n", f);
    fprintf(f, "#     iter = %d\n#     grad_samples = %d\n#     elbo_samples = %d\n", cfg->iter,
            cfg->grad_samples, cfg->elbo_samples);
    fprintf(f, "#     eta = %g\n#     adapt\n#       engaged = %d\n#       iter = %d\n", cfg->eta,
            cfg->adapt_engaged ? 1 : 0, cfg->adapt_iter);
    fprintf(f, "#     tol_rel_obj = %g\n#     eval_elbo = %d\n#     output_samples = %d\n",
            cfg->tol_rel_obj, cfg->eval_elbo, cfg->output_samples);
    write_header_tail(f, prob, 1, (unsigned long long)cfg->seed, path);
    for (int j = 0; j < 3; ++j) fprintf(f, "%s,", kVbLead[j]);
    for (size_t j = 0; j < lay.size(); ++j)
      fprintf(f, "%s%s", lay[j].name.c_str(), j + 1 < lay.size() ? "," : "\n");
    fputs("# Stepsize adaptation complete.\n# eta = ", f);
    put_num(f, eta);
    fputc('\n', f);
    std::vector<double> r(D + 1), o(3 + lay.size());
    auto put_row = [&](const double* qi, double lp, double lg, double s2) {
      constrain(fam, Nn, qi, r.data());
      r[D] = s2 / prob->N;
      o[0] = 0.0;
      o[1] = lp;
      o[2] = lg;
      fill_row(prob, lay, r.data(), o.data() + 3);
      for (size_t j = 0; j < o.size(); ++j) {
        put_num(f, o[j]);
        fputc(j + 1 < o.size() ? ',' : '\n', f);
      }
    };
    // first row: the mean of the approximation (CmdStan's convention)
    put_row(mu, 0.0, 0.0, mean_sumr2);
    for (int i = 0; i < n; ++i)
      put_row(q + (size_t)i * D, log_p[i], log_g[i], sumr2 ? sumr2[i] : NAN);
    const bool ok = !ferror(f);
    if (fclose(f) != 0 || !ok) return fail(FITOCT_E_ARG, std::string("write error on ") + path);
    return FITOCT_OK;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "fitoct_write_vb_csv: out of memory");
  }
}

int32_t fitoct_progress_line(int64_t done, int64_t total, int32_t warmup, int32_t samples,
                             char* buf, int32_t buflen) {
  if (total <= 0 || done < 0 || warmup < 0 || samples < 1 || !buf || buflen < 80)
    return fail(FITOCT_E_ARG, "bad progress arguments");
  if (done > total) done = total;
  const int64_t n = (int64_t)warmup + samples;
  // 4 f = (k - 1) + p / 100 with p in [0, 100]: k = 4, p = 100 at the end (server.R:469)
  const int64_t quarter_pct = 400 * done / total;          // floor(400 f)
  const int k = (int)std::min<int64_t>(4, quarter_pct / 100 + 1);
  const int p = (int)(quarter_pct - 100 * (int64_t)(k - 1));
  const long long it = (long long)((p * n + 50) / 100);
  const int w = snprintf(nullptr, 0, "%lld", (long long)n);
  snprintf(buf, (size_t)buflen, "Chain %d: Iteration: %*lld / %lld [%3d%%]  (%s)", k, w,
           it, (long long)n, p, it <= warmup ? "Warmup" : "Sampling");
  return (int32_t)(100 * done / total);
}

int32_t fitoct_expgp_curves(const fitoct_problem* prob, int32_t n, const double* theta,
                            const double* ygp, double* dL, double* m, double* resid,
                            double* br) {
  try {
    if (!prob || !prob->x || !prob->y || !prob->uy || prob->N < 2)
      return fail(FITOCT_E_ARG, "need a problem with x, y, uy and N >= 2");
    if (n < 0 || (n > 0 && !theta)) return fail(FITOCT_E_ARG, "bad buffers");
    const bool mono = prob->prior_type == FITOCT_MODEL_MONOEXP;
    if (!mono && n > 0 && !ygp) return fail(FITOCT_E_ARG, "yGP is required for the ExpGP model");
    const int N = prob->N, Nn = mono ? 0 : prob->Nn;
    std::vector<double> B, xg;
    if (!mono) {
      if (prob->B) {
        B.assign(prob->B, prob->B + (size_t)N * Nn);
      } else {
        const int rc = build_basis(prob, B, xg);
        if (rc) return rc;
      }
    }
    const double c = (double)prob->data_type;
    for (int s = 0; s < n; ++s) {
      const double* th = theta + (size_t)s * 3;
      double acc = 0.0;
      for (int i = 0; i < N; ++i) {
        double d = 0.0;   // dL_i = B_i . yGP   
        for (int k = 0; k < Nn; ++k) d += B[(size_t)i * Nn + k] * ygp[(size_t)s * Nn + k];
        // m_i = theta1 + theta2 exp(-c x_i / (theta3 (1 + dL_i)))   (ui.R:88, synthData.R:22)
        const double mi = th[0] + th[1] * exp(-c * prob->x[i] / (th[2] * (1.0 + d)));
        const double ri = (prob->y[i] - mi) / prob->uy[i];
        acc += ri * ri;
        const size_t o = (size_t)s * N + i;
        if (dL) dL[o] = d;
        if (m) m[o] = mi;
        if (resid) resid[o] = ri;
      }
      if (br) br[s] = acc / N;
    }
    return FITOCT_OK;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "fitoct_expgp_curves: out of memory");
  }
}

}  // extern "C"
