// Host-only parts of libfitoct: GP basis precompute (fp64 Cholesky), model
// layout / column names, and the rstan-style convergence diagnostics.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <string>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"

namespace fitoct {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// --------------------------------------------------------------------------
// GP basis: B = K(x~, xGP) (K(xGP,xGP) + nugget I)^-1   
// --------------------------------------------------------------------------
static double se_kernel(double d, double rho, int conv) {
  if (conv == 0) return exp(-(d * d) / (2.0 * rho * rho));  // Stan cov_exp_quad
  const double s = d / rho;
  return exp(-s * s);                                          // RMgauss(scale = rho)
}

int build_basis(const fitoct_problem* p, std::vector<double>& B, std::vector<double>& xg) {
  const int N = p->N, Nn = p->Nn;
  if (N < 2 || Nn < 2) return fail(FITOCT_E_ARG, "need N >= 2 and Nn >= 2");
  double xmin = p->x[0], xmax = p->x[0];
  for (int i = 1; i < N; ++i) {
    xmin = std::min(xmin, p->x[i]);
    xmax = std::max(xmax, p->x[i]);
  }
  if (!(xmax > xmin)) return fail(FITOCT_E_ARG, "x must not be constant");
  const double rho = (p->rho > 0.0) ? p->rho : 1.0 / Nn;  // FitOCT.R:119
  xg.assign(Nn, 0.0);
  // server.R:627-631
  if (p->grid_type == FITOCT_GRID_INTERNAL) {
    const double dx = 1.0 / (Nn + 1);
    for (int k = 0; k < Nn; ++k) xg[k] = dx / 2 + (1.0 - dx) * k / (Nn - 1);
  } else if (p->grid_type == FITOCT_GRID_EXTREMAL) {
    for (int k = 0; k < Nn; ++k) xg[k] = (double)k / (Nn - 1);
  } else {
    return fail(FITOCT_E_ARG, "grid_type must be internal (0) or extremal (1)");
  }
  // Cholesky of K_GG (row-major lower triangle)
  std::vector<double> L(Nn * Nn, 0.0);
  for (int i = 0; i < Nn; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = se_kernel(xg[i] - xg[j], rho, p->kernel_conv) + (i == j ? p->nugget : 0.0);
      for (int k = 0; k < j; ++k) s -= L[i * Nn + k] * L[j * Nn + k];
      if (i == j) {
        if (!(s > 0.0)) return fail(FITOCT_E_ARG, "K(xGP,xGP) not positive definite (raise nugget)");
        L[i * Nn + i] = sqrt(s);
      } else {
        L[i * Nn + j] = s / L[j * Nn + j];
      }
    }
  B.assign((size_t)N * Nn, 0.0);
  std::vector<double> z(Nn);
  for (int i = 0; i < N; ++i) {
    const double xt = (p->x[i] - xmin) / (xmax - xmin);   // server.R:635
    // solve L z = k_i ; L^T b = z
    for (int a = 0; a < Nn; ++a) {
      double s = se_kernel(xt - xg[a], rho, p->kernel_conv);
      for (int k = 0; k < a; ++k) s -= L[a * Nn + k] * z[k];
      z[a] = s / L[a * Nn + a];
    }
    for (int a = Nn - 1; a >= 0; --a) {
      double s = z[a];
      for (int k = a + 1; k < Nn; ++k) s -= L[k * Nn + a] * B[(size_t)i * Nn + k];
      B[(size_t)i * Nn + a] = s / L[a * Nn + a];
    }
  }
  return FITOCT_OK;
}

int model_dim(int prior, int Nn) {
  switch (prior) {
    case FITOCT_PRIOR_NORMAL: return Nn + 5;
    case FITOCT_PRIOR_LASSO: return Nn + 4;
    case FITOCT_PRIOR_HORSESHOE: return 3 * Nn + 6;
    case FITOCT_MODEL_MONOEXP: return 3;
    default: return -1;
  }
}

static const char* kSamplerCols[7] = {"lp__", "accept_stat__", "stepsize__", "treedepth__",
                                      "n_leapfrog__", "divergent__", "energy__"};

std::string column_name(int prior, int Nn, int i) {
  const int D = model_dim(prior, Nn);
  if (i < 0 || D < 0 || i >= D + 8) return "";
  if (i < 7) return kSamplerCols[i];
  if (i == D + 7) return "br";
  const int k = i - 7;
  char buf[64];
  if (k < 3) {
    snprintf(buf, sizeof buf, "theta.%d", k + 1);
    return buf;
  }
  if (k == D - 1) return "sigma";
  const int r = k - 3;
  if (prior == FITOCT_PRIOR_HORSESHOE) {
    if (r < Nn) snprintf(buf, sizeof buf, "z.%d", r + 1);
    else if (r == Nn) snprintf(buf, sizeof buf, "r1_global");
    else if (r == Nn + 1) snprintf(buf, sizeof buf, "r2_global");
    else if (r < 2 * Nn + 2) snprintf(buf, sizeof buf, "r1_local.%d", r - Nn - 1);
    else snprintf(buf, sizeof buf, "r2_local.%d", r - 2 * Nn - 1);
    return buf;
  }
  if (r < Nn) {
    snprintf(buf, sizeof buf, "yGP.%d", r + 1);
    return buf;
  }
  return "lambda";
}

// --------------------------------------------------------------------------
// diagnostics (stan::analyze, as printed by rstan::summary)
// --------------------------------------------------------------------------
static double mean_of(const double* x, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += x[i];
  return s / n;
}
static double var_of(const double* x, int n) {  // sample variance (n-1)
  const double m = mean_of(x, n);
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += (x[i] - m) * (x[i] - m);
  return s / (n - 1);
}

// potential scale reduction on already-split chains c[m][n]
static double psr(const std::vector<const double*>& c, int n) {
  const int m = (int)c.size();
  std::vector<double> cm(m), cv(m);
  for (int j = 0; j < m; ++j) {
    cm[j] = mean_of(c[j], n);
    cv[j] = var_of(c[j], n);
  }
  const double B = n * var_of(cm.data(), m);
  const double W = mean_of(cv.data(), m);
  return sqrt((B / W + n - 1) / n);
}

// stan::analyze::compute_effective_sample_size on already-split chains
static double ess_chains(const std::vector<const double*>& c, int n) {
  const int m = (int)c.size();
  std::vector<double> cm(m), cvar(m);
  for (int j = 0; j < m; ++j) {
    cm[j] = mean_of(c[j], n);
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += (c[j][i] - cm[j]) * (c[j][i] - cm[j]);
    cvar[j] = s / (n - 1);  // acov(0) * n/(n-1)
  }
  auto acov_mean = [&](int lag) {  // mean over chains of the biased autocovariance
    double tot = 0.0;
    for (int j = 0; j < m; ++j) {
      double s = 0.0;
      for (int i = 0; i + lag < n; ++i) s += (c[j][i] - cm[j]) * (c[j][i + lag] - cm[j]);
      tot += s / n;
    }
    return tot / m;
  };
  const double mean_var = mean_of(cvar.data(), m);
  double var_plus = mean_var * (n - 1) / n;
  if (m > 1) var_plus += var_of(cm.data(), m);
  if (!(var_plus > 0.0)) return NAN;
  std::vector<double> rho(n + 2, 0.0);
  double rho_even = 1.0;
  double rho_odd = 1.0 - (mean_var - acov_mean(1)) / var_plus;
  rho[0] = 1.0;
  rho[1] = rho_odd;
  int t = 1;
  while (t < n - 4 && (rho_even + rho_odd) > 0.0) {
    rho_even = 1.0 - (mean_var - acov_mean(t + 1)) / var_plus;
    rho_odd = 1.0 - (mean_var - acov_mean(t + 2)) / var_plus;
    if ((rho_even + rho_odd) >= 0.0) {
      rho[t + 1] = rho_even;
      rho[t + 2] = rho_odd;
    }
    t += 2;
  }
  const int max_t = t;
  if (rho_even > 0.0) rho[max_t + 1] = rho_even;
  t = 1;
  while (t <= max_t - 2) {
    if (rho[t + 1] + rho[t + 2] > rho[t - 1] + rho[t]) {
      rho[t + 1] = (rho[t - 1] + rho[t]) / 2.0;
      rho[t + 2] = rho[t + 1];
    }
    t += 2;
  }
  const double ess = (double)m * n;
  double tau = -1.0;
  for (int i = 0; i <= max_t; ++i) tau += 2.0 * rho[i];
  tau += rho[max_t + 1];
  tau = std::max(tau, 1.0 / log10(ess));
  return ess / tau;
}

int split_rhat_ess(const double* x, int chains, int n, double* rhat, double* ess) {
  if (chains < 1 || n < 4) return fail(FITOCT_E_ARG, "need >= 1 chain and >= 4 draws");
  const int h = n / 2;                 // drop the middle draw when n is odd
  std::vector<const double*> sp;
  for (int c = 0; c < chains; ++c) {
    const double* base = x + (size_t)c * n;
    sp.push_back(base);
    sp.push_back(base + (n - h));
  }
  bool constant = true;
  for (int c = 0; c < chains && constant; ++c)
    for (int i = 1; i < n; ++i)
      if (x[(size_t)c * n + i] != x[(size_t)c * n]) {
        constant = false;
        break;
      }
  if (rhat) *rhat = constant ? NAN : psr(sp, h);
  if (ess) *ess = constant ? NAN : ess_chains(sp, h);
  return FITOCT_OK;
}

// rank-normalised split-R-hat (Vehtari, Gelman, Simpson, Carpenter, Buerkner 2021)
static double inv_normal_cdf(double p) {
  // Acklam's rational approximation + one Newton step (|err| < 1e-13)
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02,
                             -2.759285104469687e+02, 1.383577518672690e+02,
                             -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02,
                             -1.556989798598866e+02, 6.680131188771972e+01,
                             -1.328068155288572e+01};
  static const double c[] = {-7.784894002430293e-03, -3.223964580411365e-01,
                             -2.400758277161838e+00, -2.549732539343734e+00,
                             4.374664141464968e+00, 2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01,
                             2.445134137142996e+00, 3.754408661907416e+00};
  double q, r, x;
  if (p < 0.02425) {
    q = sqrt(-2 * log(p));
    x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
        ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  } else if (p > 1 - 0.02425) {
    q = sqrt(-2 * log(1 - p));
    x = -(((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
        ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
  } else {
    q = p - 0.5;
    r = q * q;
    x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
        (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
  }
  const double e = 0.5 * erfc(-x / sqrt(2.0)) - p;
  const double u = e * sqrt(2 * M_PI) * exp(x * x / 2);
  return x - u / (1 + x * u / 2);
}

static void rank_normalise(const std::vector<double>& v, std::vector<double>& z) {
  const size_t S = v.size();
  std::vector<size_t> idx(S);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return v[a] < v[b]; });
  z.assign(S, 0.0);
  size_t i = 0;
  while (i < S) {  // average ranks for ties
    size_t j = i;
    while (j + 1 < S && v[idx[j + 1]] == v[idx[i]]) ++j;
    const double r = 0.5 * (double)(i + j) + 1.0;
    for (size_t k = i; k <= j; ++k) z[idx[k]] = inv_normal_cdf((r - 0.375) / (S + 0.25));
    i = j + 1;
  }
}

int rank_rhat(const double* x, int chains, int n, double* out) {
  if (chains < 1 || n < 4) return fail(FITOCT_E_ARG, "need >= 1 chain and >= 4 draws");
  const int h = n / 2;
  // split, then rank-normalise pooled split draws
  std::vector<double> pooled, folded;
  std::vector<int> off;
  for (int c = 0; c < chains; ++c)
    for (int half = 0; half < 2; ++half) {
      const double* base = x + (size_t)c * n + (half ? n - h : 0);
      for (int i = 0; i < h; ++i) pooled.push_back(base[i]);
    }
  std::vector<double> sorted(pooled);
  std::nth_element(sorted.begin(), sorted.begin() + sorted.size() / 2, sorted.end());
  double med = sorted[sorted.size() / 2];
  if (sorted.size() % 2 == 0) {
    const double lo = *std::max_element(sorted.begin(), sorted.begin() + sorted.size() / 2);
    med = 0.5 * (med + lo);
  }
  for (double v : pooled) folded.push_back(fabs(v - med));
  std::vector<double> z1, z2;
  rank_normalise(pooled, z1);
  rank_normalise(folded, z2);
  std::vector<const double*> c1, c2;
  for (int j = 0; j < 2 * chains; ++j) {
    c1.push_back(z1.data() + (size_t)j * h);
    c2.push_back(z2.data() + (size_t)j * h);
  }
  *out = std::max(psr(c1, h), psr(c2, h));
  return FITOCT_OK;
}

// --------------------------------------------------------------------------
// parameter transforms (Appendix A: positive parameters are log-transformed)
// --------------------------------------------------------------------------
bool log_transformed(int prior, int Nn, int j) {
  const int D = model_dim(prior, Nn);
  if (j < 3 || j == D - 1) return true;          // theta, sigma (mono: theta only, D = 3)
  switch (prior) {
    case FITOCT_PRIOR_NORMAL: return j == 3 + Nn;                 // lambda
    case FITOCT_PRIOR_HORSESHOE: return j >= 3 + Nn;              // r1/r2 global and local
    default: return false;                                        // yGP
  }
}

void constrain(int prior, int Nn, const double* q, double* out) {
  const int D = model_dim(prior, Nn);
  for (int j = 0; j < D; ++j) out[j] = log_transformed(prior, Nn, j) ? exp(q[j]) : q[j];
}

// Constants dropped from lp by Stan's `~` statements (log_prob<propto=true>)
// and restored by log_prob<propto=false>: one term per sampling statement of
// the model contract (Appendix A; horseShoePrior.stan:37-42).
double lp_constant(const fitoct_problem* p) {
  const double l2pi = log(2.0 * M_PI);
  const int Nn = p->Nn;
  double c = 0.0;
  if (!p->prior_PD) {
    c -= 0.5 * p->N * l2pi;
    for (int i = 0; i < p->N; ++i) c -= log(p->uy[i]);
  }
  if (p->prior_type == FITOCT_MODEL_MONOEXP) return c;
  // theta ~ multi_normal(theta0, Sigma0)
  const double* S = p->Sigma0;
  const double det = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) +
                     S[2] * (S[3] * S[7] - S[4] * S[6]);
  c += -1.5 * l2pi - 0.5 * log(det);
  c += -0.5 * l2pi - log(p->sigma_scale);        // sigma ~ normal(0, sigma_scale)
  if (p->prior_type == FITOCT_PRIOR_NORMAL) {
    const double rate = (p->lambda_conv == 0) ? 1.0 / p->lambda_rate : p->lambda_rate;
    c += -0.5 * Nn * l2pi + log(rate);           // yGP ~ normal(0, lambda), lambda ~ exp(rate)
  } else if (p->prior_type == FITOCT_PRIOR_HORSESHOE) {
    const double a = 0.5 * p->nu;
    c += -Nn * l2pi;                                    // z, r1_local ~ normal(0, 1)
    c += Nn * (a * log(a) - lgamma(a));                 // r2_local ~ inv_gamma(nu/2, nu/2)
    c += -0.5 * l2pi + 0.5 * log(0.5) - lgamma(0.5);    // r1_global, r2_global
  }
  return c;                                      // lasso: `target +=` only, no constant
}

}  // namespace fitoct

extern "C" int32_t fitoct_constrain(int32_t prior_type, int32_t Nn, int32_t n, const double* q,
                                    double* out) {
  using namespace fitoct;
  const int D = model_dim(prior_type, Nn);
  if (D < 0) return fail(FITOCT_E_ARG, "unknown prior_type");
  if (n < 0 || (n > 0 && (!q || !out))) return fail(FITOCT_E_ARG, "bad buffers");
  for (int i = 0; i < n; ++i) constrain(prior_type, Nn, q + (size_t)i * D, out + (size_t)i * D);
  return FITOCT_OK;
}

extern "C" int32_t fitoct_mono_initial_theta(int32_t N, const double* x, const double* y,
                                             int32_t data_type, double* theta) {
  using namespace fitoct;
  try {
    if (N < 2 || N > FITOCT_MAX_BINS || !x || !y || !theta)
      return fail(FITOCT_E_ARG, "need x, y with 2 <= N <= FITOCT_MAX_BINS and theta_out");
    for (int i = 0; i < N; ++i)
      if (!isfinite(x[i]) || !isfinite(y[i])) return fail(FITOCT_E_ARG, "x and y must be finite");
    std::vector<int> order(N);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return x[a] < x[b]; });
    std::vector<double> xs(N), ys(N);
    for (int i = 0; i < N; ++i) {
      xs[i] = x[order[i]];
      ys[i] = y[order[i]];
    }
    const int tail = std::min(N, std::max(3, N / 10));
    std::vector<double> t(ys.end() - tail, ys.end());
    std::sort(t.begin(), t.end());
    const double t1 = (tail % 2) ? t[tail / 2] : 0.5 * (t[tail / 2 - 1] + t[tail / 2]);
    double amax = -INFINITY;
    for (int i = 0; i < N; ++i) amax = std::max(amax, ys[i] - t1);
    const double thr = 0.05 * std::max(amax, 1e-12);
    double sx = 0, sy = 0;
    int n = 0;
    for (int i = 0; i < N; ++i)
      if (ys[i] - t1 > thr) {
        sx += xs[i];
        sy += log(ys[i] - t1);
        ++n;
      }
    double slope, icpt;
    if (n >= 3) {   // least-squares line through (x, log(y - theta1))
      const double mx = sx / n, my = sy / n;
      double sxy = 0, sxx = 0;
      for (int i = 0; i < N; ++i)
        if (ys[i] - t1 > thr) {
          sxy += (xs[i] - mx) * (log(ys[i] - t1) - my);
          sxx += (xs[i] - mx) * (xs[i] - mx);
        }
      slope = sxx > 0 ? sxy / sxx : -1.0 / std::max(xs[N - 1] - xs[0], 1e-12);
      icpt = my - slope * mx;
    } else {
      slope = -1.0 / std::max(xs[N - 1] - xs[0], 1e-12);
      icpt = log(std::max(amax, 1e-12));
    }
    slope = std::min(slope, -1e-12);
    theta[0] = std::max(fabs(t1), 1e-6);
    theta[1] = std::max(exp(icpt), 1e-6);
    theta[2] = std::max((double)data_type / -slope, 1e-6);
    return FITOCT_OK;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "fitoct_mono_initial_theta: out of memory");
  }
}

int fitoct::chain_outcome(int C, int D, const int* st, double* eps, double* minv, double* q) {
  // A chain that timed out may have left a speculative booking in flight while it wrote
  // its final state, so its warm-restart outputs could be torn: they are reported as NaN
  // (fitoct_plan_set_init rejects them).  Done on the host, not in the kernel: any code
  // added to the sampler's finishing action moved the headline kernel's layout and cost
  // 2 % (profiles/r04_ab_regression.txt).
  for (int c = 0; c < C; ++c)
    if (st[c] == FITOCT_E_TIMEOUT) {
      if (eps) eps[c] = NAN;
      for (int j = 0; j < D; ++j) {
        if (minv) minv[(size_t)c * D + j] = NAN;
        if (q) q[(size_t)c * D + j] = NAN;
      }
    }
  // a chain's own failure is reported before the cancellations it may have caused
  // (a multi-device plan cancels the other devices' chains when one fails)
  for (int c = 0; c < C; ++c)
    if (st[c] != 0 && st[c] != FITOCT_E_CANCELLED) return c;
  for (int c = 0; c < C; ++c)
    if (st[c] != 0) return c;
  return -1;
}

// Not in include/fitoct.h: the host bookkeeping of fitoct_plan_download, exported for the
// CPU test suite (tests/test_abi.py), which cannot make a kernel time out.
extern "C" int32_t fitoct_internal_chain_outcome(int32_t C, int32_t D, const int32_t* status,
                                                 double* stepsize, double* inv_metric,
                                                 double* last_q) {
  return fitoct::chain_outcome(C, D, status, stepsize, inv_metric, last_q);
}

extern "C" const char* fitoct_last_error(void) { return fitoct::g_last_error.c_str(); }
