// Host drivers of FitOCTLib::fitExpGP's other two methods (FitOCT.R:42,
// ui.R:107-114): method='optim' (rstan::optimizing: L-BFGS + optimHess) and
// method='vb' (rstan::vb: mean-field ADVI).  Both are sequences of batched
// density/gradient evaluations; each batch is one launch of the sampler's
// gradient kernel through a fitoct_evaluator (problem staged once in HBM).
//
// The algorithms restate Stan's services (stan/optimization/bfgs.hpp,
// bfgs_linesearch.hpp, lbfgs_update.hpp; stan/variational/advi.hpp,
// families/normal_meanfield.hpp), which are not in /root/reference (rstan is
// an external dependency): parity against rstan is unpinned, the
// tests pin the optimum against an independent optimiser and the ADVI
// trajectory against the CPU oracle's restatement (oracle/fitoct_oracle.c).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <limits>
#include <numeric>
#include <string>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"
#include "philox.h"

namespace fitoct {
namespace {

using Vec = std::vector<double>;

double dot(const Vec& a, const Vec& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}
double norm(const Vec& a) { return sqrt(dot(a, a)); }

struct DeviceError {
  int code;
};

// theta = theta0, lambda at its prior mean (normal family), everything else 0:
// the centre of the sampler's initialisation (nuts_device.hip act_init_start)
void default_init(const fitoct_problem* p, Vec& q) {
  const int D = model_dim(p->prior_type, p->Nn);
  q.assign(D, 0.0);
  for (int j = 0; j < 3; ++j) q[j] = log(p->theta0[j]);
  if (p->prior_type == FITOCT_PRIOR_NORMAL) {
    const double rate = (p->lambda_conv == 0) ? 1.0 / p->lambda_rate : p->lambda_rate;
    q[3 + p->Nn] = -log(rate);
  }
}

// RAII owner of an evaluator
struct Evaluator {
  fitoct_evaluator* ev = nullptr;
  int D = 0;
  long long points = 0;
  ~Evaluator() { fitoct_evaluator_destroy(ev); }
  void run(int n, const double* q, int jacobian, int normalised, double* lp, double* g,
           double* s2) {
    const int rc = fitoct_evaluator_run(ev, n, q, jacobian, normalised, lp, g, s2);
    if (rc) throw DeviceError{rc};
    points += n;
  }
};

// ============================================================================
// L-BFGS (minimises f = -lp)
// ============================================================================
struct Objective {
  Evaluator* E;
  int jacobian;
  // 0 = finite value and gradient
  int operator()(const Vec& x, double& f, Vec& g) {
    double lp;
    E->run(1, x.data(), jacobian, 0, &lp, g.data(), nullptr);
    if (!isfinite(lp)) return 1;
    for (double& v : g) {
      v = -v;
      if (!isfinite(v)) return 1;
    }
    f = -lp;
    return 0;
  }
};

// minimiser on [lo, hi] of the cubic c with c(0) = 0, c'(0) = df0, c(x1) = f1,
// c'(x1) = df1 (bfgs_linesearch.hpp CubicInterp, one-point form)
double cubic_interp(double df0, double x1, double f1, double df1, double lo, double hi) {
  const double c3 = (-12.0 * f1 + 6.0 * x1 * (df0 + df1)) / (x1 * x1 * x1);
  const double c2 = -(4.0 * df0 + 2.0 * df1) / x1 + 6.0 * f1 / (x1 * x1);
  const double c1 = df0;
  auto c = [&](double x) { return x * (c1 + x * (0.5 * c2 + x * c3 / 6.0)); };
  double best = lo, fbest = c(lo);
  auto consider = [&](double x) {
    if (x >= lo && x <= hi && isfinite(x)) {
      const double v = c(x);
      if (v < fbest) {
        best = x;
        fbest = v;
      }
    }
  };
  consider(hi);
  const double disc = c2 * c2 - 2.0 * c1 * c3;
  if (disc >= 0.0 && c3 != 0.0) {
    const double t = sqrt(disc);
    consider(-(c2 + t) / c3);
    consider(-(c2 - t) / c3);
  } else if (c3 == 0.0 && c2 > 0.0) {
    consider(-c1 / c2);
  }
  return best;
}

// minimiser of the cubic Hermite interpolant through (a, fa, da), (b, fb, db)
// (two-point CubicInterp), safeguarded into the middle 80 % of the bracket
double cubic_interp2(double a, double fa, double da, double b, double fb, double db) {
  const double lo = std::min(a, b), hi = std::max(a, b), w = hi - lo;
  const double d1 = da + db - 3.0 * (fa - fb) / (a - b);
  const double disc = d1 * d1 - da * db;
  double x = 0.5 * (a + b);
  if (disc >= 0.0) {
    const double d2 = (b > a ? 1.0 : -1.0) * sqrt(disc);
    const double den = db - da + 2.0 * d2;
    if (den != 0.0) x = b - (b - a) * (db + d2 - d1) / den;
  }
  if (!isfinite(x) || x < lo + 0.1 * w || x > hi - 0.1 * w) x = 0.5 * (a + b);
  return x;
}

struct LineSearchResult {
  double alpha, f;
  Vec x, g;
};

// Strong-Wolfe line search (bfgs_linesearch.hpp WolfeLineSearch / WolfLSZoom,
// Nocedal & Wright Alg. 3.5-3.6): c1 = 1e-4, c2 = 0.9, min step 1e-12,
// 40 bracketing steps, 10 halvings after a non-finite evaluation.
int wolfe_search(Objective& F, double alpha1, const Vec& x0, double f0, const Vec& g0,
                 const Vec& p, LineSearchResult& out) {
  const double c1 = 1e-4, c2 = 0.9, min_alpha = 1e-12;
  const int max_its = 40, max_restarts = 10;
  const int D = (int)x0.size();
  const double dfp0 = dot(g0, p);
  if (!(dfp0 < 0.0)) return 1;
  Vec x1(D), g1(D);
  double f1 = 0.0, alpha_prev = 0.0, f_prev = f0, dfp_prev = dfp0;
  int its = 0, restarts = 0;
  auto eval_at = [&](double a, double& f, Vec& g, Vec& x) {
    for (int j = 0; j < D; ++j) x[j] = x0[j] + a * p[j];
    return F(x, f, g);
  };
  auto zoom = [&](double alo, double flo, double dlo, double ahi, double fhi, double dhi) -> int {
    for (int it = 1;; ++it) {
      if (fabs(alo - ahi) < min_alpha) return 1;
      double a = (it % 5) ? cubic_interp2(alo, flo, dlo, ahi, fhi, dhi) : 0.5 * (alo + ahi);
      double f;
      while (eval_at(a, f, g1, x1)) {  // non-finite: back off towards the low end
        a = 0.5 * (a + alo);
        if (fabs(a - alo) < min_alpha) return 1;
      }
      const double d = dot(g1, p);
      if (f > f0 + a * c1 * dfp0 || f >= flo) {
        ahi = a;
        fhi = f;
        dhi = d;
      } else {
        if (fabs(d) <= -c2 * dfp0) {
          out.alpha = a;
          out.f = f;
          out.x = x1;
          out.g = g1;
          return 0;
        }
        if (d * (ahi - alo) >= 0.0) {
          ahi = alo;
          fhi = flo;
          dhi = dlo;
        }
        alo = a;
        flo = f;
        dlo = d;
      }
      if (it > 100) return 1;
    }
  };
  for (;;) {
    if (its >= max_its) return 1;
    if (eval_at(alpha1, f1, g1, x1)) {
      if (restarts >= max_restarts) return 1;
      alpha1 = 0.5 * (alpha_prev + alpha1);
      ++restarts;
      continue;
    }
    restarts = 0;
    const double dfp1 = dot(g1, p);
    if (f1 > f0 + alpha1 * c1 * dfp0 || (f1 >= f_prev && its > 0))
      return zoom(alpha_prev, f_prev, dfp_prev, alpha1, f1, dfp1);
    if (fabs(dfp1) <= -c2 * dfp0) {
      out.alpha = alpha1;
      out.f = f1;
      out.x = x1;
      out.g = g1;
      return 0;
    }
    if (dfp1 >= 0.0) return zoom(alpha1, f1, dfp1, alpha_prev, f_prev, dfp_prev);
    alpha_prev = alpha1;
    f_prev = f1;
    dfp_prev = dfp1;
    alpha1 *= 10.0;
    ++its;
  }
}

// limited-memory inverse-Hessian (lbfgs_update.hpp): two-loop recursion
struct LbfgsMemory {
  int m;
  std::vector<Vec> s, y;
  Vec rho;
  double gamma = 1.0;
  void clear() {
    s.clear();
    y.clear();
    rho.clear();
    gamma = 1.0;
  }
  void update(const Vec& sk, const Vec& yk) {
    const double sy = dot(sk, yk);
    if (!(sy > 0.0)) return;  // keep the approximation positive definite
    if ((int)s.size() == m) {
      s.erase(s.begin());
      y.erase(y.begin());
      rho.erase(rho.begin());
    }
    s.push_back(sk);
    y.push_back(yk);
    rho.push_back(1.0 / sy);
    gamma = sy / dot(yk, yk);
  }
  void direction(const Vec& g, Vec& p) const {
    const int D = (int)g.size(), k = (int)s.size();
    p.resize(D);
    for (int j = 0; j < D; ++j) p[j] = -g[j];
    Vec a(k);
    for (int i = k - 1; i >= 0; --i) {
      a[i] = rho[i] * dot(s[i], p);
      for (int j = 0; j < D; ++j) p[j] -= a[i] * y[i][j];
    }
    for (int j = 0; j < D; ++j) p[j] *= gamma;
    for (int i = 0; i < k; ++i) {
      const double b = rho[i] * dot(y[i], p);
      for (int j = 0; j < D; ++j) p[j] += (a[i] - b) * s[i][j];
    }
  }
};

int run_optimize(const fitoct_problem* prob, const fitoct_optim_config* c, const double* init_q,
                 fitoct_optim_result* res) {
  const int D = model_dim(prob->prior_type, prob->Nn);
  if (D < 0) return fail(FITOCT_E_ARG, "unknown prior_type");
  Evaluator E;
  int rc = fitoct_evaluator_create(prob, std::max(2 * D, 1), c->precision, c->device, &E.ev);
  if (rc) return rc;
  E.D = D;
  Objective F{&E, c->jacobian};
  Vec x, g(D), p(D);
  if (init_q) x.assign(init_q, init_q + D);
  else default_init(prob, x);
  double f;
  if (F(x, f, g)) return fail(FITOCT_E_INIT, "log density not finite at the initial point");
  const double eps = std::numeric_limits<double>::epsilon();
  LbfgsMemory mem{std::max(1, c->history)};
  p = g;
  for (double& v : p) v = -v;
  int term = FITOCT_TERM_MAXIT, it = 0;
  double alpha_prev = 0.0, f_prev = f;
  Vec g_prev = g, p_prev = p;
  bool fresh = true;  // first iteration or after a reset: -g direction, alpha = init_alpha
  while (true) {
    ++it;
    LineSearchResult ls;
    int lsrc;
    for (;;) {
      double alpha0 = c->init_alpha;
      if (!fresh) {
        alpha0 = std::min(1.0, 1.01 * cubic_interp(dot(g_prev, p_prev), alpha_prev, f - f_prev,
                                                   dot(g, p_prev) * alpha_prev, 1e-12, 1.0));
        if (!(alpha0 > 0.0)) alpha0 = 1.0;
      }
      lsrc = wolfe_search(F, alpha0, x, f, g, p, ls);
      if (lsrc == 0 || fresh) break;
      // line search failed: reset the Hessian approximation and retry once
      mem.clear();
      p = g;
      for (double& v : p) v = -v;
      fresh = true;
    }
    if (lsrc) {
      term = FITOCT_TERM_LSFAIL;
      break;
    }
    Vec s(D), yv(D);
    for (int j = 0; j < D; ++j) {
      s[j] = ls.x[j] - x[j];
      yv[j] = ls.g[j] - g[j];
    }
    f_prev = f;
    g_prev = g;
    p_prev = p;
    alpha_prev = ls.alpha;
    const double df = fabs(f_prev - ls.f);
    x = ls.x;
    f = ls.f;
    g = ls.g;
    fresh = false;
    // convergence tests (bfgs.hpp BFGSMinimizer::step)
    if (df < c->tol_obj) term = FITOCT_TERM_ABSF;
    else if (norm(g) < c->tol_grad) term = FITOCT_TERM_ABSGRAD;
    else if (df / std::max(std::max(fabs(f_prev), fabs(f)), 1.0) < c->tol_rel_obj * eps)
      term = FITOCT_TERM_RELF;
    else if (norm(s) < c->tol_param) term = FITOCT_TERM_ABSX;
    else if (it >= c->iter) term = FITOCT_TERM_MAXIT;
    else term = FITOCT_TERM_SUCCESS;
    mem.update(s, yv);
    mem.direction(g, p);
    if (term == FITOCT_TERM_SUCCESS &&
        fabs(dot(g, p)) / std::max(fabs(f), 1.0) < c->tol_rel_grad * eps)
      term = FITOCT_TERM_RELGRAD;
    if (term != FITOCT_TERM_SUCCESS) break;
  }
  // value, sumr2 at the optimum
  double lp, s2;
  E.run(1, x.data(), c->jacobian, 0, &lp, g.data(), &s2);
  memcpy(res->par, x.data(), sizeof(double) * D);
  res->value = lp;
  res->sumr2 = s2;
  res->iterations = it;
  res->termination = term;
  res->return_code = (term >= 0) ? 0 : 70;
  if (c->hessian && res->hessian) {
    // optimHess: central differences of the gradient, one batched launch
    const double h = c->hessian_step;
    Vec Q((size_t)2 * D * D), G((size_t)2 * D * D), L(2 * D);
    for (int j = 0; j < D; ++j)
      for (int sgn = 0; sgn < 2; ++sgn) {
        double* q = &Q[(size_t)(2 * j + sgn) * D];
        memcpy(q, x.data(), sizeof(double) * D);
        q[j] += sgn ? -h : h;
      }
    E.run(2 * D, Q.data(), c->jacobian, 0, L.data(), G.data(), nullptr);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        const double a = (G[(size_t)(2 * i) * D + j] - G[(size_t)(2 * i + 1) * D + j]) / (2 * h);
        const double b = (G[(size_t)(2 * j) * D + i] - G[(size_t)(2 * j + 1) * D + i]) / (2 * h);
        res->hessian[(size_t)i * D + j] = 0.5 * (a + b);
      }
  }
  res->n_evals = (int)E.points;
  return FITOCT_OK;
}

// ============================================================================
// mean-field ADVI
// ============================================================================
enum : uint32_t { ADVI_GRAD = 0xAD01u, ADVI_ELBO = 0xAD02u, ADVI_OUT = 0xAD03u };
// random streams: eta-adaptation candidate e -> stream e; then:
enum : uint32_t { STREAM_ELBO_INIT = 16, STREAM_SGA = 17, STREAM_OUT = 18 };

// standard normals eta[d], d < D, of draw `s` at iteration `it` (Box-Muller on
// Philox pairs; the oracle's advi restatement addresses the same numbers)
void normals(uint64_t seed, uint32_t stream, uint32_t tag, uint32_t it, uint32_t s, int D,
             double* eta) {
  const RngKey key = make_key(seed, stream);
  for (int d = 0; d < D; d += 2) {
    U4 c = {it, tag, s, (uint32_t)(d >> 1)};
    U4 r = philox4x32_10(c, key.k0, key.k1);
    const double u1 = u53(r.x, r.y), u2 = u53(r.z, r.w);
    const double rad = sqrt(-2.0 * log(1.0 - u1));
    eta[d] = rad * cos(2.0 * M_PI * u2);
    if (d + 1 < D) eta[d + 1] = rad * sin(2.0 * M_PI * u2);
  }
}

struct Meanfield {
  Vec mu, omega;
};

struct Advi {
  const fitoct_vb_config* c;
  Evaluator* E;
  int D;
  Vec Q, G, L, ETA;

  double entropy(const Meanfield& v) const {
    return 0.5 * D * (1.0 + log(2.0 * M_PI)) + std::accumulate(v.omega.begin(), v.omega.end(), 0.0);
  }
  // ELBO of each candidate (one launch for all); -inf where every draw was dropped
  void elbo(const std::vector<Meanfield*>& vs, const std::vector<uint32_t>& streams, uint32_t it,
            std::vector<double>& out) {
    const int n = c->elbo_samples, K = (int)vs.size();
    Q.resize((size_t)K * n * D);
    L.resize((size_t)K * n);
    ETA.resize(D);
    for (int k = 0; k < K; ++k)
      for (int s = 0; s < n; ++s) {
        normals(c->seed, streams[k], ADVI_ELBO, it, (uint32_t)s, D, ETA.data());
        double* q = &Q[((size_t)k * n + s) * D];
        for (int d = 0; d < D; ++d) q[d] = vs[k]->mu[d] + exp(vs[k]->omega[d]) * ETA[d];
      }
    E->run(K * n, Q.data(), 1, 1, L.data(), nullptr, nullptr);
    out.assign(K, 0.0);
    for (int k = 0; k < K; ++k) {
      double sum = 0.0;
      int dropped = 0;
      for (int s = 0; s < n; ++s) {
        const double v = L[(size_t)k * n + s];
        if (isfinite(v)) sum += v;
        else ++dropped;
      }
      out[k] = (dropped >= n) ? -INFINITY : sum / n + entropy(*vs[k]);
    }
  }
  // ELBO gradient of each candidate.  A draw whose log density or gradient is
  // not finite is dropped (it contributes 0; the mean stays over all draws, as
  // calc_ELBO does for its draws); ok[k] = 0 when every draw was dropped, and
  // the caller then takes a zero step.  Stan instead throws from calc_grad: the
  // restated model's hard boundary 1 + dL > 0 (Appendix A guard) is crossed by
  // unit-scale initial approximations often enough to make that unusable.
  void grad(const std::vector<Meanfield*>& vs, const std::vector<uint32_t>& streams, uint32_t it,
            std::vector<Meanfield>& out, std::vector<int>& ok) {
    const int n = c->grad_samples, K = (int)vs.size();
    Q.resize((size_t)K * n * D);
    G.resize((size_t)K * n * D);
    L.resize((size_t)K * n);
    std::vector<double> eta((size_t)K * n * D);
    for (int k = 0; k < K; ++k)
      for (int s = 0; s < n; ++s) {
        double* e = &eta[((size_t)k * n + s) * D];
        normals(c->seed, streams[k], ADVI_GRAD, it, (uint32_t)s, D, e);
        double* q = &Q[((size_t)k * n + s) * D];
        for (int d = 0; d < D; ++d) q[d] = vs[k]->mu[d] + exp(vs[k]->omega[d]) * e[d];
      }
    E->run(K * n, Q.data(), 1, 0, L.data(), G.data(), nullptr);
    out.assign(K, Meanfield{Vec(D, 0.0), Vec(D, 0.0)});
    ok.assign(K, 0);
    for (int k = 0; k < K; ++k) {
      for (int s = 0; s < n; ++s) {
        const double* g = &G[((size_t)k * n + s) * D];
        const double* e = &eta[((size_t)k * n + s) * D];
        bool valid = isfinite(L[(size_t)k * n + s]);
        for (int d = 0; d < D; ++d) valid = valid && isfinite(g[d]);
        if (!valid) continue;
        ok[k] = 1;
        for (int d = 0; d < D; ++d) {
          out[k].mu[d] += g[d];
          out[k].omega[d] += g[d] * e[d];
        }
      }
      if (!ok[k]) continue;
      for (int d = 0; d < D; ++d) {
        out[k].mu[d] /= n;
        out[k].omega[d] = out[k].omega[d] / n * exp(vs[k]->omega[d]) + 1.0;  // + entropy grad
      }
    }
  }
};

// adaGrad-style step of advi.hpp: history of squared gradients, eta / sqrt(iter)
void sga_step(Meanfield& v, const Meanfield& g, Meanfield& hist, int iter, double eta) {
  const double pre = 0.9, post = 0.1, tau = 1.0;
  const double es = eta / sqrt((double)iter);
  const int D = (int)v.mu.size();
  for (int d = 0; d < D; ++d) {
    if (iter == 1) {
      hist.mu[d] += g.mu[d] * g.mu[d];
      hist.omega[d] += g.omega[d] * g.omega[d];
    } else {
      hist.mu[d] = pre * hist.mu[d] + post * g.mu[d] * g.mu[d];
      hist.omega[d] = pre * hist.omega[d] + post * g.omega[d] * g.omega[d];
    }
    v.mu[d] += es * g.mu[d] / (tau + sqrt(hist.mu[d]));
    v.omega[d] += es * g.omega[d] / (tau + sqrt(hist.omega[d]));
  }
}

int run_vb(const fitoct_problem* prob, const fitoct_vb_config* c, const double* init_q,
           fitoct_vb_result* res) {
  const int D = model_dim(prob->prior_type, prob->Nn);
  if (D < 0) return fail(FITOCT_E_ARG, "unknown prior_type");
  if (c->iter < 1 || c->grad_samples < 1 || c->elbo_samples < 1 || c->eval_elbo < 1 ||
      c->output_samples < 0 || (c->adapt_engaged && c->adapt_iter < 1) || !(c->tol_rel_obj > 0.0))
    return fail(FITOCT_E_ARG, "bad vb config");
  if (!c->adapt_engaged && !(c->eta > 0.0)) return fail(FITOCT_E_ARG, "eta must be > 0");
  const double etas[5] = {100.0, 10.0, 1.0, 0.1, 0.01};
  const int K = c->adapt_engaged ? 5 : 1;
  const int cap = std::max({K * c->grad_samples, K * c->elbo_samples, 256});
  Evaluator E;
  int rc = fitoct_evaluator_create(prob, cap, c->precision, c->device, &E.ev);
  if (rc) return rc;
  E.D = D;
  Advi A{c, &E, D, {}, {}, {}, {}};
  Vec q0;
  if (init_q) q0.assign(init_q, init_q + D);
  else default_init(prob, q0);
  const Meanfield init{q0, Vec(D, 0.0)};

  double eta = c->eta;
  if (c->adapt_engaged) {
    // five candidate step sizes run side by side from the same start
    std::vector<Meanfield> cand(K, init), hist(K, Meanfield{Vec(D, 0.0), Vec(D, 0.0)}), g;
    std::vector<Meanfield*> vs;
    std::vector<uint32_t> streams;
    for (int k = 0; k < K; ++k) {
      vs.push_back(&cand[k]);
      streams.push_back((uint32_t)k);
    }
    std::vector<int> ok;
    for (int it = 1; it <= c->adapt_iter; ++it) {
      A.grad(vs, streams, (uint32_t)it, g, ok);
      for (int k = 0; k < K; ++k) sga_step(cand[k], g[k], hist[k], it, etas[k]);
    }
    std::vector<double> elbos, e0;
    A.elbo(vs, streams, 0u, elbos);
    Meanfield init_copy = init;
    A.elbo({&init_copy}, {STREAM_ELBO_INIT}, 0u, e0);
    const double elbo_init = e0[0];
    // advi.hpp adapt_eta: sequential decision over the candidates' ELBOs
    double elbo_best = -INFINITY, eta_best = 0.0;
    bool found = false;
    for (int k = 0; k < K; ++k) {
      const double el = isfinite(elbos[k]) ? elbos[k] : -INFINITY;
      if (el < elbo_best && elbo_best > elbo_init) {
        found = true;
        break;
      }
      if (k < K - 1) {
        elbo_best = el;
        eta_best = etas[k];
      } else if (el > elbo_init) {
        eta_best = etas[k];
        found = true;
      }
    }
    if (!found)
      return fail(FITOCT_E_NUMERIC, "vb: all proposed step-sizes failed (ELBO diverged)");
    eta = eta_best;
  }

  // stochastic gradient ascent (advi.hpp stochastic_gradient_ascent)
  Meanfield v = init, hist{Vec(D, 0.0), Vec(D, 0.0)};
  std::vector<Meanfield> g;
  std::vector<int> ok;
  std::vector<double> el;
  const int cb_size = (int)std::max(0.1 * c->iter / c->eval_elbo, 2.0);
  std::vector<double> cb;  // circular buffer of relative ELBO changes
  double elbo = 0.0, elbo_prev;
  int it = 1, converged = 0;
  for (;; ++it) {
    A.grad({&v}, {STREAM_SGA}, (uint32_t)it, g, ok);
    sga_step(v, g[0], hist, it, eta);
    if (it % c->eval_elbo == 0) {
      elbo_prev = elbo;
      A.elbo({&v}, {STREAM_SGA}, (uint32_t)it, el);
      elbo = el[0];
      if (!isfinite(elbo)) return fail(FITOCT_E_NUMERIC, "vb: every ELBO draw was dropped");
      const double rel = fabs((elbo_prev - elbo) / elbo);
      if ((int)cb.size() == cb_size) cb.erase(cb.begin());
      cb.push_back(rel);
      const double mean = std::accumulate(cb.begin(), cb.end(), 0.0) / cb.size();
      std::vector<double> tmp(cb);
      std::nth_element(tmp.begin(), tmp.begin() + tmp.size() / 2, tmp.end());
      const double med = tmp[tmp.size() / 2];
      if (mean < c->tol_rel_obj || med < c->tol_rel_obj) {
        converged = 1;
        break;
      }
    }
    if (it >= c->iter) break;
  }
  memcpy(res->mu, v.mu.data(), sizeof(double) * D);
  memcpy(res->omega, v.omega.data(), sizeof(double) * D);
  res->eta = eta;
  res->elbo = elbo;
  res->iterations = it;
  res->converged = converged;
  // draws from the approximation (rstan::vb output_samples)
  const int S = c->output_samples;
  Vec q((size_t)cap * D), lp(cap), s2(cap), e(D);
  for (int s0 = 0; s0 < S; s0 += cap) {
    const int n = std::min(cap, S - s0);
    std::vector<double> lg(n);
    for (int s = 0; s < n; ++s) {
      normals(c->seed, STREAM_OUT, ADVI_OUT, 0u, (uint32_t)(s0 + s), D, e.data());
      double ss = 0.0;
      for (int d = 0; d < D; ++d) {
        q[(size_t)s * D + d] = v.mu[d] + exp(v.omega[d]) * e[d];
        ss += e[d] * e[d];
      }
      lg[s] = -0.5 * ss;
    }
    E.run(n, q.data(), 1, 1, lp.data(), nullptr, s2.data());
    for (int s = 0; s < n; ++s) {
      if (res->draws) memcpy(res->draws + (size_t)(s0 + s) * D, &q[(size_t)s * D], sizeof(double) * D);
      if (res->log_p) res->log_p[s0 + s] = lp[s];
      if (res->log_g) res->log_g[s0 + s] = lg[s];
      if (res->sumr2) res->sumr2[s0 + s] = s2[s];
    }
  }
  res->n_evals = (int)E.points;
  return FITOCT_OK;
}

}  // namespace
}  // namespace fitoct

using namespace fitoct;

extern "C" {

void fitoct_default_optim_config(fitoct_optim_config* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  c->iter = 2000;
  c->history = 5;
  c->init_alpha = 1e-3;
  c->tol_obj = 1e-12;
  c->tol_rel_obj = 1e4;
  c->tol_grad = 1e-8;
  c->tol_rel_grad = 1e7;
  c->tol_param = 1e-8;
  c->hessian = 1;
  c->jacobian = 0;
  c->hessian_step = 1e-3;
  c->precision = FITOCT_PREC_F64;
}

int32_t fitoct_optimize(const fitoct_problem* prob, const fitoct_optim_config* cfg,
                        const double* init_q, fitoct_optim_result* res) {
  if (!prob || !cfg || !res || !res->par) return fail(FITOCT_E_ARG, "NULL argument");
  if (cfg->iter < 1 || cfg->history < 1 || !(cfg->init_alpha > 0.0) ||
      (cfg->hessian && !(cfg->hessian_step > 0.0)))
    return fail(FITOCT_E_ARG, "bad optim config");
  try {
    return run_optimize(prob, cfg, init_q, res);
  } catch (const DeviceError& e) {
    return e.code;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "exception in fitoct_optimize");
  }
}

void fitoct_default_vb_config(fitoct_vb_config* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  c->iter = 10000;
  c->grad_samples = 1;
  c->elbo_samples = 100;
  c->eval_elbo = 100;
  c->eta = 1.0;
  c->adapt_engaged = 1;
  c->adapt_iter = 50;
  c->tol_rel_obj = 0.01;
  c->output_samples = 1000;
  c->seed = 1234;
  c->precision = FITOCT_PREC_F64;
}

int32_t fitoct_vb(const fitoct_problem* prob, const fitoct_vb_config* cfg, const double* init_q,
                  fitoct_vb_result* res) {
  if (!prob || !cfg || !res || !res->mu || !res->omega) return fail(FITOCT_E_ARG, "NULL argument");
  try {
    return run_vb(prob, cfg, init_q, res);
  } catch (const DeviceError& e) {
    return e.code;
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, "exception in fitoct_vb");
  }
}

}  // extern "C"
