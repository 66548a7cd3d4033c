/*
 * ORACLE (test infrastructure only) -- CPU restatement of the FitOCT ExpGP
 * posterior and of Stan's NUTS with warm-up adaptation.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library (oracle/build/liboracle.so).  The product path never does.
 *
 * Parity status: **parity unpinned** against rstan/FitOCTLib -- neither R, rstan,
 * Stan nor FitOCTLib exists in this container.  This file is an
 * independent restatement, written from:
 *   - the model contract of SURVEY.md Appendix A (same anchors as
 *     oracle/model_np.py: ui.R:88, synthData.R:22, server.R:623-650,
 *     Tests/horseShoePrior.stan:16-43, Tests/lassoPrior.stan:9-12,
 *     Tests/testGamma.R:19-28, FitOCT.R:116-117, priPost.R:14);
 *   - Stan's sampler as described in SURVEY.md Appendix B [ext]:
 *     stan/mcmc/hmc/nuts/base_nuts.hpp (transition, build_tree,
 *     compute_criterion), hmc/base_hmc.hpp (init_stepsize),
 *     hmc/integrators/expl_leapfrog.hpp, stepsize_adaptation.hpp (dual
 *     averaging), windowed_adaptation.hpp + var_adaptation.hpp (diagonal
 *     metric), adapt_diag_e_nuts.hpp (the adaptation order).
 * build_tree is written RECURSIVELY here, as in Stan; the HIP library replays
 * it iteratively.  Random numbers: Philox4x32-10 (Random123 known-answer
 * vectors checked in tests) addressed by (seed, chain, purpose, indices) --
 * the same addressing the HIP sampler uses, so both produce the same draws
 * while no floating-point near-tie flips a decision.
 * It is pinned by: prior-only known answers (testGamma.R's exponential mean =
 * sd = 10, the horseshoe's half-Cauchy quantiles, the lasso density, the theta
 * prior), finite differences, and the numpy restatement (golden vectors).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/fitoct.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al. 2011)                                          */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t v[4]; } ctr4;

static ctr4 philox10(ctr4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
    ctr4 n;
    n.v[0] = (uint32_t)(p1 >> 32) ^ c.v[1] ^ k0;
    n.v[1] = (uint32_t)p1;
    n.v[2] = (uint32_t)(p0 >> 32) ^ c.v[3] ^ k1;
    n.v[3] = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  ctr4 c = {{ctr[0], ctr[1], ctr[2], ctr[3]}};
  ctr4 r = philox10(c, key[0], key[1]);
  memcpy(out, r.v, sizeof r.v);
}

enum { T_INIT = 1, T_SSMOM = 2, T_MOM = 3, T_DIR = 4, T_TOP = 5, T_MERGE = 6 };

typedef struct { uint32_t k0, k1; } rkey;

static rkey chain_key(uint64_t seed, uint32_t gid) {
  rkey k;
  k.k0 = (uint32_t)seed;
  k.k1 = (uint32_t)(seed >> 32) ^ (gid * 0x9E3779B9u + 0x7F4A7C15u);
  return k;
}
static double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
static double unif(rkey k, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  ctr4 c = {{c0, c1, c2, c3}};
  ctr4 r = philox10(c, k.k0, k.k1);
  return u53(r.v[0], r.v[1]);
}
/* Box-Muller pair: angle 2*pi*u2 */
static void normal2(rkey k, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, double* n0,
                    double* n1) {
  ctr4 c = {{c0, c1, c2, c3}};
  ctr4 r = philox10(c, k.k0, k.k1);
  const double a = u53(r.v[0], r.v[1]), b = u53(r.v[2], r.v[3]);
  const double rad = sqrt(-2.0 * log(1.0 - a));
  const double ang = 6.283185307179586 * b;
  *n0 = rad * cos(ang);
  *n1 = rad * sin(ang);
}

/* ------------------------------------------------------------------------ */
/* model                                                                       */
/* ------------------------------------------------------------------------ */
typedef struct {
  int N, Nn, D, fam, prior_PD;
  double c;             /* dataType */
  const double *x, *y, *uy;
  double* B;            /* [N][Nn] */
  double th0[3], Si[9]; /* Sigma0^-1 */
  double rate, ls, nu, ss;
  double trate; /* mono-exp, theta_prior = 1: theta_k ~ exponential(trate) (testGamma.R) */
} model;

static int dimof(int fam, int Nn) {
  /* fam 3: mono-exponential model (FitOCTLib::fitMonoExp; include/fitoct.h) */
  return fam == 0 ? Nn + 5 : fam == 1 ? Nn + 4 : fam == 2 ? 3 * Nn + 6 : 3;
}

static double kern(double d, double rho, int conv) {
  return conv == 0 ? exp(-(d * d) / (2.0 * rho * rho)) : exp(-(d / rho) * (d / rho));
}

/* B = K(x~, xGP) K(xGP,xGP)^-1 via Cholesky (server.R:623-650) */
static int basis(const fitoct_problem* p, double* B) {
  const int N = p->N, Nn = p->Nn;
  double xmin = p->x[0], xmax = p->x[0];
  for (int i = 1; i < N; ++i) {
    if (p->x[i] < xmin) xmin = p->x[i];
    if (p->x[i] > xmax) xmax = p->x[i];
  }
  const double rho = p->rho > 0 ? p->rho : 1.0 / Nn;
  double* xg = (double*)malloc(sizeof(double) * Nn);
  double* L = (double*)calloc((size_t)Nn * Nn, sizeof(double));
  double* z = (double*)malloc(sizeof(double) * Nn);
  for (int k = 0; k < Nn; ++k) {
    if (p->grid_type == 0) {
      const double dx = 1.0 / (Nn + 1);
      xg[k] = dx / 2 + (1.0 - dx) * k / (Nn - 1);
    } else {
      xg[k] = (double)k / (Nn - 1);
    }
  }
  int rc = 0;
  for (int i = 0; i < Nn && !rc; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = kern(xg[i] - xg[j], rho, p->kernel_conv) + (i == j ? p->nugget : 0.0);
      for (int k = 0; k < j; ++k) s -= L[i * Nn + k] * L[j * Nn + k];
      if (i == j) {
        if (!(s > 0)) { rc = -1; break; }
        L[i * Nn + i] = sqrt(s);
      } else {
        L[i * Nn + j] = s / L[j * Nn + j];
      }
    }
  for (int i = 0; i < N && !rc; ++i) {
    const double xt = (p->x[i] - xmin) / (xmax - xmin);
    for (int a = 0; a < Nn; ++a) {
      double s = kern(xt - xg[a], rho, p->kernel_conv);
      for (int k = 0; k < a; ++k) s -= L[a * Nn + k] * z[k];
      z[a] = s / L[a * Nn + a];
    }
    for (int a = Nn - 1; a >= 0; --a) {
      double s = z[a];
      for (int k = a + 1; k < Nn; ++k) s -= L[k * Nn + a] * B[(size_t)i * Nn + k];
      B[(size_t)i * Nn + a] = s / L[a * Nn + a];
    }
  }
  free(xg);
  free(L);
  free(z);
  return rc;
}

static int model_init(model* m, const fitoct_problem* p) {
  memset(m, 0, sizeof *m);
  m->N = p->N;
  m->fam = p->prior_type;
  m->Nn = m->fam == 3 ? 0 : p->Nn;
  m->D = dimof(p->prior_type, p->Nn);
  m->prior_PD = p->prior_PD;
  m->c = p->data_type;
  m->x = p->x;
  m->y = p->y;
  m->uy = p->uy;
  m->B = (double*)malloc(sizeof(double) * (size_t)p->N * (m->Nn > 0 ? m->Nn : 1));
  if (m->fam == 3) {
    /* no GP term */
  } else if (p->B) {
    memcpy(m->B, p->B, sizeof(double) * (size_t)p->N * p->Nn);
  } else if (basis(p, m->B)) {
    return -1;
  }
  memcpy(m->th0, p->theta0, sizeof m->th0);
  if (m->fam == 3) { /* flat prior on theta (or testGamma.R's exponential), sigma fixed at 1 */
    memset(m->Si, 0, sizeof m->Si);
    m->ss = 1.0;
    m->trate = p->theta_prior == 1 ? 1.0 / p->lambda_scale : 0.0;
    return 0;
  }
  const double* S = p->Sigma0;
  const double A = S[4] * S[8] - S[5] * S[7], Bc = -(S[3] * S[8] - S[5] * S[6]),
               Cc = S[3] * S[7] - S[4] * S[6];
  const double det = S[0] * A + S[1] * Bc + S[2] * Cc;
  m->Si[0] = A / det;
  m->Si[1] = -(S[1] * S[8] - S[2] * S[7]) / det;
  m->Si[2] = (S[1] * S[5] - S[2] * S[4]) / det;
  m->Si[3] = Bc / det;
  m->Si[4] = (S[0] * S[8] - S[2] * S[6]) / det;
  m->Si[5] = -(S[0] * S[5] - S[2] * S[3]) / det;
  m->Si[6] = Cc / det;
  m->Si[7] = -(S[0] * S[7] - S[1] * S[6]) / det;
  m->Si[8] = (S[0] * S[4] - S[1] * S[3]) / det;
  m->rate = p->lambda_conv == 0 ? 1.0 / p->lambda_rate : p->lambda_rate;
  m->ls = p->lambda_scale;
  m->nu = p->nu;
  m->ss = p->sigma_scale;
  return 0;
}

/* log density (Stan log_prob<propto, jacobian>) and gradient; work: [Nn] */
static double logp_grad(const model* m, const double* q, double* g, double* sumr2, double* work) {
  const int Nn = m->Nn, D = m->D, N = m->N, fam = m->fam;
  double* ygp = work;           /* [Nn] */
  double* gy = work + Nn;       /* [Nn] */
  double* lam = work + 2 * Nn;  /* [Nn] horseshoe local scales */
  const double th[3] = {exp(q[0]), exp(q[1]), exp(q[2])};
  const int mono = fam == 3;
  const double usig = mono ? 0.0 : q[D - 1], sig = mono ? 1.0 : exp(usig);
  double tau = 0.0, lam_s = 0.0;
  /* horseshoe (Tests/horseShoePrior.stan:30-32): lam[k] holds lambda_k * tau =
   * r1_l sqrt(r2_l) r1_g sqrt(r2_g), evaluated in the exponent as
   * exp(u1_l + u2_l/2 + u1_g + u2_g/2) -- the same expression as the HIP sampler */
  for (int k = 0; k < Nn; ++k) {
    if (fam == 2) {
      lam[k] = exp(fma(0.5, q[5 + 2 * Nn + k], q[5 + Nn + k]) + fma(0.5, q[4 + Nn], q[3 + Nn]));
    }
    gy[k] = 0.0;
  }
  if (fam == 2) tau = 1.0; /* folded into lam[] */
  for (int k = 0; k < Nn; ++k) ygp[k] = fam == 2 ? q[3 + k] * lam[k] : q[3 + k];
  if (fam == 0) lam_s = exp(q[3 + Nn]);
  double lp = 0.0, gth[3] = {0, 0, 0}, gsig = 0.0;
  int bad = 0;
  double s2 = NAN;
  if (m->prior_PD == 0) {
    double Sd2 = 0, Sa = 0, Sae = 0, Sw = 0;
    for (int i = 0; i < N; ++i) {
      const double* Bi = m->B + (size_t)i * Nn;
      double dL = 0.0;
      for (int k = 0; k < Nn; ++k) dL += Bi[k] * ygp[k];
      const double u = 1.0 + dL;
      if (!(u > 0.0)) { bad = 1; break; }
      const double L = th[2] * u, cx = m->c * m->x[i];
      const double e = exp(-cx / L);
      const double mu = th[0] + th[1] * e;
      const double isu = 1.0 / m->uy[i];
      const double d = (m->y[i] - mu) * isu;
      const double a = d * isu, ae = a * e, w = ae * cx / L, h = w / L;
      Sd2 += d * d;
      Sa += a;
      Sae += ae;
      Sw += w;
      for (int k = 0; k < Nn; ++k) gy[k] += Bi[k] * h;
    }
    if (bad) {
      if (sumr2) *sumr2 = INFINITY;
      return -INFINITY;
    }
    s2 = Sd2;
    const double is2 = 1.0 / (sig * sig);
    lp += -0.5 * Sd2 * is2 - N * usig;
    gth[0] = Sa * is2;
    gth[1] = Sae * is2;
    gth[2] = th[1] * Sw * is2 / th[2];
    gsig = (Sd2 * is2 - N) / sig;
    for (int k = 0; k < Nn; ++k) gy[k] *= th[1] * th[2] * is2;
  }
  if (sumr2) *sumr2 = s2;
  /* theta ~ multi_normal(theta0, Sigma0) + log-Jacobian */
  const double dt[3] = {th[0] - m->th0[0], th[1] - m->th0[1], th[2] - m->th0[2]};
  for (int j = 0; j < 3; ++j) {
    const double sd = m->Si[3 * j] * dt[0] + m->Si[3 * j + 1] * dt[1] + m->Si[3 * j + 2] * dt[2];
    lp += -0.5 * dt[j] * sd + q[j];
    g[j] = th[j] * (gth[j] - sd) + 1.0;
  }
  if (mono) {
    /* theta_prior = 1 (Tests/testGamma.R:19-28): theta_k ~ exponential(trate) */
    for (int j = 0; j < 3; ++j) {
      lp += -m->trate * th[j];
      g[j] -= m->trate * th[j];
    }
    if (!isfinite(lp)) lp = -INFINITY;
    return lp;
  }
  /* sigma ~ half-normal(0, sigma_scale) */
  lp += -0.5 * (sig / m->ss) * (sig / m->ss) + usig;
  g[D - 1] = sig * (gsig - sig / (m->ss * m->ss)) + 1.0;
  if (fam == 0) {
    double S2 = 0;
    for (int k = 0; k < Nn; ++k) {
      S2 += ygp[k] * ygp[k];
      g[3 + k] = gy[k] - ygp[k] / (lam_s * lam_s);
    }
    lp += -Nn * log(lam_s) - S2 / (2 * lam_s * lam_s) - m->rate * lam_s + q[3 + Nn];
    g[3 + Nn] = lam_s * (-Nn / lam_s + S2 / (lam_s * lam_s * lam_s) - m->rate) + 1.0;
  } else if (fam == 1) {
    for (int k = 0; k < Nn; ++k) {
      const double yv = ygp[k];
      lp += -m->ls * fabs(yv) - m->ls * yv * yv;
      g[3 + k] = gy[k] - m->ls * (yv > 0 ? 1.0 : yv < 0 ? -1.0 : 0.0) - 2.0 * m->ls * yv;
    }
  } else {
    double SGy = 0;
    const double r1g = exp(q[3 + Nn]), r2g = exp(q[4 + Nn]);
    for (int k = 0; k < Nn; ++k) {
      const double z = q[3 + k];
      const double r1 = exp(q[5 + Nn + k]), r2 = exp(q[5 + 2 * Nn + k]);
      const double Gy = gy[k] * ygp[k];
      SGy += Gy;
      lp += -0.5 * z * z - 0.5 * r1 * r1 + q[5 + Nn + k];
      lp += -(0.5 * m->nu + 1.0) * q[5 + 2 * Nn + k] - 0.5 * m->nu / r2 + q[5 + 2 * Nn + k];
      g[3 + k] = gy[k] * lam[k] * tau - z;
      g[5 + Nn + k] = Gy - r1 * r1 + 1.0;
      g[5 + 2 * Nn + k] = 0.5 * Gy - (0.5 * m->nu + 1.0) + 0.5 * m->nu / r2 + 1.0;
    }
    lp += -0.5 * r1g * r1g + q[3 + Nn] - 1.5 * q[4 + Nn] - 0.5 / r2g + q[4 + Nn];
    g[3 + Nn] = SGy - r1g * r1g + 1.0;
    g[4 + Nn] = 0.5 * SGy - 1.5 + 0.5 / r2g + 1.0;
  }
  if (!isfinite(lp)) lp = -INFINITY;
  return lp;
}

/* ------------------------------------------------------------------------ */
/* NUTS (Stan base_nuts, diagonal metric)                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
  double *q, *p, *g;
  double lp, s2;
} ps_point;

typedef struct {
  const model* m;
  int D;
  double* minv;
  double* work;
  rkey key;
  uint32_t t;        /* iteration */
  int top_depth;     /* depth of the subtree being built at the top level */
  int leaf;          /* leaf counter inside the current top-level subtree */
  double H0, eps;
  int n_leapfrog, divergent;
  double sum_metro;
  ps_point z;        /* the point being integrated */
} nuts_ctx;

static void pt_alloc(ps_point* a, int D) {
  a->q = (double*)calloc(D, sizeof(double));
  a->p = (double*)calloc(D, sizeof(double));
  a->g = (double*)calloc(D, sizeof(double));
}
static void pt_free(ps_point* a) {
  free(a->q);
  free(a->p);
  free(a->g);
}
static void pt_copy(ps_point* dst, const ps_point* src, int D) {
  memcpy(dst->q, src->q, sizeof(double) * D);
  memcpy(dst->p, src->p, sizeof(double) * D);
  memcpy(dst->g, src->g, sizeof(double) * D);
  dst->lp = src->lp;
  dst->s2 = src->s2;
}
static double kinetic(const double* p, const double* minv, int D) {
  double s = 0;
  for (int k = 0; k < D; ++k) s += p[k] * minv[k] * p[k];
  return 0.5 * s;
}
static double hamiltonian(const ps_point* z, const double* minv, int D) {
  return -z->lp + kinetic(z->p, minv, D);
}
/* expl_leapfrog::evolve */
static void leapfrog(nuts_ctx* c, ps_point* z, double e) {
  const int D = c->D;
  for (int k = 0; k < D; ++k) z->p[k] += 0.5 * e * z->g[k];
  for (int k = 0; k < D; ++k) z->q[k] += e * c->minv[k] * z->p[k];
  z->lp = logp_grad(c->m, z->q, z->g, &z->s2, c->work);
  for (int k = 0; k < D; ++k) z->p[k] += 0.5 * e * z->g[k];
}
/* Multinomial weights exp(H0 - H) as extended-exponent floats m * 2^e
 * (m in [1/2, 1) or 0).  Stan keeps log weights and merges them with
 * log_sum_exp; the linear form is the same arithmetic up to rounding, cannot
 * overflow, and is what the HIP sampler uses (nuts_device.hip, struct XF), so
 * both take the same merge decisions. */
typedef struct {
  double m;
  int e;
} xf;
static xf xf_norm(double m, int e) {
  int k;
  const double f = frexp(m, &k);
  xf r = {f, f == 0.0 ? 0 : e + k};
  return r;
}
static xf xf_exp(double x) {
  if (x > -700.0 && x < 700.0) return xf_norm(exp(x), 0);
  /* above 1e8 (an energy drop no trajectory of a finite start reaches) the weight
   * saturates: the exponent stays within int and exponent differences of two weights
   * (xf_u_below) stay within int too (>= -1.45e9 - 1.45e8) */
  if (!(x < 1.0e8)) x = 1.0e8;
  /* below -1e9 (a divergent leaf, never merged) the exponent would overflow an int
   * (UBSan, scripts/cpu_sanitized_suite.sh); the weight is 0 to every resolvable digit */
  if (!(x > -1.0e9)) {
    xf z = {0.0, 0};
    return z;
  }
  const double k = floor(x * 1.4426950408889634);
  return xf_norm(exp(fma(-k, 0.6931471805599453, x)), (int)k);
}
static xf xf_add(xf a, xf b) {
  if (a.m == 0.0) return b;
  if (b.m == 0.0) return a;
  const int e = a.e > b.e ? a.e : b.e;
  return xf_norm(ldexp(a.m, a.e - e) + ldexp(b.m, b.e - e), e);
}
static int xf_gt(xf a, xf b) {
  if (a.m == 0.0) return 0;
  if (b.m == 0.0) return 1;
  return a.e != b.e ? a.e > b.e : a.m > b.m;
}
static int xf_u_below(double u, xf a, xf b) { /* u < a / b */
  if (b.m == 0.0) return 0;
  return ldexp(u * b.m, b.e - a.e) < a.m;
}
static double xf_val(xf a) { return ldexp(a.m, a.e); }

/* compute_criterion on p_sharp = minv .* p */
static int criterion(const double* pm, const double* pp, const double* rho, const double* minv,
                     int D) {
  double a = 0, b = 0;
  for (int k = 0; k < D; ++k) {
    a += minv[k] * pp[k] * rho[k];
    b += minv[k] * pm[k] * rho[k];
  }
  return a > 0 && b > 0;
}

/* base_nuts::build_tree.  Vectors: p_beg/p_end (momenta at the subtree ends),
 * rho (momentum sum, accumulated into), z_propose (out).  Returns validity. */
static int build_tree(nuts_ctx* c, int depth, ps_point* z_propose, double* p_beg, double* p_end,
                      double* rho, double sign, xf* sum_weight) {
  const int D = c->D;
  if (depth == 0) {
    leapfrog(c, &c->z, sign * c->eps);
    ++c->n_leapfrog;
    double h = hamiltonian(&c->z, c->minv, D);
    if (isnan(h)) h = INFINITY;
    if (h - c->H0 > 1000.0) c->divergent = 1;
    const xf wleaf = xf_exp(c->H0 - h);
    *sum_weight = xf_add(*sum_weight, wleaf);
    if (c->H0 - h > 0) c->sum_metro += 1.0;
    else c->sum_metro += xf_val(wleaf);
    pt_copy(z_propose, &c->z, D);
    for (int k = 0; k < D; ++k) {
      rho[k] += c->z.p[k];
      p_beg[k] = c->z.p[k];
      p_end[k] = c->z.p[k];
    }
    ++c->leaf;
    return !c->divergent;
  }
  /* initial subtree */
  xf w_init = {0.0, 0};
  double* p_init_end = (double*)calloc(D, sizeof(double));
  double* rho_init = (double*)calloc(D, sizeof(double));
  double* p_final_beg = (double*)calloc(D, sizeof(double));
  double* rho_final = (double*)calloc(D, sizeof(double));
  double* tmp = (double*)calloc(D, sizeof(double));
  ps_point z_final;
  pt_alloc(&z_final, D);
  int ok = build_tree(c, depth - 1, z_propose, p_beg, p_init_end, rho_init, sign, &w_init);
  if (ok) {
    xf w_final = {0.0, 0};
    ok = build_tree(c, depth - 1, &z_final, p_final_beg, p_end, rho_final, sign, &w_final);
    if (ok) {
      const xf w_sub = xf_add(w_init, w_final);
      *sum_weight = xf_add(*sum_weight, w_sub);
      if (xf_gt(w_final, w_sub)) {
        pt_copy(z_propose, &z_final, D);
      } else {
        /* the merge completes at the subtree's last leaf: (level, top depth, leaf) */
        const double u = unif(c->key, c->t,
                              T_MERGE | ((uint32_t)(depth - 1) << 8) | ((uint32_t)c->top_depth << 16),
                              (uint32_t)(c->leaf - 1), 0u);
        if (xf_u_below(u, w_final, w_sub)) pt_copy(z_propose, &z_final, D);
      }
      for (int k = 0; k < D; ++k) {
        const double rs = rho_init[k] + rho_final[k];
        rho[k] += rs;
        tmp[k] = rs;
      }
      ok = criterion(p_beg, p_end, tmp, c->minv, D);
      for (int k = 0; k < D; ++k) tmp[k] = rho_init[k] + p_final_beg[k];
      ok = ok && criterion(p_beg, p_final_beg, tmp, c->minv, D);
      for (int k = 0; k < D; ++k) tmp[k] = rho_final[k] + p_init_end[k];
      ok = ok && criterion(p_init_end, p_end, tmp, c->minv, D);
    }
  }
  free(p_init_end);
  free(rho_init);
  free(p_final_beg);
  free(rho_final);
  free(tmp);
  pt_free(&z_final);
  return ok;
}

typedef struct {
  double accept, energy;
  int depth, n_leapfrog, divergent;
} trans_info;

/* base_nuts::transition from z_sample (q, g, lp set); p is sampled here */
static void transition(nuts_ctx* c, ps_point* z_sample, int max_depth, trans_info* info) {
  const int D = c->D;
  for (int k = 0; k < D; ++k) {
    double n0, n1;
    normal2(c->key, c->t, T_MOM, (uint32_t)(k >> 1), 0u, &n0, &n1);
    z_sample->p[k] = ((k & 1) ? n1 : n0) / sqrt(c->minv[k]);
  }
  ps_point z_fwd, z_bck, z_propose;
  pt_alloc(&z_fwd, D);
  pt_alloc(&z_bck, D);
  pt_alloc(&z_propose, D);
  pt_copy(&z_fwd, z_sample, D);
  pt_copy(&z_bck, z_sample, D);
  double* p_fwd_fwd = (double*)malloc(sizeof(double) * D);
  double* p_fwd_bck = (double*)malloc(sizeof(double) * D);
  double* p_bck_fwd = (double*)malloc(sizeof(double) * D);
  double* p_bck_bck = (double*)malloc(sizeof(double) * D);
  double* rho = (double*)malloc(sizeof(double) * D);
  double* rho_fwd = (double*)malloc(sizeof(double) * D);
  double* rho_bck = (double*)malloc(sizeof(double) * D);
  double* tmp = (double*)malloc(sizeof(double) * D);
  for (int k = 0; k < D; ++k) {
    p_fwd_fwd[k] = p_fwd_bck[k] = p_bck_fwd[k] = p_bck_bck[k] = rho[k] = z_sample->p[k];
  }
  xf sum_weight = {0.5, 1}; /* exp(0): the initial point */
  c->H0 = hamiltonian(z_sample, c->minv, D);
  c->n_leapfrog = 0;
  c->sum_metro = 0.0;
  c->divergent = 0;
  int depth = 0;
  while (depth < max_depth) {
    for (int k = 0; k < D; ++k) rho_fwd[k] = rho_bck[k] = 0.0;
    xf w_sub = {0.0, 0};
    int valid;
    c->top_depth = depth;
    c->leaf = 0;
    if (unif(c->key, c->t, T_DIR, (uint32_t)depth, 0u) > 0.5) {
      pt_copy(&c->z, &z_fwd, D);
      memcpy(rho_bck, rho, sizeof(double) * D);
      memcpy(p_bck_fwd, p_fwd_fwd, sizeof(double) * D);
      valid = build_tree(c, depth, &z_propose, p_fwd_bck, p_fwd_fwd, rho_fwd, 1.0, &w_sub);
      pt_copy(&z_fwd, &c->z, D);
    } else {
      pt_copy(&c->z, &z_bck, D);
      memcpy(rho_fwd, rho, sizeof(double) * D);
      memcpy(p_fwd_bck, p_bck_bck, sizeof(double) * D);
      valid = build_tree(c, depth, &z_propose, p_bck_fwd, p_bck_bck, rho_bck, -1.0, &w_sub);
      pt_copy(&z_bck, &c->z, D);
    }
    if (!valid) break;
    ++depth;
    if (xf_gt(w_sub, sum_weight)) {
      pt_copy(z_sample, &z_propose, D);
    } else {
      const double u = unif(c->key, c->t, T_TOP, (uint32_t)(depth - 1), 0u);
      if (xf_u_below(u, w_sub, sum_weight)) pt_copy(z_sample, &z_propose, D);
    }
    sum_weight = xf_add(sum_weight, w_sub);
    for (int k = 0; k < D; ++k) rho[k] = rho_bck[k] + rho_fwd[k];
    int persist = criterion(p_bck_bck, p_fwd_fwd, rho, c->minv, D);
    for (int k = 0; k < D; ++k) tmp[k] = rho_bck[k] + p_fwd_bck[k];
    persist = persist && criterion(p_bck_bck, p_fwd_bck, tmp, c->minv, D);
    for (int k = 0; k < D; ++k) tmp[k] = rho_fwd[k] + p_bck_fwd[k];
    persist = persist && criterion(p_bck_fwd, p_fwd_fwd, tmp, c->minv, D);
    if (!persist) break;
  }
  info->depth = depth;
  info->n_leapfrog = c->n_leapfrog;
  info->divergent = c->divergent;
  info->accept = c->sum_metro / (double)c->n_leapfrog;
  info->energy = hamiltonian(z_sample, c->minv, D);
  pt_free(&z_fwd);
  pt_free(&z_bck);
  pt_free(&z_propose);
  free(p_fwd_fwd);
  free(p_fwd_bck);
  free(p_bck_fwd);
  free(p_bck_bck);
  free(rho);
  free(rho_fwd);
  free(rho_bck);
  free(tmp);
}

/* base_hmc::init_stepsize: z holds q, g, lp (p resampled per trial) */
static int init_stepsize(nuts_ctx* c, ps_point* z, uint32_t window, double* eps) {
  const int D = c->D;
  if (*eps == 0 || *eps > 1e7 || isnan(*eps)) return 0;
  ps_point w;
  pt_alloc(&w, D);
  int direction = 0, rc = 0;
  for (uint32_t trial = 0;; ++trial) {
    pt_copy(&w, z, D);
    for (int k = 0; k < D; ++k) {
      double n0, n1;
      normal2(c->key, window, T_SSMOM, (uint32_t)(k >> 1), trial, &n0, &n1);
      w.p[k] = ((k & 1) ? n1 : n0) / sqrt(c->minv[k]);
    }
    const double H0 = hamiltonian(&w, c->minv, D);
    leapfrog(c, &w, *eps);
    double h = hamiltonian(&w, c->minv, D);
    if (isnan(h)) h = INFINITY;
    const double dH = H0 - h;
    if (trial == 0) {
      direction = dH > log(0.8) ? 1 : -1;
      continue;
    }
    if (direction == 1 && !(dH > log(0.8))) break;
    if (direction == -1 && !(dH < log(0.8))) break;
    *eps = direction == 1 ? 2 * *eps : 0.5 * *eps;
    if (*eps > 1e7 || *eps == 0 || trial > 2000) {
      rc = FITOCT_E_NUMERIC;
      break;
    }
  }
  pt_free(&w);
  return rc;
}

/* warm restart (oracle_sample_init, the restatement of fitoct_plan_set_init): per-chain
 * initial position [chains][D], step size [chains] and inverse metric [chains][D];
 * NULL = the defaults below.  Caller-owned, read-only, passed per call (no global state:
 * concurrent oracle_sample calls from several host threads are independent). */
typedef struct {
  const double *q, *eps, *minv;
} warm_init;

/* one chain: init, adaptation (adapt_diag_e_nuts), sampling */
static int run_chain(const model* m, const fitoct_config* cfg, const warm_init* wi, int lc,
                     double* draws, int ncols, int iters_saved, double* out_eps, double* out_minv,
                     long long* out_lf) {
  const int D = m->D, Nn = m->Nn, W = cfg->warmup, S = cfg->samples;
  const uint32_t gid = (uint32_t)(cfg->chain_offset + lc);
  nuts_ctx c;
  memset(&c, 0, sizeof c);
  c.m = m;
  c.D = D;
  c.key = chain_key(cfg->seed, gid);
  c.minv = (double*)malloc(sizeof(double) * D);
  c.work = (double*)malloc(sizeof(double) * 3 * (Nn + 1));
  pt_alloc(&c.z, D);
  for (int k = 0; k < D; ++k) c.minv[k] = wi->minv ? wi->minv[(size_t)lc * D + k] : 1.0;
  ps_point z;
  pt_alloc(&z, D);
  /* initial point: jitter around theta0 (inits) */
  int attempt = 0, rc = 0;
  for (;; ++attempt) {
    for (int k = 0; k < D; ++k) {
      double base = 0, w = 0;
      if (k < 3) {
        base = log(m->th0[k]);
        w = 0.025;
      } else if (k < 3 + Nn) {
        w = 0.05;
      } else {
        w = 0.25;
        if (m->fam == 0 && k == 3 + Nn) base = -log(m->rate);
      }
      z.q[k] = base + cfg->init_radius * w * (2.0 * unif(c.key, (uint32_t)attempt, T_INIT, (uint32_t)k, 0u) - 1.0);
      if (wi->q) z.q[k] = wi->q[(size_t)lc * D + k];
    }
    z.lp = logp_grad(m, z.q, z.g, &z.s2, c.work);
    int finite = z.lp > -INFINITY;
    for (int k = 0; k < D; ++k) finite = finite && isfinite(z.g[k]);
    if (finite) break;
    if (attempt + 1 >= 100 || wi->q) { /* a given start is not retried */
      rc = FITOCT_E_INIT;
      break;
    }
  }
  double eps = wi->eps ? wi->eps[lc] : cfg->stepsize;
  /* dual averaging */
  double mu = log(10 * eps), s_bar = 0, x_bar = 0;
  int da_n = 0;
  /* windowed adaptation */
  int ib = cfg->init_buffer, tb = cfg->term_buffer, bw = cfg->window;
  const int win_on = W >= 20;
  if (win_on && ib + bw + tb > W) {
    ib = (int)(0.15 * W);
    tb = (int)(0.1 * W);
    bw = W - (ib + tb);
  }
  int win_counter = 0, win_size = bw, win_next = ib + bw - 1, wf_n = 0;
  double* wf_m = (double*)calloc(D, sizeof(double));
  double* wf_m2 = (double*)calloc(D, sizeof(double));
  uint32_t window = 0;
  long long lf = 0;
  if (!rc && cfg->adapt_engaged) rc = init_stepsize(&c, &z, window, &eps);
  for (int t = 0; t < W + S && !rc; ++t) {
    if (t == W && cfg->adapt_engaged && W > 0) eps = exp(x_bar); /* complete_adaptation */
    c.t = (uint32_t)t;
    c.eps = eps;
    trans_info info;
    transition(&c, &z, cfg->max_treedepth, &info);
    lf += info.n_leapfrog;
    if (t >= W || cfg->save_warmup) {
      const int it = cfg->save_warmup ? t : t - W;
      double* rec = draws + ((size_t)lc * iters_saved + it) * ncols;
      rec[0] = z.lp;
      rec[1] = info.accept;
      rec[2] = eps;
      rec[3] = info.depth;
      rec[4] = info.n_leapfrog;
      rec[5] = info.divergent;
      rec[6] = info.energy;
      for (int k = 0; k < D; ++k) rec[7 + k] = (k < 3 || k >= 3 + Nn) ? exp(z.q[k]) : z.q[k];
      rec[7 + D] = m->prior_PD ? NAN : z.s2 / m->N;
    }
    if (t < W && cfg->adapt_engaged) {
      /* stepsize_adaptation::learn_stepsize */
      ++da_n;
      const double as = info.accept > 1 ? 1 : info.accept;
      const double eta = 1.0 / (da_n + cfg->t0);
      s_bar = (1 - eta) * s_bar + eta * (cfg->adapt_delta - as);
      const double x = mu - s_bar * sqrt((double)da_n) / cfg->gamma;
      const double xe = pow((double)da_n, -cfg->kappa);
      x_bar = (1 - xe) * x_bar + xe * x;
      eps = exp(x);
      /* var_adaptation::learn_variance */
      int update = 0;
      if (win_on && win_counter >= ib && win_counter < W - tb && win_counter != W) {
        ++wf_n;
        for (int k = 0; k < D; ++k) {
          const double delta = z.q[k] - wf_m[k];
          wf_m[k] += delta / wf_n;
          wf_m2[k] += (z.q[k] - wf_m[k]) * delta;
        }
      }
      if (win_on && win_counter == win_next && win_counter != W) {
        const int last = W - tb - 1;
        if (win_next != last) {
          win_size *= 2;
          win_next = win_counter + win_size;
          if (win_next != last && win_next + 2 * win_size >= W - tb) win_next = last;
        }
        const double n = wf_n;
        for (int k = 0; k < D; ++k) {
          double v = c.minv[k];
          if (wf_n > 1) v = wf_m2[k] / (n - 1);
          c.minv[k] = (n / (n + 5.0)) * v + 1e-3 * (5.0 / (n + 5.0));
          wf_m[k] = wf_m2[k] = 0;
        }
        wf_n = 0;
        update = 1;
      }
      ++win_counter;
      if (update) {
        ++window;
        rc = init_stepsize(&c, &z, window, &eps);
        mu = log(10 * eps);
        s_bar = x_bar = 0;
        da_n = 0;
      }
    }
  }
  if (out_eps) out_eps[lc] = eps;
  if (out_minv) memcpy(out_minv + (size_t)lc * D, c.minv, sizeof(double) * D);
  if (out_lf) out_lf[lc] = lf;
  free(wf_m);
  free(wf_m2);
  free(c.minv);
  free(c.work);
  pt_free(&c.z);
  pt_free(&z);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* C ABI of the oracle                                                         */
/* ------------------------------------------------------------------------ */
int oracle_basis(const fitoct_problem* p, double* B) { return basis(p, B); }

int oracle_logp_grad(const fitoct_problem* p, int n_points, const double* q, double* lp,
                     double* grad, double* sumr2) {
  model m;
  if (model_init(&m, p)) return -1;
  double* work = (double*)malloc(sizeof(double) * 3 * (p->Nn + 1));
  for (int i = 0; i < n_points; ++i)
    lp[i] = logp_grad(&m, q + (size_t)i * m.D, grad + (size_t)i * m.D, sumr2 ? sumr2 + i : NULL,
                      work);
  free(work);
  free(m.B);
  return 0;
}

/* standard normals of the ADVI addressing contract (optimize.cpp normals()):
 * key (seed, stream), counter (it, tag, s, d/2), Box-Muller pairs over d */
void oracle_normals(uint64_t seed, uint32_t stream, uint32_t tag, uint32_t it, uint32_t s, int D,
                    double* eta) {
  const rkey k = chain_key(seed, stream);
  for (int d = 0; d < D; d += 2) {
    double n0, n1;
    normal2(k, it, tag, s, (uint32_t)(d >> 1), &n0, &n1);
    eta[d] = n0;
    if (d + 1 < D) eta[d + 1] = n1;
  }
}

/* draws: [chains][iters_saved][D + 8] (same columns as libfitoct); q_init / init_eps /
 * init_minv: the warm restart above (each may be NULL) */
int oracle_sample_init(const fitoct_problem* p, const fitoct_config* cfg, double* draws,
                       double* stepsize, double* inv_metric, long long* leapfrogs, int nthreads,
                       const double* q_init, const double* init_eps, const double* init_minv) {
  const warm_init wi = {q_init, init_eps, init_minv};
  model m;
  if (model_init(&m, p)) return -1;
  const int ncols = m.D + 8;
  const int iters_saved = cfg->save_warmup ? cfg->warmup + cfg->samples : cfg->samples;
  int rc_all = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(min : rc_all)
#endif
  for (int lc = 0; lc < cfg->chains; ++lc) {
    const int rc =
        run_chain(&m, cfg, &wi, lc, draws, ncols, iters_saved, stepsize, inv_metric, leapfrogs);
    if (rc < rc_all) rc_all = rc;
  }
  (void)nthreads;
  free(m.B);
  return rc_all;
}

int oracle_sample(const fitoct_problem* p, const fitoct_config* cfg, double* draws,
                  double* stepsize, double* inv_metric, long long* leapfrogs, int nthreads) {
  return oracle_sample_init(p, cfg, draws, stepsize, inv_metric, leapfrogs, nthreads, NULL, NULL,
                            NULL);
}
