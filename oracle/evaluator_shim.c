/*
 * ORACLE (test infrastructure only) -- a CPU fitoct_evaluator over the C
 * oracle's density, linked with libfitoct's HOST drivers (optimize.cpp,
 * host_model.cpp) into oracle/build/libdrivers_cpu.so.  It lets the CPU test
 * suite exercise the L-BFGS and ADVI drivers without a GPU; the product
 * library (fitoct_amd/libfitoct.so) never contains or loads it.
 *
 * The propto=false constants are restated here in C (independently of
 * host_model.cpp lp_constant) from the sampling statements of the model
 * contract (Tests/horseShoePrior.stan:37-42).
 */
#include "fitoct_oracle.c"

struct fitoct_evaluator {
  model m;
  fitoct_problem p;
  int capacity;
  double cst;
  char mask[3 * 24 + 6];
  double* work;
};

static double shim_constant(const fitoct_problem* p) {
  const double l2pi = log(2.0 * M_PI);
  double c = 0.0;
  if (!p->prior_PD) {
    c -= 0.5 * p->N * l2pi;
    for (int i = 0; i < p->N; ++i) c -= log(p->uy[i]);
  }
  if (p->prior_type == 3) return c;
  const double* S = p->Sigma0;
  const double det = S[0] * (S[4] * S[8] - S[5] * S[7]) - S[1] * (S[3] * S[8] - S[5] * S[6]) +
                     S[2] * (S[3] * S[7] - S[4] * S[6]);
  c += -1.5 * l2pi - 0.5 * log(det) - 0.5 * l2pi - log(p->sigma_scale);
  if (p->prior_type == 0) {
    const double rate = p->lambda_conv ? p->lambda_rate : 1.0 / p->lambda_rate;
    c += -0.5 * p->Nn * l2pi + log(rate);
  } else if (p->prior_type == 2) {
    const double a = 0.5 * p->nu;
    c += p->Nn * (-l2pi + a * log(a) - lgamma(a)) - 0.5 * l2pi + 0.5 * log(0.5) - lgamma(0.5);
  }
  return c;
}

int fitoct_evaluator_create(const fitoct_problem* prob, int32_t capacity, int32_t precision,
                            int32_t device, fitoct_evaluator** out) {
  (void)precision;
  (void)device;
  fitoct_evaluator* e = (fitoct_evaluator*)calloc(1, sizeof *e);
  if (model_init(&e->m, prob)) {
    free(e);
    return FITOCT_E_ARG;
  }
  e->p = *prob;
  e->capacity = capacity;
  e->cst = shim_constant(prob);
  const int D = e->m.D, Nn = prob->Nn, f = prob->prior_type;
  for (int j = 0; j < D; ++j)
    e->mask[j] = j < 3 || (f != 3 && j == D - 1) || (f == 0 && j == 3 + Nn) ||
                 (f == 2 && j >= 3 + Nn);
  e->work = (double*)malloc(sizeof(double) * 3 * (Nn + 1));
  *out = e;
  return 0;
}

int fitoct_evaluator_run(fitoct_evaluator* e, int32_t n, const double* q, int32_t jacobian,
                         int32_t normalised, double* lp_out, double* grad_out, double* sumr2_out) {
  if (n < 1 || n > e->capacity) return FITOCT_E_ARG;
  const int D = e->m.D;
  double* g = (double*)malloc(sizeof(double) * D);
  for (int i = 0; i < n; ++i) {
    const double* qi = q + (size_t)i * D;
    double s2 = NAN;
    memset(g, 0, sizeof(double) * D);
    double lp = logp_grad(&e->m, qi, g, &s2, e->work);
    if (!isfinite(lp)) lp = -INFINITY;
    for (int j = 0; j < D; ++j) {
      if (!jacobian && e->mask[j]) {
        lp -= qi[j];
        g[j] -= 1.0;
      }
      if (grad_out) grad_out[(size_t)i * D + j] = g[j];
    }
    if (normalised) lp += e->cst;
    lp_out[i] = lp;
    if (sumr2_out) sumr2_out[i] = s2;
  }
  free(g);
  return 0;
}

void fitoct_evaluator_destroy(fitoct_evaluator* e) {
  if (!e) return;
  free(e->work);
  free(e->m.B);
  free(e);
}
