// C ABI of libfitoct (include/fitoct.h): argument checking, device planning,
// data staging in HBM, kernel dispatch and result download.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <climits>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"
#include "kernel_params.h"
#include "plan_internal.h"

namespace fitoct {
hipError_t launch_family_0(bool logp, bool mixed, int bpt, int nnp, const KParams& P,
                           const KParams* dP, int tiles, hipStream_t st, const int* tile_map);
hipError_t launch_family_1(bool logp, bool mixed, int bpt, int nnp, const KParams& P,
                           const KParams* dP, int tiles, hipStream_t st, const int* tile_map);
hipError_t launch_family_2(bool logp, bool mixed, int bpt, int nnp, const KParams& P,
                           const KParams* dP, int tiles, hipStream_t st, const int* tile_map);
hipError_t launch_family_3(bool logp, bool mixed, int bpt, int nnp, const KParams& P,
                           const KParams* dP, int tiles, hipStream_t st, const int* tile_map);
// the sampler is compiled per prior family (nuts_device.hip, -DFITOCT_FAMILY)
inline hipError_t launch(bool logp, bool mixed, int bpt, int nnp, const KParams& P,
                         const KParams* dP, int tiles, hipStream_t st,
                         const int* tile_map = nullptr) {
  switch (P.family) {
    case 0: return launch_family_0(logp, mixed, bpt, nnp, P, dP, tiles, st, tile_map);
    case 1: return launch_family_1(logp, mixed, bpt, nnp, P, dP, tiles, st, tile_map);
    case 2: return launch_family_2(logp, mixed, bpt, nnp, P, dP, tiles, st, tile_map);
    case 3: return launch_family_3(logp, mixed, bpt, nnp, P, dP, tiles, st, tile_map);
    default: return hipErrorInvalidValue;
  }
}
int lds_bytes(int ppl, int G, int max_depth);
int mig_img_words(int ppl);
}  // namespace fitoct

using namespace fitoct;

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(FITOCT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)


int fitoct::check_init(int C, int D, const double* q, const double* eps, const double* minv) {
  if (eps)
    for (int c = 0; c < C; ++c)
      if (!(eps[c] > 0.0 && eps[c] < INFINITY))
        return fail(FITOCT_E_ARG, "stepsize must be finite and > 0");
  if (minv)
    for (size_t i = 0; i < (size_t)C * D; ++i)
      if (!(minv[i] > 0.0 && minv[i] < INFINITY))
        return fail(FITOCT_E_ARG, "inv_metric must be finite and > 0");
  if (q)
    for (size_t i = 0; i < (size_t)C * D; ++i)
      if (!isfinite(q[i])) return fail(FITOCT_E_ARG, "q_init must be finite");
  return FITOCT_OK;
}

struct fitoct_evaluator {
  fitoct_plan* pl = nullptr;
  int capacity = 0, D = 0, cur_n = -1;
  long long evals = 0;
  double lp_const = 0.0;
  double* d_q = nullptr;
  double* d_out = nullptr;
  std::vector<char> logmask;
  std::vector<double> host;
};

namespace {

int check_problem(const fitoct_problem* p) {
  if (!p) return fail(FITOCT_E_ARG, "problem is NULL");
  if (p->N < 2) return fail(FITOCT_E_ARG, "N must be >= 2");
  if (p->N > FITOCT_MAX_BINS)
    return fail(FITOCT_E_ARG, "N must be <= FITOCT_MAX_BINS (" + std::to_string(FITOCT_MAX_BINS) + ")");
  if (!p->x || !p->y || !p->uy) return fail(FITOCT_E_ARG, "x, y, uy must be non-NULL");
  const bool mono = p->prior_type == FITOCT_MODEL_MONOEXP;
  if (!mono && (p->Nn < 2 || p->Nn > 24)) return fail(FITOCT_E_ARG, "Nn must be in [2, 24]");
  if (p->theta_prior != 0 && p->theta_prior != 1)
    return fail(FITOCT_E_ARG, "theta_prior must be 0 or 1");
  if (p->theta_prior == 1 && !mono)
    return fail(FITOCT_E_ARG, "theta_prior = 1 is the mono-exponential model's switch");
  if (p->theta_prior == 1 && !(p->lambda_scale > 0.0))
    return fail(FITOCT_E_ARG, "lambda_scale must be > 0");
  if (mono && p->prior_PD && p->theta_prior == 0)
    return fail(FITOCT_E_ARG, "the mono-exponential model has a flat prior: prior_PD must be 0");
  if (model_dim(p->prior_type, p->Nn) < 0) return fail(FITOCT_E_ARG, "unknown prior_type");
  if (p->data_type != 1 && p->data_type != 2) return fail(FITOCT_E_ARG, "data_type must be 1 or 2");
  for (int i = 0; i < p->N; ++i) {
    if (!isfinite(p->x[i]) || !isfinite(p->y[i]) || !(p->uy[i] > 0.0) || !isfinite(p->uy[i]))
      return fail(FITOCT_E_ARG, "x, y must be finite and uy > 0 at bin " + std::to_string(i));
  }
  if (!mono && !p->B) {   // x~ = (x - min x) / (max x - min x) (server.R:635)
    double xmin = p->x[0], xmax = p->x[0];
    for (int i = 1; i < p->N; ++i) {
      xmin = fmin(xmin, p->x[i]);
      xmax = fmax(xmax, p->x[i]);
    }
    if (!(xmax > xmin)) return fail(FITOCT_E_ARG, "x must not be constant");
  }
  for (int j = 0; j < 3; ++j)
    if (!(p->theta0[j] > 0.0)) return fail(FITOCT_E_ARG, "theta0 must be > 0");
  if (p->prior_type == FITOCT_PRIOR_NORMAL && !(p->lambda_rate > 0.0))
    return fail(FITOCT_E_ARG, "lambda_rate must be > 0");
  if (p->prior_type == FITOCT_PRIOR_LASSO && !(p->lambda_scale > 0.0))
    return fail(FITOCT_E_ARG, "lambda_scale must be > 0");
  if (p->prior_type == FITOCT_PRIOR_HORSESHOE && !(p->nu >= 1.0))
    return fail(FITOCT_E_ARG, "nu must be >= 1 (horseShoePrior.stan:13)");
  if (!(p->sigma_scale > 0.0)) return fail(FITOCT_E_ARG, "sigma_scale must be > 0");
  return FITOCT_OK;
}

int invert3(const double* S, double* Si) {
  const double a = S[0], b = S[1], c = S[2], d = S[3], e = S[4], f = S[5], g = S[6], h = S[7],
               i = S[8];
  const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
  const double det = a * A + b * B + c * C;
  if (!(fabs(det) > 0.0) || !isfinite(det)) return fail(FITOCT_E_ARG, "Sigma0 is singular");
  Si[0] = A / det;
  Si[1] = -(b * i - c * h) / det;
  Si[2] = (b * f - c * e) / det;
  Si[3] = B / det;
  Si[4] = (a * i - c * g) / det;
  Si[5] = -(a * f - c * d) / det;
  Si[6] = C / det;
  Si[7] = -(a * h - b * g) / det;
  Si[8] = (a * e - b * d) / det;
  if (!(A > 0.0) || !(det > 0.0)) return fail(FITOCT_E_ARG, "Sigma0 must be positive definite");
  return FITOCT_OK;
}

// Shapes: bins are strided over the 512 lanes of a tile's gradient waves; up to
// 4 bins per lane keep their data in VGPRs for the whole run (MODE_POLY: 5 f64
// values per bin; MODE_ROWS: 3 + NNP fp32 values), beyond that they are streamed.
// bins per gradient lane kept in registers (0 = streamed from HBM/L2 every sweep).
// The factorised f64 basis holds 5 values per bin, so up to 8 bins per lane fit;
// explicit fp32 basis rows hold NNP + 3 values per bin, up to 4.
void choose_bins(int N, int max_bpt, int& bpt, int& n_pad) {
  bpt = 0;
  for (int b = 1; b <= max_bpt; b *= 2)
    if (N <= b * GT) { bpt = b; break; }
  n_pad = bpt ? bpt * GT : (N + GT - 1) / GT * GT;
}

// MODE_POLY factors of the SE basis on the uniform grid g_l = g_0 + l*dg:
//   K(x~_i, g_l) = a_i t_i^l b_l, a_i = exp(-(x~_i-g_0)^2/(2s2)),
//   t_i = exp((x~_i-g_0) dg/s2), b_l = exp(-(l dg)^2/(2s2)),
// and K^-1 = (K(xGP,xGP) + nugget I)^-1.  Accepted only if the factorised basis
// reproduces the Cholesky basis B to 1e-10 (relative to max|B|) and no power
// t^l (l < nnp) can overflow; otherwise the caller falls back to streamed rows.
bool build_poly(const fitoct_problem* p, const std::vector<double>& B, int nnp,
                std::vector<double>& ta, std::vector<double>& kinv, std::vector<double>& bv) {
  const int N = p->N, Nn = p->Nn;
  double xmin = p->x[0], xmax = p->x[0];
  for (int i = 1; i < N; ++i) {
    xmin = std::min(xmin, p->x[i]);
    xmax = std::max(xmax, p->x[i]);
  }
  const double rho = (p->rho > 0.0) ? p->rho : 1.0 / Nn;
  const double s2 = (p->kernel_conv == 0) ? rho * rho : 0.5 * rho * rho;
  double g0, dg;
  if (p->grid_type == FITOCT_GRID_INTERNAL) {
    const double dx = 1.0 / (Nn + 1);
    g0 = dx / 2;
    dg = (1.0 - dx) / (Nn - 1);
  } else {
    g0 = 0.0;
    dg = 1.0 / (Nn - 1);
  }
  ta.assign((size_t)2 * N, 0.0);
  for (int i = 0; i < N; ++i) {
    const double u = (p->x[i] - xmin) / (xmax - xmin) - g0;
    const double lt = u * dg / s2, la = -u * u / (2.0 * s2);
    if (fabs(lt) * (nnp - 1) > 650.0 || la < -650.0) return false;
    ta[2 * i] = exp(lt);
    ta[2 * i + 1] = exp(la);
  }
  bv.assign(Nn, 0.0);
  for (int l = 0; l < Nn; ++l) bv[l] = exp(-(l * dg) * (l * dg) / (2.0 * s2));
  // K^-1 by Cholesky
  std::vector<double> xg(Nn), L((size_t)Nn * Nn, 0.0);
  for (int k = 0; k < Nn; ++k) xg[k] = g0 + k * dg;
  for (int i = 0; i < Nn; ++i)
    for (int j = 0; j <= i; ++j) {
      const double d = xg[i] - xg[j];
      double sum = exp(-d * d / (2.0 * s2)) + (i == j ? p->nugget : 0.0);
      for (int k = 0; k < j; ++k) sum -= L[i * Nn + k] * L[j * Nn + k];
      if (i == j) {
        if (!(sum > 0.0)) return false;
        L[i * Nn + i] = sqrt(sum);
      } else {
        L[i * Nn + j] = sum / L[j * Nn + j];
      }
    }
  std::vector<double> Li((size_t)Nn * Nn, 0.0);  // L^-1 (lower)
  for (int j = 0; j < Nn; ++j) {
    Li[j * Nn + j] = 1.0 / L[j * Nn + j];
    for (int i = j + 1; i < Nn; ++i) {
      double sum = 0.0;
      for (int k = j; k < i; ++k) sum -= L[i * Nn + k] * Li[k * Nn + j];
      Li[i * Nn + j] = sum / L[i * Nn + i];
    }
  }
  kinv.assign((size_t)Nn * Nn, 0.0);
  for (int i = 0; i < Nn; ++i)
    for (int j = 0; j < Nn; ++j) {
      double sum = 0.0;
      for (int k = std::max(i, j); k < Nn; ++k) sum += Li[k * Nn + i] * Li[k * Nn + j];
      kinv[i * Nn + j] = sum;
    }
  // exactness check against the Cholesky basis
  double bmax = 0.0, err = 0.0;
  std::vector<double> row(Nn);
  for (int i = 0; i < N; ++i) {
    double tp = ta[2 * i + 1];
    for (int l = 0; l < Nn; ++l) {
      row[l] = tp * bv[l];
      tp *= ta[2 * i];
    }
    for (int k = 0; k < Nn; ++k) {
      double v = 0.0;
      for (int l = 0; l < Nn; ++l) v += row[l] * kinv[l * Nn + k];
      const double b = B[(size_t)i * Nn + k];
      bmax = std::max(bmax, fabs(b));
      err = std::max(err, fabs(v - b));
    }
  }
  return err <= 1e-10 * std::max(1.0, bmax);
}

// MODE_POLY with bins in registers: on an arithmetic depth grid the bins
// tid + b*GT of one lane have t = t_tid * R^b (t_i = exp(u_i dg / s2), u_i linear
// in i), which lets the sweep form a lane's moments by Horner in R^l
// (nuts_device.hip moments_geo).  Accepted only if every x_i lies on the line
// through x_0 and x_{N-1} to 1e-12 of the range and no (R^l)^b can overflow.
bool geo_ratios(const fitoct_problem* p, int nnp, int bpt, double* R) {
  const int N = p->N, Nn = p->Nn;
  if (bpt < 2 || Nn < 2) return false;
  double xmin = p->x[0], xmax = p->x[0];
  for (int i = 1; i < N; ++i) {
    xmin = std::min(xmin, p->x[i]);
    xmax = std::max(xmax, p->x[i]);
  }
  const double range = xmax - xmin, step = (p->x[N - 1] - p->x[0]) / (N - 1);
  for (int i = 0; i < N; ++i)
    if (fabs(p->x[i] - (p->x[0] + i * step)) > 1e-12 * range) return false;
  const double rho = (p->rho > 0.0) ? p->rho : 1.0 / Nn;
  const double s2 = (p->kernel_conv == 0) ? rho * rho : 0.5 * rho * rho;
  const double dg = (p->grid_type == FITOCT_GRID_INTERNAL) ? (1.0 - 1.0 / (Nn + 1)) / (Nn - 1)
                                                           : 1.0 / (Nn - 1);
  const double logR = GT * (step / range) * dg / s2;
  if (fabs(logR) * (nnp - 1) * (bpt - 1) > 600.0) return false;
  if (bpt == 16) {   // c*x_b and t_b are formed in the kernel: x must be on the line to ~ulps
    for (int i = 0; i < N; ++i)
      if (fabs(p->x[i] - (p->x[0] + i * step)) > 4e-16 * std::max(fabs(xmin), fabs(xmax)) + 1e-300)
        return false;
    if (fabs(logR) * (bpt - 1) > 600.0) return false;
  }
  for (int l = 0; l < 24; ++l) R[l] = exp(l * logR);
  return true;
}

template <class R>
void stage(const fitoct_problem* p, const std::vector<double>& B, const std::vector<double>& ta,
           int mode, int n_pad, int nnp, std::vector<char>& out) {
  const size_t n = (size_t)n_pad;
  const int nr = (mode == MODE_POLY) ? 2 : nnp;
  out.assign(sizeof(R) * (3 * n + n * nr), 0);
  R* cx = (R*)out.data();
  R* y = cx + n;
  R* isu = y + n;
  R* Bp = isu + n;
  for (int i = 0; i < p->N; ++i) {
    cx[i] = (R)((double)p->data_type * p->x[i]);
    y[i] = (R)(p->y[i] / p->uy[i]);   // y / uy: the sweep forms (y - m) / uy as one FMA
    isu[i] = (R)(1.0 / p->uy[i]);
    if (mode == MODE_POLY) {
      Bp[2 * (size_t)i] = (R)ta[2 * (size_t)i];
      Bp[2 * (size_t)i + 1] = (R)ta[2 * (size_t)i + 1];
    } else {
      for (int k = 0; k < p->Nn; ++k) Bp[(size_t)i * nnp + k] = (R)B[(size_t)i * p->Nn + k];
    }
  }
}

// common planning for the sampler and the logp kernel
int plan_common(fitoct_plan* pl, const fitoct_problem* p, int chains, int precision, int device,
                int max_depth, int g_chains = 0, int force_bpt = -1, bool poly_only = false) {
  int rc = check_problem(p);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(FITOCT_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(FITOCT_E_ARG, "device ordinal out of range");
  HIP_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));

  pl->prob = *p;
  pl->prob.x = pl->prob.y = pl->prob.uy = pl->prob.B = nullptr;  // never keep caller pointers
  pl->mixed = (precision == FITOCT_PREC_MIXED);
  const int D = model_dim(p->prior_type, p->Nn);
  // NNP: padded control-point count of the kernel instantiation (15 = FitOCT's Nn,
  // ctrlParams.yaml:4, with no padding work in the sweep; 24 covers Nn = 16..24)
  pl->nnp = (p->Nn <= 15) ? 15 : 24;
  pl->ppl = (D <= WAVE) ? 1 : 2;
  if (pl->nnp == 15 && pl->ppl == 2) pl->nnp = 24;  // the (24, 2) instantiation covers it
  if (pl->nnp == 24) pl->ppl = 2;
  const bool mono = p->prior_type == FITOCT_MODEL_MONOEXP;
  std::vector<double> B, xg;
  if (mono) {
    // no GP term: a factorised basis of zeros (dL = 0); Nn = 0 inside the kernel
  } else if (p->B) {
    B.assign(p->B, p->B + (size_t)p->N * p->Nn);
  } else {
    rc = build_basis(p, B, xg);
    if (rc) return rc;
  }
  // basis mode (see kernel_params.h BasisMode)
  std::vector<double> ta, kinv, bv;
  int mode;
  bool rows_res = false;
  if (mono && !pl->mixed) {
    mode = MODE_POLY;
    ta.assign(2 * (size_t)p->N, 0.0);
  } else if (mono) {   // the mixed kernels are row-mode only: rows of zeros (dL = 0)
    mode = MODE_ROWS;
    B.assign((size_t)p->N * p->Nn, 0.0);
  } else if (pl->mixed) {
    mode = MODE_ROWS;
  } else {
    // N <= 512 (configs 2 and 5): the basis rows themselves, 1-2 bins of 15 doubles per lane
    // in the gradient waves' registers -- the sampler's leaf then has no K^-1 products
    // (write_mp, finish_grad) on its critical path.  Wider problems: the factorised basis.
    rows_res = !poly_only && p->N <= 2 * GT && pl->nnp == 15;
    const bool poly = !rows_res && !p->B && build_poly(p, B, pl->nnp, ta, kinv, bv);
    mode = poly ? MODE_POLY : MODE_ROWS;
  }
  // f64 rows (NNP doubles per bin) are streamed, but for N <= 512 (rows_res)
  int n_pad;
  choose_bins(p->N, mode == MODE_POLY ? 8 : pl->mixed ? 4 : rows_res ? 2 : 0, pl->bpt, n_pad);
  // N in (2048, 4096] on an arithmetic depth grid: 16 bins per lane in the compact
  // layout (y, 1/uy, a in registers; c*x and t formed from the lane's first bin)
  double R16[24];
  if (mode == MODE_POLY && !mono && !pl->mixed && pl->bpt == 0 && p->N <= 16 * GT &&
      force_bpt < 0 && getenv("FITOCT_NO_GEO") == nullptr &&
      geo_ratios(p, pl->nnp, 16, R16)) {
    pl->bpt = 16;
    n_pad = 16 * GT;
  }
  if (force_bpt >= 0 && force_bpt != pl->bpt) {   // batch: the batch's common bin layout
    if (force_bpt != 0 && force_bpt < pl->bpt) return fail(FITOCT_E_ARG, "bin layout too small");
    pl->bpt = force_bpt;
    n_pad = force_bpt ? force_bpt * GT : (p->N + GT - 1) / GT * GT;
  }
  std::vector<char> staged;
  if (pl->mixed) stage<float>(p, B, ta, mode, n_pad, pl->nnp, staged);
  else stage<double>(p, B, ta, mode, n_pad, pl->nnp, staged);
  const size_t kbytes = sizeof(double) * (kinv.size() + bv.size());
  HIP_TRY(hipMalloc(&pl->d_data, staged.size() + kbytes + 16));
  HIP_TRY(hipMemcpy(pl->d_data, staged.data(), staged.size(), hipMemcpyHostToDevice));
  double* dk = (double*)((char*)pl->d_data + (staged.size() + 15) / 16 * 16);
  if (mode == MODE_POLY) {
    HIP_TRY(hipMemcpy(dk, kinv.data(), sizeof(double) * kinv.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dk + kinv.size(), bv.data(), sizeof(double) * bv.size(),
                      hipMemcpyHostToDevice));
  }
  const size_t rs = pl->mixed ? sizeof(float) : sizeof(double);
  KParams& k = pl->kp;
  k.cx = pl->d_data;
  k.y = (const char*)pl->d_data + rs * n_pad;
  k.isu = (const char*)pl->d_data + 2 * rs * n_pad;
  k.B = (const char*)pl->d_data + 3 * rs * n_pad;
  k.mode = mode;
  k.Kinv = dk;
  k.bvec = dk + kinv.size();
  k.N = p->N;
  k.n_pad = n_pad;
  k.geo = (mode == MODE_POLY && !mono && !pl->mixed && getenv("FITOCT_NO_GEO") == nullptr)
              ? geo_ratios(p, pl->nnp, pl->bpt, k.geo_R) : 0;
  if (pl->bpt == 16) {
    if (!k.geo) return fail(FITOCT_E_INTERNAL, "16-bin layout without a geometric grid");
    const double cstep = (double)p->data_type * (p->x[p->N - 1] - p->x[0]) / (p->N - 1);
    for (int b = 0; b < 16; ++b) k.geo_dcx[b] = (double)b * GT * cstep;
    k.geo_tmax = 0.0;
    for (int i = 0; i < p->N; ++i) k.geo_tmax = std::max(k.geo_tmax, ta[2 * (size_t)i]);
  }
  k.Nn = mono ? 0 : p->Nn;
  k.D = D;
  k.family = p->prior_type;
  k.prior_PD = p->prior_PD ? 1 : 0;
  for (int j = 0; j < 3; ++j) k.theta0[j] = p->theta0[j];
  if (mono) {
    for (int j = 0; j < 9; ++j) k.S0inv[j] = 0.0;
  } else {
    rc = invert3(p->Sigma0, k.S0inv);
    if (rc) return rc;
  }
  k.lambda_rate_eff = (p->lambda_conv == 0) ? 1.0 / p->lambda_rate : p->lambda_rate;
  k.lambda_scale = p->lambda_scale;
  k.nu = p->nu;
  k.sigma_scale = p->sigma_scale;
  k.sigma_scale_inv = 1.0 / p->sigma_scale;
  k.theta_rate = p->theta_prior == 1 ? 1.0 / p->lambda_scale : 0.0;
  k.chains = chains;

  // chains per tile: fill every CU with one tile first, then stack chains
  const int ncu = std::max(1, prop.multiProcessorCount);
  pl->ncu = ncu;
  // (a batch plans every problem's tiles from the batch's total chain count)
  const int gc = g_chains > 0 ? g_chains : chains;
  int G = std::max(1, std::min(GMAX, (gc + ncu - 1) / ncu));
  // (the kernel's static LDS comes on top of the carve: STATIC_LDS_RESERVE)
  while (G > 1 && lds_bytes(pl->ppl, G, max_depth) > 160 * 1024 - STATIC_LDS_RESERVE) --G;
  if (lds_bytes(pl->ppl, G, max_depth) > 160 * 1024 - STATIC_LDS_RESERVE)
    return fail(FITOCT_E_ARG, "max_treedepth too large for the LDS budget");
  k.G = G;
  k.max_depth = max_depth;
  k.spec = 0;   // set below, once migration is decided
  pl->tiles = (chains + G - 1) / G;
  pl->lds = lds_bytes(pl->ppl, G, max_depth);
  return FITOCT_OK;
}

int plan_create(const fitoct_problem* prob, const fitoct_config* cfg, int g_chains,
                int force_bpt, fitoct_plan** out, bool poly_only = false);

// Migrating tiles of several chains speculate once they host <= this many live chains.
// Measured on config 3 at full length (profiles/r03_ab_spec_live.txt, two interleaved
// runs each): 0 (no speculation) 119.1 k draws/s, 1: 119.7-120.2 k, 2: 121.2-121.4 k,
// 3: 121.5-122.0 k, 4 (always): 119.5-120.3 k.  Tiles that do not migrate (batch mode,
// config 5) lose 7 % with any tail speculation (the speculative kernel's extra registers
// and per-leaf policy read), so they do not speculate.
constexpr int kSpecLiveMigrating = 3;

void free_plan(fitoct_plan* pl) {
  if (!pl) return;
  for (fitoct_plan* sh : pl->shards) free_plan(sh);
  (void)hipFree(pl->d_data);
  (void)hipFree(pl->d_draws);
  (void)hipFree(pl->d_stack);
  (void)hipFree(pl->d_fin);
  (void)hipFree(pl->d_init);
  (void)hipFree(pl->d_status);
  (void)hipFree(pl->d_leap);
  (void)hipFree(pl->d_kp);
  (void)hipFree(pl->d_mig);
  (void)hipFree(pl->d_mig_img);
  (void)hipFree(pl->d_stamps);
  (void)hipFree(pl->d_pair_hdr);
  (void)hipFree(pl->d_pair_buf);
  if (pl->h_prog) (void)hipHostFree(pl->h_prog);
  if (pl->h_cancel) (void)hipHostFree(pl->h_cancel);
  if (pl->ev0) (void)hipEventDestroy(pl->ev0);
  if (pl->ev1) (void)hipEventDestroy(pl->ev1);
  if (pl->own_stream) (void)hipStreamDestroy(pl->own_stream);
  delete pl;
}

}  // namespace

extern "C" {

int32_t fitoct_abi_version(void) { return FITOCT_ABI_VERSION; }

int32_t fitoct_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int32_t fitoct_struct_sizes(int32_t* problem, int32_t* config, int32_t* result, int32_t* info) {
  if (problem) *problem = (int32_t)sizeof(fitoct_problem);
  if (config) *config = (int32_t)sizeof(fitoct_config);
  if (result) *result = (int32_t)sizeof(fitoct_result);
  if (info) *info = (int32_t)sizeof(fitoct_plan_info);
  return FITOCT_OK;
}

void fitoct_default_config(fitoct_config* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  c->chains = 4;  // server.R:469
  c->warmup = 500;
  c->samples = 1000;
  c->seed = 1234;
  c->adapt_delta = 0.8;
  c->max_treedepth = 10;
  c->adapt_engaged = 1;
  c->stepsize = 1.0;
  c->gamma = 0.05;
  c->kappa = 0.75;
  c->t0 = 10.0;
  c->init_buffer = 75;
  c->term_buffer = 50;
  c->window = 25;
  c->init_radius = 2.0;
  c->save_warmup = 1;
  c->precision = FITOCT_PREC_F64;
}

void fitoct_default_problem(fitoct_problem* p) {
  if (!p) return;
  memset(p, 0, sizeof *p);
  p->data_type = 2;
  p->Nn = 10;
  p->grid_type = FITOCT_GRID_INTERNAL;
  p->prior_type = FITOCT_PRIOR_NORMAL;
  p->lambda_rate = 0.1;
  p->lambda_scale = 10.0;
  p->nu = 1.0;
  p->sigma_scale = 10.0;
  p->nugget = 1e-9;
  p->theta0[0] = 1000.0;
  p->theta0[1] = 2000.0;
  p->theta0[2] = 300.0;
  for (int j = 0; j < 3; ++j) p->Sigma0[4 * j] = (0.05 * p->theta0[j]) * (0.05 * p->theta0[j]);
}

int32_t fitoct_dim(int32_t prior_type, int32_t Nn) { return model_dim(prior_type, Nn); }

int32_t fitoct_n_cols(int32_t prior_type, int32_t Nn) {
  const int D = model_dim(prior_type, Nn);
  return D < 0 ? -1 : D + 8;
}

int32_t fitoct_column_name(int32_t prior_type, int32_t Nn, int32_t i, char* buf, int32_t buflen) {
  return guarded(__func__, [&]() -> int32_t {
    const std::string s = column_name(prior_type, Nn, i);
    if (s.empty()) return fail(FITOCT_E_ARG, "column index out of range");
    if (!buf || buflen < (int32_t)s.size() + 1) return fail(FITOCT_E_ARG, "buffer too small");
    memcpy(buf, s.c_str(), s.size() + 1);
    return FITOCT_OK;
  });
}

int32_t fitoct_build_basis(const fitoct_problem* prob, double* B_out, double* xGP_out) {
  return guarded(__func__, [&]() -> int32_t {
    if (!prob || !B_out) return fail(FITOCT_E_ARG, "NULL argument");
    if (prob->N < 2 || !prob->x) return fail(FITOCT_E_ARG, "need x with N >= 2");
    std::vector<double> B, xg;
    const int rc = build_basis(prob, B, xg);
    if (rc) return rc;
    memcpy(B_out, B.data(), B.size() * sizeof(double));
    if (xGP_out) memcpy(xGP_out, xg.data(), xg.size() * sizeof(double));
    return FITOCT_OK;
  });
}

int32_t fitoct_evaluator_create(const fitoct_problem* prob, int32_t capacity, int32_t precision,
                                int32_t device, fitoct_evaluator** out) {
  return guarded(__func__, [&]() -> int32_t {
    if (!out) return fail(FITOCT_E_ARG, "out is NULL");
    *out = nullptr;
    if (capacity < 1) return fail(FITOCT_E_ARG, "capacity must be >= 1");
    // released on every early return or exception until handed to the caller
    std::unique_ptr<fitoct_evaluator, void (*)(fitoct_evaluator*)> guard(new fitoct_evaluator(),
                                                                       fitoct_evaluator_destroy);
    fitoct_evaluator* ev = guard.get();
    ev->pl = new fitoct_plan();
    int rc = plan_common(ev->pl, prob, capacity, precision, device, 0);
    ev->pl->cfg.device = device;
    auto run = [&]() -> int {
      if (rc) return rc;
      const int D = ev->pl->kp.D;
      ev->capacity = capacity;
      ev->D = D;
      ev->lp_const = lp_constant(prob);
      ev->logmask.resize(D);
      for (int j = 0; j < D; ++j) ev->logmask[j] = log_transformed(prob->prior_type, prob->Nn, j);
      HIP_TRY(hipMalloc(&ev->d_q, sizeof(double) * (size_t)capacity * D));
      HIP_TRY(hipMalloc(&ev->d_out, sizeof(double) * (size_t)capacity * (D + 2)));
      HIP_TRY(hipMalloc(&ev->pl->d_kp, sizeof(KParams)));
      KParams& k = ev->pl->kp;
      k.q_in = ev->d_q;
      k.grad_out = ev->d_out;
      return FITOCT_OK;
    };
    rc = run();
    if (rc) return rc;
    *out = guard.release();
    return FITOCT_OK;
  });
}

int32_t fitoct_evaluator_run(fitoct_evaluator* ev, int32_t n, const double* q, int32_t jacobian,
                             int32_t normalised, double* lp_out, double* grad_out,
                             double* sumr2_out) {
  return guarded(__func__, [&]() -> int32_t {
    if (!ev || !q || !lp_out) return fail(FITOCT_E_ARG, "bad buffers");
    if (n < 1 || n > ev->capacity) return fail(FITOCT_E_ARG, "n_points must be in [1, capacity]");
    fitoct_plan* pl = ev->pl;
    KParams& k = pl->kp;
    const int D = ev->D;
    HIP_TRY(hipSetDevice(pl->cfg.device));
    if (n != ev->cur_n) {  // outputs are laid out for n points: grad[n][D] | lp[n] | sumr2[n]
      k.chains = n;
      k.lp_out = ev->d_out + (size_t)n * D;
      k.s2_out = k.lp_out + n;
      pl->tiles = (n + k.G - 1) / k.G;
      HIP_TRY(hipMemcpy(pl->d_kp, &k, sizeof(KParams), hipMemcpyHostToDevice));
      ev->cur_n = n;
    }
    HIP_TRY(hipMemcpy(ev->d_q, q, sizeof(double) * (size_t)n * D, hipMemcpyHostToDevice));
    HIP_TRY(launch(true, pl->mixed, pl->bpt, pl->nnp, k, pl->d_kp, pl->tiles, 0));
    // one copy back of grad | lp | sumr2 (contiguous)
    ev->host.resize((size_t)n * (D + 2));
    HIP_TRY(hipMemcpy(ev->host.data(), ev->d_out, sizeof(double) * ev->host.size(),
                      hipMemcpyDeviceToHost));
    const double* g = ev->host.data();
    const double* lp = g + (size_t)n * D;
    for (int i = 0; i < n; ++i) {
      double v = lp[i];
      const double* qi = q + (size_t)i * D;
      if (!jacobian)
        for (int j = 0; j < D; ++j)
          if (ev->logmask[j]) v -= qi[j];
      if (normalised) v += ev->lp_const;
      lp_out[i] = isfinite(lp[i]) ? v : -INFINITY;
      if (grad_out)
        for (int j = 0; j < D; ++j)
          grad_out[(size_t)i * D + j] = g[(size_t)i * D + j] - ((!jacobian && ev->logmask[j]) ? 1.0 : 0.0);
      if (sumr2_out) sumr2_out[i] = lp[n + i];
    }
    ev->evals += n;
    return FITOCT_OK;
  });
}

void fitoct_evaluator_destroy(fitoct_evaluator* ev) {
  if (!ev) return;
  (void)hipFree(ev->d_q);
  (void)hipFree(ev->d_out);
  free_plan(ev->pl);
  delete ev;
}

int32_t fitoct_logp_grad(const fitoct_problem* prob, int32_t n_points, const double* q,
                         double* lp_out, double* grad_out, double* sumr2_out, int32_t precision,
                         int32_t device) {
  return guarded(__func__, [&]() -> int32_t {
    if (n_points < 1 || !q || !lp_out || !grad_out) return fail(FITOCT_E_ARG, "bad buffers");
    fitoct_evaluator* ev = nullptr;
    int rc = fitoct_evaluator_create(prob, n_points, precision, device, &ev);
    if (rc) return rc;
    rc = fitoct_evaluator_run(ev, n_points, q, 1, 0, lp_out, grad_out, sumr2_out);
    fitoct_evaluator_destroy(ev);
    return rc;
  });
}

int32_t fitoct_plan_create(const fitoct_problem* prob, const fitoct_config* cfg,
                           fitoct_plan** out) {
  return guarded(__func__, [&]() -> int32_t {
    if (!out) return fail(FITOCT_E_ARG, "out is NULL");
    *out = nullptr;
    if (!cfg) return fail(FITOCT_E_ARG, "config is NULL");
    if (cfg->chains < 1) return fail(FITOCT_E_ARG, "chains must be >= 1");
    std::vector<int> devs;
    const int rc = resolve_devices(cfg, cfg->chains, devs);
    if (rc) return rc;
    if (devs.size() > 1) return group_plan_create(prob, cfg, devs, out);
    fitoct_config c = *cfg;
    c.device = devs[0];
    c.n_devices = 0;
    return plan_create(prob, &c, 0, -1, out);
  });
}

}  // extern "C"

namespace {
// Paired tiles (nuts_device.hip "paired tiles"): a launch of one-chain tiles with two-ended
// trajectories whose 2 x tiles (in whole groups of 8 + 8 blocks) fit on the chip grows each
// trajectory's forward end in a partner tile with its own gradient waves, instead of sharing
// the tile's.  Same draws bit for bit: the partner runs the same producer on the same values.
// A partner that does not get a CU at launch leaves its primary to grow both ends (the pair's
// hand-shake), so this is safe on a shared GPU too.  FITOCT_NO_PAIR=1: off.
bool want_pairs(const KParams& k, int tiles, int ncu) {
  if (!(k.bidi && k.G == 1 && pair_grid(tiles) <= ncu) || getenv("FITOCT_NO_PAIR") != nullptr)
    return false;
  // with the basis rows (N <= 512) an unpaired tile is faster (its chain's wave books the
  // forward end: config 2 253 k vs 245 k draws/s, profiles/r06_ab_unpaired.txt), so there the
  // pairing is on only with FITOCT_PAIR=1
  return k.mode == MODE_POLY || getenv("FITOCT_PAIR") != nullptr;
}
// the pairs' hand-off words and buffers for `tiles` tiles; sets every k.pair_* but the count
int alloc_pairs(KParams& k, int tiles, int ppl, int** hdr, double** buf) {
  k.pair = 1;
  k.pair_tiles = tiles;
  // the start (q, p, g, minv + scalars), then two subtree record slots (5 vectors + 16 scalars)
  k.pair_stride = (PAIR_START_DOUBLES + WAVE * ppl * 4 + 2 * (WAVE * ppl * 5 + 16) + 15) / 16 * 16;
  HIP_TRY(hipMalloc(hdr, sizeof(int) * PAIR_HDR_INTS * (size_t)tiles));
  HIP_TRY(hipMalloc(buf, sizeof(double) * (size_t)k.pair_stride * tiles));
  k.pair_hdr = *hdr;
  k.pair_buf = *buf;
  const char* t = getenv("FITOCT_TEST_PAIR_ABSENT");   // test hook: partners never join
  k.pair_test_absent = (t && atoi(t) != 0) ? 1 : 0;
  return FITOCT_OK;
}

int plan_create(const fitoct_problem* prob, const fitoct_config* cfg, int g_chains,
                int force_bpt, fitoct_plan** out, bool poly_only) {
  if (!out) return fail(FITOCT_E_ARG, "out is NULL");
  *out = nullptr;
  if (!cfg) return fail(FITOCT_E_ARG, "config is NULL");
  if (cfg->chains < 1) return fail(FITOCT_E_ARG, "chains must be >= 1");
  if (cfg->warmup < 0 || cfg->samples < 1) return fail(FITOCT_E_ARG, "warmup >= 0, samples >= 1");
  if (cfg->max_treedepth < 1 || cfg->max_treedepth > MAXDEPTH)
    return fail(FITOCT_E_ARG, "max_treedepth must be in [1, 16]");
  if (!(cfg->adapt_delta > 0.0 && cfg->adapt_delta < 1.0))
    return fail(FITOCT_E_ARG, "adapt_delta must be in (0, 1)");
  if (!(cfg->stepsize > 0.0)) return fail(FITOCT_E_ARG, "stepsize must be > 0");
  // released on every early return or exception until handed to the caller
  std::unique_ptr<fitoct_plan, void (*)(fitoct_plan*)> guard(new fitoct_plan(), free_plan);
  fitoct_plan* pl = guard.get();
  int rc = plan_common(pl, prob, cfg->chains, cfg->precision, cfg->device, cfg->max_treedepth,
                       g_chains, force_bpt, poly_only);
  if (rc) return rc;
  pl->cfg = *cfg;
  KParams& k = pl->kp;
  const int C = cfg->chains, D = k.D;
  k.chain_offset = cfg->chain_offset;
  k.warmup = cfg->warmup;
  k.samples = cfg->samples;
  k.max_depth = cfg->max_treedepth;
  k.save_warmup = cfg->save_warmup ? 1 : 0;
  k.adapt = cfg->adapt_engaged ? 1 : 0;
  k.seed = cfg->seed;
  k.adapt_delta = cfg->adapt_delta;
  k.gamma = cfg->gamma > 0 ? cfg->gamma : 0.05;
  k.kappa = cfg->kappa > 0 ? cfg->kappa : 0.75;
  k.t0 = cfg->t0 > 0 ? cfg->t0 : 10.0;
  k.stepsize0 = cfg->stepsize;
  k.init_radius = cfg->init_radius;
  k.init_buffer = cfg->init_buffer;
  k.term_buffer = cfg->term_buffer;
  k.base_window = cfg->window;
  const long long iters = (long long)cfg->warmup + cfg->samples;
  k.max_steps = iters * ((1LL << cfg->max_treedepth) + 1) + 4000LL * (cfg->warmup / 10 + 4) + 10000;
  k.iters_saved = cfg->save_warmup ? (int)iters : cfg->samples;
  k.ncols = D + 8;
  pl->draws_bytes = sizeof(double) * (size_t)C * k.iters_saved * k.ncols;
  const int vlen = WAVE * pl->ppl;
  auto setup = [&]() -> int {
    // proposal pools: the chains', then the two-ended producers' (GMAX per tile; produce)
    const size_t pools = (size_t)C + (size_t)GMAX * ((C + pl->kp.G - 1) / pl->kp.G);
    HIP_TRY(hipMalloc(&pl->d_stack, sizeof(double) * pools * (cfg->max_treedepth + 1) * POOL_VECS * vlen));
    HIP_TRY(hipMalloc(&pl->d_fin, sizeof(double) * (size_t)C * (1 + 2 * D)));
    HIP_TRY(hipMalloc(&pl->d_status, sizeof(int) * C));
    // [chains] leapfrogs per chain, then the launch's two-ended and paired transition counts
    HIP_TRY(hipMalloc(&pl->d_leap, sizeof(long long) * (C + 2)));
    HIP_TRY(hipEventCreate(&pl->ev0));
    HIP_TRY(hipEventCreate(&pl->ev1));
    return FITOCT_OK;
  };
  rc = setup();
  if (rc) return rc;
  k.stack = pl->d_stack;
  k.fin_eps = pl->d_fin;
  k.fin_minv = pl->d_fin + C;
  k.fin_q = pl->d_fin + C + (size_t)C * D;
  k.chain_status = pl->d_status;
  k.leapfrogs = pl->d_leap;
  k.bidi_count = (unsigned long long*)(pl->d_leap + C);
  k.pair_count = (unsigned long long*)(pl->d_leap + C + 1);
  if (g_chains == 0) {   // progress / cancellation (fitoct_plan_poll / _cancel); batch: off
    auto prog_setup = [&]() -> int {
      HIP_TRY(hipHostMalloc((void**)&pl->h_prog, sizeof(int) * C,
                            hipHostMallocMapped | hipHostMallocCoherent));
      HIP_TRY(hipHostMalloc((void**)&pl->h_cancel, sizeof(int),
                            hipHostMallocMapped | hipHostMallocCoherent));
      memset(pl->h_prog, 0, sizeof(int) * C);
      *pl->h_cancel = 0;
      int *dp = nullptr, *dc = nullptr;
      HIP_TRY(hipHostGetDevicePointer((void**)&dp, pl->h_prog, 0));
      HIP_TRY(hipHostGetDevicePointer((void**)&dc, pl->h_cancel, 0));
      k.progress = dp;
      k.cancel = dc;
      return FITOCT_OK;
    };
    rc = prog_setup();
    if (rc) return rc;
  }
  // Chain migration (work balance): only when every tile of the launch is
  // co-resident (one tile per CU), so an idle tile waiting for a migrant never
  // keeps a pending tile off the chip; off in batch mode (a tile holds one
  // problem's bins) and with FITOCT_NO_MIGRATE.
  if (g_chains == 0 && k.G >= 2 && pl->tiles <= pl->ncu && getenv("FITOCT_NO_MIGRATE") == nullptr) {
    const int T = pl->tiles, words = mig_img_words(pl->ppl);
    pl->mig_bytes = sizeof(int) * (MIG_HDR + 2 * (size_t)T + (size_t)T * GMAX);
    auto mig_setup = [&]() -> int {
      HIP_TRY(hipMalloc(&pl->d_mig, pl->mig_bytes));
      HIP_TRY(hipMalloc(&pl->d_mig_img, sizeof(double) * (size_t)T * GMAX * words));
      return FITOCT_OK;
    };
    rc = mig_setup();
    if (rc) return rc;
    k.mig = pl->d_mig;
    k.mig_img = pl->d_mig_img;
    k.mig_tiles = T;
    k.mig_img_words = words;
  }
  // Speculative leaves (nuts_device.hip leaf_spec).  A tile of one (two) chain(s) always
  // speculates, with a spare NUTS wave helping each chain (config 2 +4 %).  A tile of several chains
  // has no spare wave: while it hosts 4 live chains the sweep hides the sampler's latency
  // and speculation only adds work, so a migrating chain speculates only once its tile has
  // thinned out to <= kSpecLiveMigrating chains (the launch's tail, config 3 +2 %).  Draws
  // are the same bit for bit either way.  FITOCT_SPEC_LIVE=n overrides spec_live (0: never; GMAX:
  // always), FITOCT_SPEC=1 is FITOCT_SPEC_LIVE=GMAX (tests), FITOCT_NO_SPEC=1 builds the
  // plain sampler.
  {
    // (tiles of two chains without migration -- a batch of 257..512 chains, config 5's
    // per-GPU share at 2 GPUs -- have a spare NUTS wave per chain too: deep speculation)
    int live = pl->mig_bytes > 0 ? kSpecLiveMigrating : k.G <= 2 ? 1 : 0;
    if (const char* fs = getenv("FITOCT_SPEC")) live = atoi(fs) != 0 ? GMAX : live;
    if (const char* fl = getenv("FITOCT_SPEC_LIVE")) live = atoi(fl);
    if (getenv("FITOCT_NO_SPEC") != nullptr) live = 0;
    k.spec_live = std::max(0, std::min(live, GMAX));
    k.spec = k.spec_live > 0 ? 1 : 0;
  }
  // Two-ended trajectories (nuts_device.hip): tiles of one chain grow the trajectory's two
  // ends at once -- two spare NUTS waves build the subtrees of each direction whole, each in a
  // chain area of its own, and the chain's wave books the trajectory level from one record per
  // subtree.  Same draws bit for bit.  The three chain areas must fit, else the tile stays on
  // the one-ended path (at Nn 16..24 a chain area holds two parameters per lane: three of
  // them at max_treedepth 10 take ~181 KB of the 160 KB).  FITOCT_NO_BIDI=1: off.
  k.bidi = 0;
  if (k.spec && k.G == 1 && pl->mig_bytes == 0 && getenv("FITOCT_NO_BIDI") == nullptr) {
    const int base = lds_bytes(pl->ppl, 3, k.max_depth);
    if (base <= 160 * 1024 - STATIC_LDS_RESERVE) {
      k.bidi = 1;
      pl->lds = base;
    }
  }
  // Two-ended trajectories in the tail of a migrating launch (nuts_device.hip receive_chain):
  // the producers are idle receivers of the tile (their own chain areas: no LDS added).  Same
  // draws bit for bit.  FITOCT_NO_TAIL_BIDI=1: off; FITOCT_TAIL_LEFT=n: start at n unfinished
  // chains (default: every chain of the launch -- a chain alone in its tile goes two-ended
  // whenever two receivers are idle; one per tile measured 1 % slower on config 3).
  k.tail_bidi = 0;
  if (pl->mig_bytes > 0 && k.spec && getenv("FITOCT_NO_TAIL_BIDI") == nullptr) {
    k.tail_bidi = 1;
    k.tail_left = k.chains;   // from the start (config 3: +1.0 % over one per tile, profiles/r05_ab_tail_left.txt)
    if (const char* e = getenv("FITOCT_TAIL_LEFT")) k.tail_left = std::max(0, atoi(e));
    if (const char* e = getenv("FITOCT_TEST_TAIL_IDLE_US"))   // test hook: producers give up early
      k.tail_idle_ticks = 100ULL * (unsigned long long)std::max(1, atoi(e));
  }
  // (a batch pairs its tiles itself: fitoct_batch_create)
  if (g_chains == 0 && want_pairs(k, pl->tiles, pl->ncu)) {
    rc = alloc_pairs(k, pl->tiles, pl->ppl, &pl->d_pair_hdr, &pl->d_pair_buf);
    if (rc) return rc;
  }
  *out = guard.release();
  return FITOCT_OK;
}
}  // namespace

extern "C" {

int32_t fitoct_plan_get_info(const fitoct_plan* pl, fitoct_plan_info* info) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl || !info) return fail(FITOCT_E_ARG, "NULL argument");
    if (!pl->shards.empty()) return group_plan_info(pl, info);
    info->dim = pl->kp.D;
    info->n_cols = pl->kp.ncols;
    info->iters_saved = pl->kp.iters_saved;
    info->chains = pl->kp.chains;
    info->tiles = pl->tiles;
    info->chains_per_tile = pl->kp.G;
    info->sampler = pl->mig_bytes > 0
                        ? (pl->kp.spec ? FITOCT_SAMPLER_MIGRATE_SPEC : FITOCT_SAMPLER_MIGRATE)
                    : pl->kp.spec ? FITOCT_SAMPLER_SPECULATIVE : FITOCT_SAMPLER_PLAIN;
    info->n_devices = 1;
    info->bins_per_thread = pl->bpt;
    info->threads_per_tile = TPB;
    info->lds_bytes = pl->lds;
    info->n_pad = pl->kp.n_pad;
    info->draws_bytes = (int64_t)pl->draws_bytes;
    const bool te = pl->kp.bidi || pl->kp.tail_bidi;
    info->two_ended = pl->kp.bidi ? 1 : pl->kp.tail_bidi ? 2 : 0;
    info->ring_records = te ? 1 : 0;   // (ABI 7: one subtree record per end)
    info->ring_records_in_levels = 0;
    info->paired = pl->kp.pair;
    info->workgroups = pl->grid();
    info->basis_mode = pl->kp.mode;
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_set_init(fitoct_plan* pl, const double* q_init, const double* stepsize,
                             const double* inv_metric) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl) return fail(FITOCT_E_ARG, "plan is NULL");
    if (!pl->shards.empty()) return group_plan_set_init(pl, q_init, stepsize, inv_metric);
    if (pl->launched) return fail(FITOCT_E_ARG, "plan is running: call fitoct_plan_wait first");
    const int C = pl->kp.chains, D = pl->kp.D;
    // checked on the host: the kernel takes every value as given
    const int ck = check_init(C, D, q_init, stepsize, inv_metric);
    if (ck) return ck;
    HIP_TRY(hipSetDevice(pl->cfg.device));
    if ((q_init || stepsize || inv_metric) && !pl->d_init)
      HIP_TRY(hipMalloc(&pl->d_init, sizeof(double) * (size_t)C * (1 + 2 * D)));
    double* d_eps = pl->d_init;
    double* d_minv = pl->d_init ? pl->d_init + C : nullptr;
    double* d_q = pl->d_init ? pl->d_init + C + (size_t)C * D : nullptr;
    if (stepsize) HIP_TRY(hipMemcpy(d_eps, stepsize, sizeof(double) * C, hipMemcpyHostToDevice));
    if (inv_metric)
      HIP_TRY(hipMemcpy(d_minv, inv_metric, sizeof(double) * C * D, hipMemcpyHostToDevice));
    if (q_init) HIP_TRY(hipMemcpy(d_q, q_init, sizeof(double) * C * D, hipMemcpyHostToDevice));
    pl->kp.init_eps = stepsize ? d_eps : nullptr;
    pl->kp.init_minv = inv_metric ? d_minv : nullptr;
    pl->kp.init_q = q_init ? d_q : nullptr;
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_launch(fitoct_plan* pl, void* d_draws, void* stream) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl) return fail(FITOCT_E_ARG, "plan is NULL");
    if (!pl->shards.empty()) return group_plan_launch(pl, d_draws, stream);
    if (pl->launched) return fail(FITOCT_E_ARG, "plan is running: call fitoct_plan_wait first");
    HIP_TRY(hipSetDevice(pl->cfg.device));
    if (pl->h_prog) {   // no launch of this plan is in flight: the kernel does not touch them
      memset(pl->h_prog, 0, sizeof(int) * pl->kp.chains);
      __atomic_store_n(pl->h_cancel, 0, __ATOMIC_SEQ_CST);
    }
    double* dst = (double*)d_draws;
    if (!dst) {
      if (!pl->d_draws) HIP_TRY(hipMalloc(&pl->d_draws, pl->draws_bytes));
      dst = pl->d_draws;
    }
    hipStream_t st = (hipStream_t)stream;
    KParams k = pl->kp;
    k.draws = dst;
    HIP_TRY(hipMemsetAsync(pl->d_status, 0, sizeof(int) * k.chains, st));
    HIP_TRY(hipMemsetAsync(k.bidi_count, 0, 2 * sizeof(long long), st));   // + pair_count
    if (pl->d_mig) HIP_TRY(hipMemsetAsync(pl->d_mig, 0, pl->mig_bytes, st));
    if (k.pair)   // every word the pairs poll: zero before every launch
      HIP_TRY(hipMemsetAsync(k.pair_hdr, 0, sizeof(int) * PAIR_HDR_INTS * (size_t)k.pair_tiles, st));
    const bool want_stamps = getenv("FITOCT_STAMPS") != nullptr;   // diagnostic only
    if (want_stamps) {
      if (!pl->d_stamps) HIP_TRY(hipMalloc(&pl->d_stamps, sizeof(long long) * NSTAMP * pl->tiles));
      HIP_TRY(hipMemsetAsync(pl->d_stamps, 0, sizeof(long long) * NSTAMP * pl->tiles, st));
      k.stamps = pl->d_stamps;
      k.bench_sweeps = getenv("FITOCT_BENCH_SWEEPS") ? atoi(getenv("FITOCT_BENCH_SWEEPS")) : 0;
    }
    HIP_TRY(hipEventRecord(pl->ev0, st));
    if (!pl->d_kp) HIP_TRY(hipMalloc(&pl->d_kp, sizeof(KParams)));
    HIP_TRY(hipMemcpyAsync(pl->d_kp, &k, sizeof(KParams), hipMemcpyHostToDevice, st));
    HIP_TRY(launch(false, pl->mixed, pl->bpt, pl->nnp, k, pl->d_kp, pl->grid(), st));
    HIP_TRY(hipEventRecord(pl->ev1, st));
    pl->last_draws = dst;
    pl->launched = true;
    pl->ran = false;
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_poll(fitoct_plan* pl, int64_t* iterations_done, int64_t* iterations_total,
                         int32_t* finished) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl) return fail(FITOCT_E_ARG, "plan is NULL");
    if (!pl->shards.empty()) return group_plan_poll(pl, iterations_done, iterations_total, finished);
    const int C = pl->kp.chains;
    int64_t done = 0;
    if (pl->h_prog)
      for (int c = 0; c < C; ++c) done += __atomic_load_n(&pl->h_prog[c], __ATOMIC_RELAXED);
    const int64_t total = (int64_t)C * (pl->kp.warmup + pl->kp.samples);
    int32_t fin = pl->ran ? 1 : 0;
    if (pl->launched) {
      HIP_TRY(hipSetDevice(pl->cfg.device));
      const hipError_t q = hipEventQuery(pl->ev1);
      if (q == hipSuccess) fin = 1;
      else if (q != hipErrorNotReady) HIP_TRY(q);
    }
    if (iterations_done) *iterations_done = (pl->h_prog || !fin) ? done : total;
    if (iterations_total) *iterations_total = total;
    if (finished) *finished = fin;
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_cancel(fitoct_plan* pl) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl) return fail(FITOCT_E_ARG, "plan is NULL");
    if (!pl->shards.empty()) return group_plan_cancel(pl);
    if (!pl->h_cancel) return fail(FITOCT_E_ARG, "this plan has no cancellation flag (batch plan)");
    __atomic_store_n(pl->h_cancel, 1, __ATOMIC_SEQ_CST);
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_wait(fitoct_plan* pl) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl) return fail(FITOCT_E_ARG, "plan is NULL");
    if (!pl->shards.empty()) return group_plan_wait(pl);
    if (!pl->launched) return pl->ran ? FITOCT_OK : fail(FITOCT_E_ARG, "plan has not been launched");
    HIP_TRY(hipSetDevice(pl->cfg.device));
    pl->launched = false;
    HIP_TRY(hipEventSynchronize(pl->ev1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, pl->ev0, pl->ev1));
    pl->kernel_ms = ms;
    if (pl->d_stamps && getenv("FITOCT_STAMPS") != nullptr) {
      std::vector<long long> h((size_t)NSTAMP * pl->tiles);
      HIP_TRY(hipMemcpy(h.data(), pl->d_stamps, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
      double steps = 0, tg = 0, tn = 0, tt = 0, smax = 0, tw = 0, nw = 0, tsw = 0, tno = 0;
      double ts0 = 0, ts1 = 0;
      double act_t[18] = {0}, act_n[18] = {0};
      for (int t = 0; t < pl->tiles; ++t) {
        const long long* o = h.data() + (size_t)NSTAMP * t;
        steps += o[0];
        tg += o[1];
        tn += o[2];
        tt += o[3];
        tw += o[40];
        nw += o[41];
        tsw += o[42];
        tno += o[43];
        ts0 += o[44];
        ts1 += o[45];
        smax = std::max(smax, (double)o[0]);
        for (int a = 0; a < 18; ++a) {
          act_t[a] += o[4 + a];
          act_n[a] += o[22 + a];
        }
      }
      double subt[12] = {0}, wb[8] = {0};
      for (int t = 0; t < pl->tiles; ++t) {
        for (int k = 0; k < 8; ++k) subt[k] += h[(size_t)NSTAMP * t + 48 + k];
        for (int k = 0; k < 4; ++k) subt[8 + k] += h[(size_t)NSTAMP * t + 68 + k];
        for (int k = 0; k < 8; ++k) wb[k] += h[(size_t)NSTAMP * t + 56 + k];
      }
      fprintf(stderr, "[fitoct stamps] gradient-wave busy per sweep by wave:");
      for (int k = 0; k < 8; ++k) fprintf(stderr, " %.0f", wb[k] / std::max(steps, 1.0));
      fprintf(stderr, "\n");
      // per gradient of chain 0 (act_n[1]: A_GRAD runs); a11 is the speculative path's
      // separate bookkeeping action (A_SPEC_BOOK)
      fprintf(stderr, "[fitoct stamps] sub-action cycles per gradient (chain 0): ");
      for (int k = 0; k < 12; ++k)
        if (subt[k] > 0) fprintf(stderr, "s%d:%.0f ", k, subt[k] / std::max(act_n[1], 1.0));
      fprintf(stderr, "\n");
      fprintf(stderr, "[fitoct stamps] per action (chain 0 of each tile): ");
      for (int a = 1; a < 18; ++a)
        if (act_n[a] > 0) fprintf(stderr, "a%d:%.0fx%.0f ", a, act_n[a] / pl->tiles, act_t[a] / act_n[a]);
      fprintf(stderr, "\n");
      fprintf(stderr,
              "[fitoct stamps] tiles=%d mean sweeps/tile=%.0f max=%.0f | per sweep: grad-wave busy %.0f "
              "nuts-wave busy %.0f wall %.0f memtime ticks\n",
              pl->tiles, steps / pl->tiles, smax, tg / steps, tn / steps, tt / steps);
      fprintf(stderr,
              "[fitoct stamps] chain 0 per NUTS round: busy %.0f, waiting for its gradient %.0f "
              "(enqueue->sweep done %.0f, sweep done->resumed %.0f)\n",
              tn / std::max(nw, 1.0), tw / std::max(nw, 1.0), tsw / std::max(nw, 1.0),
              tno / std::max(nw, 1.0));
      fprintf(stderr, "[fitoct stamps] enqueue -> first wave starts %.0f, last wave starts %.0f\n",
              ts0 / std::max(nw, 1.0), ts1 / std::max(nw, 1.0));
      // tile timeline on the 100 MHz clock: how much of the launch the tiles sit idle at
      // the end (the kernel ends with its last tile)
      {
        long long t0 = LLONG_MAX, t1 = 0;
        std::vector<double> ends, firsts;
        for (int t = 0; t < pl->tiles; ++t) {
          const long long* o = h.data() + (size_t)NSTAMP * t;
          t0 = std::min(t0, o[64]);
          t1 = std::max(t1, o[65]);
        }
        const double span = std::max(1.0, (double)(t1 - t0));
        double done_sum = 0;
        for (int t = 0; t < pl->tiles; ++t) {
          const long long* o = h.data() + (size_t)NSTAMP * t;
          ends.push_back((o[65] - t0) / span);
          if (o[66] > 0) firsts.push_back((o[66] - t0) / span);
          done_sum += o[67];
        }
        std::sort(ends.begin(), ends.end());
        std::sort(firsts.begin(), firsts.end());
        auto q = [](const std::vector<double>& v, double f) {
          return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(f * (v.size() - 1)))];
        };
        double mean_end = 0;
        for (double e : ends) mean_end += e;
        mean_end /= std::max<size_t>(1, ends.size());
        fprintf(stderr,
                "[fitoct stamps] tile ends (fraction of the launch): mean %.3f p10 %.3f p50 %.3f "
                "p90 %.3f | first chain done in a tile: p10 %.3f p50 %.3f p90 %.3f | chains "
                "finished %.0f, launch %.1f ms\n",
                mean_end, q(ends, 0.1), q(ends, 0.5), q(ends, 0.9), q(firsts, 0.1), q(firsts, 0.5),
                q(firsts, 0.9), done_sum, span / 1e5);
        // tile occupancy: share of all tiles' time, and of all sweeps, spent while a tile
        // hosted k live chains (k = 0..4; the launch's tail runs thinned-out tiles)
        double ot[5] = {0}, on[5] = {0}, st = 0, sn = 0;
        for (int t = 0; t < pl->tiles; ++t)
          for (int k = 0; k < 5; ++k) {
            ot[k] += h[(size_t)NSTAMP * t + 72 + k];
            on[k] += h[(size_t)NSTAMP * t + 77 + k];
          }
        for (int k = 0; k < 5; ++k) {
          st += ot[k];
          sn += on[k];
        }
        fprintf(stderr, "[fitoct stamps] tile occupancy (live chains k: share of tile time / of sweeps):");
        for (int k = 0; k < 5; ++k)
          fprintf(stderr, " k=%d %.4f/%.4f", k, ot[k] / std::max(st, 1.0), on[k] / std::max(sn, 1.0));
        fprintf(stderr, "\n");
      }
      if (pl->kp.bidi) {   // two-ended roles (tiles of one chain; paired: the forward end's
                           // producer runs in the partner tile)
        double hb = 0, hw = 0, hn = 0, hi = 0, pe[2][4] = {{0}};
        for (int t = 0; t < pl->tiles; ++t) {
          const long long* o = h.data() + (size_t)NSTAMP * t;
          hb += o[84];
          hw += o[85];
          hn += o[86];
          hi += o[87];
          for (int s = 0; s < 2; ++s)
            for (int k = 0; k < 4; ++k) pe[s][k] += o[88 + 4 * s + k];
        }
        fprintf(stderr,
                "[fitoct stamps] booking wave per booked leaf: busy %.0f, waiting for its record %.0f "
                "(leaves booked per tile %.0f, idle between trees %.0f per tile)\n",
                hb / std::max(hn, 1.0), hw / std::max(hn, 1.0), hn / pl->tiles, hi / pl->tiles);
        for (int s = 0; s < 2; ++s)
          fprintf(stderr,
                  "[fitoct stamps] producer of end %d per produced leaf: waiting for its sweep %.0f, "
                  "for lookahead / record slot %.0f, in trees %.0f (leaves per tile %.0f)\n",
                  s, pe[s][0] / std::max(pe[s][2], 1.0), pe[s][1] / std::max(pe[s][2], 1.0),
                  pe[s][3] / std::max(pe[s][2], 1.0), pe[s][2] / pl->tiles);
        for (int s = 0; s < 2; ++s) {
          double q[4] = {0, 0, 0, 0}, n = 0;
          for (int t = 0; t < pl->tiles; ++t) {
            for (int k = 0; k < 4; ++k) q[k] += h[(size_t)NSTAMP * t + 100 + 4 * s + k];
            n += h[(size_t)NSTAMP * t + 90 + 4 * s];
          }
          fprintf(stderr,
                  "[fitoct stamps] producer of end %d per leaf (helped): finish_grad %.0f, stage %.0f, "
                  "hand-over %.0f, prior_part %.0f\n", s, q[0] / std::max(n, 1.0),
                  q[1] / std::max(n, 1.0), q[2] / std::max(n, 1.0), q[3] / std::max(n, 1.0));
        }
        double hb2[2] = {0, 0}, hn2[2] = {0, 0};
        for (int t = 0; t < pl->tiles; ++t)
          for (int r = 0; r < 2; ++r) {
            hb2[r] += h[(size_t)NSTAMP * t + 96 + 2 * r];
            hn2[r] += h[(size_t)NSTAMP * t + 97 + 2 * r];
          }
        for (int r = 0; r < 2; ++r)
          if (hn2[r] > 0)
            fprintf(stderr,
                    "[fitoct stamps] booking helper (%s tile): %.0f cycles per booked leaf, %.0f "
                    "leaves per tile\n", r ? "partner" : "primary", hb2[r] / hn2[r], hn2[r] / pl->tiles);
      }
    }
    pl->ran = true;
    return FITOCT_OK;
  });
}

int32_t fitoct_plan_run(fitoct_plan* pl, void* d_draws, void* stream) {
  return guarded(__func__, [&]() -> int32_t {
    const int32_t rc = fitoct_plan_launch(pl, d_draws, stream);
    return rc ? rc : fitoct_plan_wait(pl);
  });
}


int32_t fitoct_plan_download(fitoct_plan* pl, fitoct_result* res) {
  return guarded(__func__, [&]() -> int32_t {
    if (!pl || !res) return fail(FITOCT_E_ARG, "NULL argument");
    if (!pl->shards.empty()) return group_plan_download(pl, res);
    if (!pl->ran) return fail(FITOCT_E_ARG, "plan has not run");
    HIP_TRY(hipSetDevice(pl->cfg.device));
    const KParams& k = pl->kp;
    const int C = k.chains, D = k.D;
    res->n_cols = k.ncols;
    res->iters_saved = k.iters_saved;
    res->dim = D;
    res->kernel_ms = pl->kernel_ms;
    res->migrations = 0;
    if (pl->d_mig) HIP_TRY(hipMemcpy(&res->migrations, pl->d_mig + MIG_MOVES, sizeof(int),
                                     hipMemcpyDeviceToHost));
    if (res->draws) {
      const int64_t need = (int64_t)C * k.iters_saved * k.ncols;
      if (res->draws_capacity < need) return fail(FITOCT_E_ARG, "draws buffer too small");
      HIP_TRY(hipMemcpy(res->draws, pl->last_draws, pl->draws_bytes, hipMemcpyDeviceToHost));
    }
    if (res->stepsize) HIP_TRY(hipMemcpy(res->stepsize, k.fin_eps, sizeof(double) * C, hipMemcpyDeviceToHost));
    if (res->inv_metric)
      HIP_TRY(hipMemcpy(res->inv_metric, k.fin_minv, sizeof(double) * C * D, hipMemcpyDeviceToHost));
    if (res->last_q) HIP_TRY(hipMemcpy(res->last_q, k.fin_q, sizeof(double) * C * D, hipMemcpyDeviceToHost));
    std::vector<int> st(C);
    HIP_TRY(hipMemcpy(st.data(), k.chain_status, sizeof(int) * C, hipMemcpyDeviceToHost));
    if (res->chain_status) memcpy(res->chain_status, st.data(), sizeof(int) * C);
    const int bad = chain_outcome(C, D, st.data(), res->stepsize, res->inv_metric, res->last_q);
    std::vector<long long> lf(C);
    HIP_TRY(hipMemcpy(lf.data(), k.leapfrogs, sizeof(long long) * C, hipMemcpyDeviceToHost));
    long long tot = 0;
    for (long long v : lf) tot += v;
    res->total_leapfrogs = tot;
    long long nb = 0;
    HIP_TRY(hipMemcpy(&nb, k.bidi_count, sizeof(long long), hipMemcpyDeviceToHost));
    res->two_ended_transitions = nb;
    HIP_TRY(hipMemcpy(&nb, k.pair_count, sizeof(long long), hipMemcpyDeviceToHost));
    res->paired_transitions = nb;
    if (bad >= 0)
      return fail(st[bad], "chain " + std::to_string(k.chain_offset + bad) + " failed with status " +
                               std::to_string(st[bad]));
    return FITOCT_OK;
  });
}

void fitoct_plan_destroy(fitoct_plan* pl) { free_plan(pl); }

int32_t fitoct_expgp_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res) {
  return guarded(__func__, [&]() -> int32_t {
    const auto t0 = std::chrono::steady_clock::now();
    if (cfg && cfg->chains >= 1) {   // several devices: one host thread per device
      std::vector<int> devs;
      const int rd = resolve_devices(cfg, cfg->chains, devs);
      if (rd) return rd;
      if (devs.size() > 1) {
        const int rg = group_sample(prob, cfg, devs, res);
        if (res)
          res->wall_ms = std::chrono::duration<double, std::milli>(
                             std::chrono::steady_clock::now() - t0).count();
        return rg;
      }
    }
    fitoct_plan* pl = nullptr;
    int rc = fitoct_plan_create(prob, cfg, &pl);
    if (rc) return rc;
    rc = fitoct_plan_run(pl, nullptr, nullptr);
    if (!rc && res) rc = fitoct_plan_download(pl, res);
    free_plan(pl);
    if (res)
      res->wall_ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
  });
}

int32_t fitoct_split_rhat_ess(const double* x, int32_t chains, int32_t n, double* rhat,
                              double* ess) {
  return guarded(__func__, [&]() -> int32_t {
    if (!x) return fail(FITOCT_E_ARG, "x is NULL");
    return split_rhat_ess(x, chains, n, rhat, ess);
  });
}

int32_t fitoct_rank_rhat(const double* x, int32_t chains, int32_t n, double* rhat) {
  return guarded(__func__, [&]() -> int32_t {
    if (!x || !rhat) return fail(FITOCT_E_ARG, "NULL argument");
    return rank_rhat(x, chains, n, rhat);
  });
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Batch mode: many problems (FitOCT.R's per-file fitExpGP calls, FitOCT.R:70-124)
// sampled by ONE persistent launch.  Each problem keeps its own staged data,
// basis factors, pool and outputs (a fitoct_plan each); the kernel receives the
// array of their parameter blocks and a tile map {problem, first chain}, so a
// tile only ever holds one problem's chains.  Chain c of problem p is keyed as
// global chain cfg.chain_offset + p*chains + c: its draws are those of a single
// plan of that problem with chain_offset = cfg.chain_offset + p*chains.
// ---------------------------------------------------------------------------

namespace {
void free_batch(fitoct_batch* b) {
  if (!b) return;
  if (b->h_cancel) (void)hipHostFree(b->h_cancel);
  for (fitoct_batch* sb : b->subs) free_batch(sb);
  for (fitoct_plan* pl : b->plans) free_plan(pl);
  (void)hipFree(b->d_kp);
  (void)hipFree(b->d_map);
  (void)hipFree(b->d_pair_hdr);
  (void)hipFree(b->d_pair_buf);
  (void)hipFree(b->d_draws);
  if (b->ev0) (void)hipEventDestroy(b->ev0);
  if (b->ev1) (void)hipEventDestroy(b->ev1);
  if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
  delete b;
}
}  // namespace

extern "C" {

int32_t fitoct_batch_create(const fitoct_problem* probs, int32_t n_problems,
                            const fitoct_config* cfg, fitoct_batch** out) {
  return guarded(__func__, [&]() -> int32_t {
    if (!out) return fail(FITOCT_E_ARG, "out is NULL");
    *out = nullptr;
    if (!probs || n_problems < 1) return fail(FITOCT_E_ARG, "need n_problems >= 1 problems");
    if (!cfg) return fail(FITOCT_E_ARG, "config is NULL");
    if (cfg->chains < 1) return fail(FITOCT_E_ARG, "chains must be >= 1");
    if ((int64_t)n_problems * cfg->chains > (int64_t)1 << 30)
      return fail(FITOCT_E_ARG, "too many chains in one batch");
    std::vector<int> devs;
    {
      const int rd = resolve_devices(cfg, n_problems, devs);
      if (rd) return rd;
    }
    if (devs.size() > 1) return group_batch_create(probs, n_problems, cfg, devs, out);
    std::unique_ptr<fitoct_batch, void (*)(fitoct_batch*)> guard(new fitoct_batch(), free_batch);
    fitoct_batch* b = guard.get();
    b->cfg = *cfg;
    b->cfg.device = devs[0];
    b->cfg.n_devices = 0;
    b->n_problems = n_problems;
    const int C = cfg->chains;
    // one basis mode for the whole batch: resident rows only if every problem has N <= 512
    bool poly_only = false;
    for (int p = 0; p < n_problems; ++p) poly_only = poly_only || probs[p].N > 2 * GT;
    auto build = [&]() -> int {
      for (int p = 0; p < n_problems; ++p) {
        if (probs[p].prior_type != probs[0].prior_type || probs[p].Nn != probs[0].Nn)
          return fail(FITOCT_E_ARG, "batch problems must share prior_type and Nn (problem " +
                                        std::to_string(p) + ")");
        fitoct_config c = b->cfg;
        c.chain_offset = cfg->chain_offset + p * C;
        fitoct_plan* pl = nullptr;
        const int rc = plan_create(&probs[p], &c, n_problems * C, -1, &pl, poly_only);
        if (rc) return fail(rc, "problem " + std::to_string(p) + ": " + fitoct_last_error());
        b->plans.push_back(pl);
      }
      // one kernel instantiation and one LDS carve must serve every problem
      int bpt = 0;
      for (fitoct_plan* pl : b->plans) bpt = std::max(bpt, pl->bpt == 0 ? 1 << 20 : pl->bpt);
      const fitoct_plan* p0 = b->plans[0];
      for (fitoct_plan* pl : b->plans) {
        if (pl->kp.mode != p0->kp.mode || pl->nnp != p0->nnp || pl->ppl != p0->ppl ||
            pl->mixed != p0->mixed || pl->kp.G != p0->kp.G)
          return fail(FITOCT_E_ARG, "batch problems plan to different kernels (basis mode)");
      }
      // bins: every tile runs the batch's widest bin layout.  A problem planned with
      // fewer bins per lane is restaged at the common n_pad (zero-weight padding).
      if (bpt == 1 << 20) bpt = 0;
      auto restage = [&](int to) -> int {
        for (size_t p = 0; p < b->plans.size(); ++p) {
          fitoct_plan* pl = b->plans[p];
          if (pl && pl->bpt == to) continue;
          fitoct_config c = b->cfg;
          c.chain_offset = cfg->chain_offset + (int)p * C;
          free_plan(pl);
          b->plans[p] = nullptr;
          const int rc = plan_create(&probs[p], &c, n_problems * C, to, &b->plans[p], poly_only);
          if (rc) return rc;
        }
        return FITOCT_OK;
      };
      int rc = restage(bpt);
      // the 16-bin layout needs an arithmetic depth grid in every problem: else stream all
      if (rc && bpt == 16) rc = restage(0);
      if (rc) return rc;
      b->per_bytes = b->plans[0]->draws_bytes;
      std::vector<int> map;
      const int G = b->plans[0]->kp.G;
      for (int p = 0; p < n_problems; ++p)
        for (int c0 = 0; c0 < C; c0 += G) {
          map.push_back(p);
          map.push_back(c0);
        }
      b->tiles = (int)map.size() / 2;
      HIP_TRY(hipSetDevice(b->cfg.device));
      HIP_TRY(hipMalloc(&b->d_map, sizeof(int) * map.size()));
      HIP_TRY(hipMemcpy(b->d_map, map.data(), sizeof(int) * map.size(), hipMemcpyHostToDevice));
      HIP_TRY(hipMalloc(&b->d_kp, sizeof(KParams) * n_problems));
      // paired tiles over the whole batch (one-chain tiles: config 5's 4- and 8-GPU shares)
      {
        KParams kq = b->plans[0]->kp;
        if (want_pairs(kq, b->tiles, b->plans[0]->ncu)) {
          const int rc2 = alloc_pairs(kq, b->tiles, b->plans[0]->ppl, &b->d_pair_hdr, &b->d_pair_buf);
          if (rc2) return rc2;
          b->pair_stride = kq.pair_stride;
        }
      }
      // cancellation flag (set by the multi-device layer when another device fails)
      HIP_TRY(hipHostMalloc((void**)&b->h_cancel, sizeof(int),
                            hipHostMallocMapped | hipHostMallocCoherent));
      *b->h_cancel = 0;
      HIP_TRY(hipHostGetDevicePointer((void**)&b->d_cancel, b->h_cancel, 0));
      HIP_TRY(hipEventCreate(&b->ev0));
      HIP_TRY(hipEventCreate(&b->ev1));
      return FITOCT_OK;
    };
    const int rc = build();
    if (rc) return rc;
    *out = guard.release();
    return FITOCT_OK;
  });
}

int32_t fitoct_batch_get_info(const fitoct_batch* b, fitoct_plan_info* info) {
  return guarded(__func__, [&]() -> int32_t {
    if (!b || !info) return fail(FITOCT_E_ARG, "NULL argument");
    if (!b->subs.empty()) return group_batch_info(b, info);
    const int rc = fitoct_plan_get_info(b->plans[0], info);
    if (rc) return rc;
    info->chains = b->cfg.chains * (int)b->plans.size();
    info->tiles = b->tiles;
    info->paired = b->d_pair_hdr ? 1 : 0;
    info->workgroups = b->d_pair_hdr ? pair_grid(b->tiles) : b->tiles;
    info->basis_mode = b->plans.empty() ? 0 : b->plans[0]->kp.mode;
    info->draws_bytes = (int64_t)(b->per_bytes * b->plans.size());
    return FITOCT_OK;
  });
}

}  // extern "C"

int fitoct::batch_run_single(fitoct_batch* b, void* d_draws, void* stream) {
    HIP_TRY(hipSetDevice(b->cfg.device));
    const size_t P = b->plans.size();
    double* dst = (double*)d_draws;
    if (!dst) {
      if (!b->d_draws) HIP_TRY(hipMalloc(&b->d_draws, b->per_bytes * P));
      dst = b->d_draws;
    }
    hipStream_t st = (hipStream_t)stream;
    std::vector<KParams> kp(P);
    for (size_t p = 0; p < P; ++p) {
      fitoct_plan* pl = b->plans[p];
      kp[p] = pl->kp;
      kp[p].draws = (double*)((char*)dst + b->per_bytes * p);
      kp[p].cancel = b->d_cancel;
      pl->last_draws = kp[p].draws;
      HIP_TRY(hipMemsetAsync(pl->d_status, 0, sizeof(int) * pl->kp.chains, st));
      HIP_TRY(hipMemsetAsync(pl->kp.bidi_count, 0, 2 * sizeof(long long), st));   // + pair_count
      if (b->d_pair_hdr) {   // paired tiles: every problem's block names the batch's pairs
        kp[p].pair = 1;
        kp[p].pair_tiles = b->tiles;
        kp[p].pair_stride = b->pair_stride;
        kp[p].pair_hdr = b->d_pair_hdr;
        kp[p].pair_buf = b->d_pair_buf;
        const char* t = getenv("FITOCT_TEST_PAIR_ABSENT");
        kp[p].pair_test_absent = (t && atoi(t) != 0) ? 1 : 0;
      }
    }
    if (b->d_pair_hdr)
      HIP_TRY(hipMemsetAsync(b->d_pair_hdr, 0, sizeof(int) * PAIR_HDR_INTS * (size_t)b->tiles, st));
    HIP_TRY(hipMemcpyAsync(b->d_kp, kp.data(), sizeof(KParams) * P, hipMemcpyHostToDevice, st));
    const fitoct_plan* p0 = b->plans[0];
    HIP_TRY(hipEventRecord(b->ev0, st));
    HIP_TRY(launch(false, p0->mixed, p0->bpt, p0->nnp, kp[0], b->d_kp,
                   b->d_pair_hdr ? pair_grid(b->tiles) : b->tiles, st, b->d_map));
    HIP_TRY(hipEventRecord(b->ev1, st));
    HIP_TRY(hipEventSynchronize(b->ev1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, b->ev0, b->ev1));
    b->kernel_ms = ms;
    for (fitoct_plan* pl : b->plans) {
      pl->kernel_ms = ms;
      pl->ran = true;
    }
    b->ran = true;
    return FITOCT_OK;
}

extern "C" {

int32_t fitoct_batch_run(fitoct_batch* b, void* d_draws, void* stream) {
  return guarded(__func__, [&]() -> int32_t {
    if (!b) return fail(FITOCT_E_ARG, "batch is NULL");
    if (!b->subs.empty()) return group_batch_run(b, d_draws, stream);
    if (b->h_cancel) __atomic_store_n(b->h_cancel, 0, __ATOMIC_SEQ_CST);
    return batch_run_single(b, d_draws, stream);
  });
}

int32_t fitoct_batch_download(fitoct_batch* b, int32_t problem, fitoct_result* res) {
  return guarded(__func__, [&]() -> int32_t {
    if (!b) return fail(FITOCT_E_ARG, "batch is NULL");
    if (problem < 0 || problem >= b->n_problems)
      return fail(FITOCT_E_ARG, "problem index out of range");
    if (!b->subs.empty()) return group_batch_download(b, problem, res);
    if (!b->ran) return fail(FITOCT_E_ARG, "batch has not run");
    return fitoct_plan_download(b->plans[problem], res);
  });
}

void fitoct_batch_destroy(fitoct_batch* b) { free_batch(b); }

}  // extern "C"
