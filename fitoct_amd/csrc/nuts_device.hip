// Device-resident NUTS for the FitOCT ExpGP posterior (gfx950 / MI355X).
//
// Replaces rstan::sampling + Stan's base_nuts / adapt_diag_e_nuts + the
// stanc-generated model with stan-math AD.
//
// Execution model ("tile" = one 512-thread workgroup, persistent for the whole run):
//   * a tile owns G <= 8 chains that advance in LOCK-STEP, one leapfrog per
//     chain per tile step.  Each chain is an explicit state machine (init ->
//     step-size search -> tree building -> adaptation -> next transition), so a
//     chain that finishes its trajectory simply starts its next transition on
//     the next step: no chain ever waits for another chain's tree.
//   * gradient phase (all 16 waves): the N depth bins are strided over the
//     1024 lanes; each lane keeps its bins' data resident in VGPRs for the
//     whole run (read from HBM once per tile, shared by all G chains).  For the
//     built-in uniform-grid SE basis (MODE_POLY) the GP basis factorises as
//     K(x~_i, g_l) = a_i t_i^l b_l, so a bin needs 5 registers (c*x, y, 1/uy,
//     t, a) instead of a 16-wide basis row: dL_i = a_i P(t_i) by Horner on the
//     chain's coefficients c = b .* K^-1 yGP, and B^T h = K^-1 (b .* M) from
//     the moments M_l = sum_i h_i a_i t_i^l.  A user-supplied basis keeps its
//     rows in registers (MODE_BREG, fp32) or streams them (MODE_STREAM).
//     Per chain a lane accumulates 4+NNP partial sums, a 64-lane transposed
//     butterfly reduces them, and 16 per-wave partials land in LDS.
//   * NUTS phase (wave c drives chain c): lane k holds parameter k.  The wave
//     sums the 16 partials, completes lp / grad with the priors and the
//     log-Jacobians, and advances the chain's state machine; Stan's recursive
//     build_tree is replayed iteratively, one leaf per step, with a per-level
//     stack (p_beg, p_end, rho, proposal q/p/g) kept in HBM (L2-resident).
//   * two workgroup barriers per step; no inter-workgroup communication at all.
//
// Random numbers are addressable Philox draws (philox.h), identical to the CPU
// oracle's, so short horizons of GPU and CPU chains coincide draw for draw.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "kernel_params.h"
#include "philox.h"

namespace fitoct {

enum { FAM_NORMAL = 0, FAM_LASSO = 1, FAM_HORSESHOE = 2 };
enum { ERR_INIT = -4, ERR_NUMERIC = -5 };

// vectors kept in LDS per chain (lane-private elements)
enum VecId : int {
  V_CUR_Q, V_CUR_P, V_CUR_G,
  V_E0_Q, V_E0_P, V_E0_G,      // backward end of the trajectory
  V_E1_Q, V_E1_P, V_E1_G,      // forward end
  V_SMP_Q, V_SMP_P, V_SMP_G,   // z_sample
  V_MINV, V_WF_M, V_WF_M2,     // metric + Welford
  V_RHO, V_PNEAR,              // trajectory momentum sum, near end of old trajectory
  NVEC
};
// global stack vectors per tree level
enum StkId : int { K_PBEG = 0, K_PEND = 1, K_RHO = 2, K_PQ = 3, K_PP = 4, K_PG = 5 };

struct ChainScalars {
  int state, t, depth, leaf, dir, n_leapfrog, divergent, init_attempt;
  int da_counter, win_counter, win_size, win_next, wf_n, ss_trial, ss_dir, ss_window;
  int status, win_on, init_buf, term_buf;
  int pad0, pad1, pad2, pad3;
  double H0, lsw, sum_metro, eps, eps_used, mu, s_bar, x_bar, ss_H0;
  double cur_lp, cur_s2, smp_lp, smp_s2;
  double end_lp[2], end_s2[2];
  double st_lsw[MAXDEPTH], st_lp[MAXDEPTH], st_s2[MAXDEPTH];
  long long leapfrogs;
};
static_assert(sizeof(ChainScalars) % 16 == 0, "LDS carve alignment");

__device__ __forceinline__ void wave_fence() {
  // orders this wave's LDS traffic: every earlier ds_* op has completed and the
  // compiler may not move memory accesses across this point.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ double wave_sum(double x) {
  // butterfly: every lane ends with the bitwise-identical sum (a+b == b+a)
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

__device__ __forceinline__ void wave_sum2(double& a, double& b) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    a += __shfl_xor(a, m);
    b += __shfl_xor(b, m);
  }
}

__device__ __forceinline__ double lse(double a, double b) {
  // log_sum_exp with -inf handling (stan::math::log_sum_exp)
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const double m = a > b ? a : b;
  return m + log1p(exp(-fabs(a - b)));
}

__device__ __forceinline__ void normal_pair(RngKey k, uint32_t c0, uint32_t c1, uint32_t c2,
                                            uint32_t c3, double& n0, double& n1) {
  U4 c = {c0, c1, c2, c3};
  U4 r = philox4x32_10(c, k.k0, k.k1);
  const double u1 = u53(r.x, r.y), u2 = u53(r.z, r.w);
  const double rad = sqrt(-2.0 * log(1.0 - u1));
  const double ang = 6.283185307179586 * u2;
  n0 = rad * cos(ang);
  n1 = rad * sin(ang);
}

// ---------------------------------------------------------------------------
// per-bin arithmetic (the likelihood sweep)
// ---------------------------------------------------------------------------
template <class R> __device__ __forceinline__ R rcp_(R x);
template <> __device__ __forceinline__ double rcp_<double>(double x) {
  double r = __builtin_amdgcn_rcp(x);          // ~2^-26 seed
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  r = fma(r, e, r);                             // two Newton steps: <= 1 ulp
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
template <> __device__ __forceinline__ float rcp_<float>(float x) {
  return __builtin_amdgcn_rcpf(x);
}
template <class R> __device__ __forceinline__ R exp_(R x);
template <> __device__ __forceinline__ double exp_<double>(double x) { return exp(x); }
template <> __device__ __forceinline__ float exp_<float>(float x) { return __expf(x); }

// Likelihood terms of one bin given its modulation dL (shared by every mode).
// acc: [0] sum d^2, [1] sum a, [2] sum a e, [3] sum w; returns h (adjoint seed of dL).
template <class R>
__device__ __forceinline__ R bin_core(R dL, R cx, R y, R isu, R th1, R th2, R th3,
                                      double (&acc)[NSLOT]) {
  const R u = R(1) + dL;
  const R L = th3 * u;                                           // decay length theta3*(1+dL)
  const R iL = rcp_<R>(L);
  const R e = exp_<R>(-cx * iL);                                 // exp(-c x / L)
  const R m = fma(th2, e, th1);                                  // ui.R:88
  const R d = (y - m) * isu;                                     // (y-m)/uy
  const R a = d * isu;                                           // dlp/dm * sigma^2
  const R ae = a * e;
  const R w = ae * cx * iL;
  acc[0] += (double)(d * d);
  acc[1] += (double)a;
  acc[2] += (double)ae;
  acc[3] += (double)w;
  if (!(u > R(0))) acc[0] = INFINITY;                            // non-physical decay length
  return w * iL;                                                 // dlp/ddL / (th2 th3) * sigma^2
}

// MODE_POLY: dL = a P(t) with P = sum_l c_l t^l ; moments M_l += h a t^l
template <class R, int NNP>
__device__ __forceinline__ void bin_poly(R cx, R y, R isu, R t, R av, R th1, R th2, R th3,
                                         const R (&cf)[NNP], double (&acc)[NSLOT]) {
  R P = cf[NNP - 1];
#pragma unroll
  for (int k = NNP - 2; k >= 0; --k) P = fma(P, t, cf[k]);
  const R h = bin_core<R>(av * P, cx, y, isu, th1, th2, th3, acc);
  R p = h * av;
  acc[4] += (double)p;
#pragma unroll
  for (int l = 1; l < NNP; ++l) {
    p *= t;
    acc[4 + l] += (double)p;
  }
}

// MODE_BREG / MODE_STREAM: dL = B_i . yGP ; (B^T h)_k += B_ik h
template <class R, int NNP>
__device__ __forceinline__ void bin_rows(R cx, R y, R isu, const R (&Brow)[NNP], R th1, R th2,
                                         R th3, const R (&yg)[NNP], double (&acc)[NSLOT]) {
  R dL = R(0);
#pragma unroll
  for (int k = 0; k < NNP; ++k) dL = fma(Brow[k], yg[k], dL);
  const R h = bin_core<R>(dL, cx, y, isu, th1, th2, th3, acc);
#pragma unroll
  for (int k = 0; k < NNP; ++k) acc[4 + k] += (double)(Brow[k] * h);
}

// One exchange step of the transposed butterfly: lanes with `MASK` set keep the
// upper half of their H live values, send the lower half, and vice versa.
template <int H, int MASK>
__device__ __forceinline__ void tr_step(double (&v)[NSLOT], bool up) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const double send = up ? v[i] : v[i + H];
    const double keep = up ? v[i + H] : v[i];
    v[i] = keep + __shfl_xor(send, MASK);
  }
}
// 32 values x 64 lanes -> lane l holds the full sum of value (l >> 1).
__device__ __forceinline__ double transpose_reduce32(double (&v)[NSLOT], int lane) {
  tr_step<16, 32>(v, (lane & 32) != 0);
  tr_step<8, 16>(v, (lane & 16) != 0);
  tr_step<4, 8>(v, (lane & 8) != 0);
  tr_step<2, 4>(v, (lane & 4) != 0);
  tr_step<1, 2>(v, (lane & 2) != 0);
  return v[0] + __shfl_xor(v[0], 1);
}

// per-lane resident bin data
template <class R, int BPT, int NNP, int MODE>
struct Bins {
  static constexpr int NB = BPT > 0 ? BPT : 1;
  static constexpr int NR = MODE == MODE_POLY ? 2 : (MODE == MODE_BREG ? NNP : 1);
  R cx[NB], y[NB], isu[NB];
  R row[NB][NR];
  __device__ void load(const KParams& P, int tid) {
    if constexpr (MODE != MODE_STREAM) {
      const R* pcx = (const R*)P.cx;
      const R* py = (const R*)P.y;
      const R* pisu = (const R*)P.isu;
      const R* pB = (const R*)P.B;
#pragma unroll
      for (int b = 0; b < BPT; ++b) {
        const int i = tid + b * TPB;
        cx[b] = pcx[i];
        y[b] = py[i];
        isu[b] = pisu[i];
#pragma unroll
        for (int k = 0; k < NR; ++k) row[b][k] = pB[(size_t)i * NR + k];
      }
    }
  }
};

// LDS carve -----------------------------------------------------------------
template <int PPL>
struct Lds {
  static constexpr int VLEN = WAVE * PPL;
  static constexpr int CHAIN_BYTES =
      (int)sizeof(ChainScalars) + (NVEC + 1) * VLEN * 8 + NSLOT * 8;
  static constexpr int KBYTES = (KMAX * KMAX + KMAX) * 8;
  static __host__ __device__ constexpr int head_bytes(int G) {
    return KBYTES + (GMAX * MPW + NW * G * NSLOT) * 8;
  }
  static __host__ __device__ constexpr int bytes(int G) { return head_bytes(G) + G * CHAIN_BYTES; }
  char* base;
  int G;
  __device__ double* kinv() const { return (double*)base; }               // [Nn][Nn]
  __device__ double* bv() const { return (double*)base + KMAX * KMAX; }   // [Nn]
  __device__ double* mp(int c) const { return (double*)(base + KBYTES) + c * MPW; }
  __device__ double* part() const { return (double*)(base + KBYTES) + GMAX * MPW; }
  __device__ char* chain(int c) const { return base + head_bytes(G) + c * CHAIN_BYTES; }
  __device__ ChainScalars& cs(int c) const { return *(ChainScalars*)chain(c); }
  __device__ double* vecs(int c) const { return (double*)(chain(c) + sizeof(ChainScalars)); }
  __device__ double* qs(int c) const { return vecs(c) + NVEC * VLEN; }
  __device__ double* sums(int c) const { return qs(c) + VLEN; }
};

template <class R, int BPT, int NNP, int MODE>
__device__ void gradient_pass(const KParams& P, const Bins<R, BPT, NNP, MODE>& bins,
                              const double* mpall, double* part, const int* act, int nct,
                              int tid, int lane, int wave) {
  for (int c = 0; c < nct; ++c) {
    if (!act[c]) continue;   // wave-uniform (LDS broadcast)
    const double* mp = mpall + c * MPW;
    const R th1 = (R)mp[0], th2 = (R)mp[1], th3 = (R)mp[2];
    R cf[NNP];   // POLY: c_l = b_l (K^-1 yGP)_l ; otherwise yGP_k
#pragma unroll
    for (int k = 0; k < NNP; ++k) cf[k] = (R)mp[4 + k];
    double acc[NSLOT];
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) acc[k] = 0.0;
    if constexpr (MODE == MODE_POLY) {
#pragma unroll
      for (int b = 0; b < BPT; ++b)
        bin_poly<R, NNP>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b][0], bins.row[b][1], th1,
                         th2, th3, cf, acc);
    } else if constexpr (MODE == MODE_BREG) {
#pragma unroll
      for (int b = 0; b < BPT; ++b)
        bin_rows<R, NNP>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b], th1, th2, th3, cf, acc);
    } else {
      const R* pcx = (const R*)P.cx;
      const R* py = (const R*)P.y;
      const R* pisu = (const R*)P.isu;
      const R* pB = (const R*)P.B;
      for (int i = tid; i < P.n_pad; i += TPB) {
        R row[NNP];
#pragma unroll
        for (int k = 0; k < NNP; ++k) row[k] = pB[(size_t)i * NNP + k];
        bin_rows<R, NNP>(pcx[i], py[i], pisu[i], row, th1, th2, th3, cf, acc);
      }
    }
    const double r = transpose_reduce32(acc, lane);
    const int idx = lane >> 1;
    if (!(lane & 1) && idx < 4 + NNP) part[(wave * nct + c) * NSLOT + idx] = r;
  }
}

// ---------------------------------------------------------------------------
// the chain (one wave; lane = parameter)
// ---------------------------------------------------------------------------
template <int PPL>
struct Vd {
  double a[PPL];
};

template <int PPL>
struct Chain {
  using V = Vd<PPL>;
  static constexpr int VLEN = WAVE * PPL;
  const KParams& P;
  ChainScalars& S;
  double* Vb;
  double* QS;
  double* SUMS;
  double* MP;
  double* part;
  double* stk;
  const double* Kinv;
  const double* bv;
  int lane, slot, lc, gid, nct;
  RngKey key;

  __device__ Chain(const KParams& P_, const Lds<PPL>& L, int slot_, int lc_, int lane_, int nct_)
      : P(P_), S(L.cs(slot_)), Vb(L.vecs(slot_)), QS(L.qs(slot_)), SUMS(L.sums(slot_)),
        MP(L.mp(slot_)), part(L.part()), Kinv(L.kinv()), bv(L.bv()), lane(lane_), slot(slot_),
        lc(lc_), nct(nct_) {
    gid = P.chain_offset + lc;
    key = make_key(P.seed, (uint32_t)gid);
    stk = P.stack ? P.stack + (size_t)lc * P.max_depth * NSTK * VLEN : nullptr;
  }

  __device__ __forceinline__ int idx(int s) const { return s * WAVE + lane; }
  __device__ __forceinline__ bool ok(int s) const { return idx(s) < P.D; }
  __device__ __forceinline__ double* vec(int v) const { return Vb + v * VLEN; }
  __device__ __forceinline__ V ld(int v) const {
    V r;
#pragma unroll
    for (int s = 0; s < PPL; ++s) r.a[s] = vec(v)[idx(s)];
    return r;
  }
  __device__ __forceinline__ void st(int v, const V& x) const {
#pragma unroll
    for (int s = 0; s < PPL; ++s) vec(v)[idx(s)] = x.a[s];
  }
  __device__ __forceinline__ double* kslot(int level, int which) const {
    return stk + ((size_t)level * NSTK + which) * VLEN;
  }
  __device__ __forceinline__ V gld(int level, int which) const {
    V r;
    const double* p = kslot(level, which);
#pragma unroll
    for (int s = 0; s < PPL; ++s) r.a[s] = p[idx(s)];
    return r;
  }
  __device__ __forceinline__ void gst(int level, int which, const V& x) const {
    double* p = kslot(level, which);
#pragma unroll
    for (int s = 0; s < PPL; ++s) p[idx(s)] = x.a[s];
  }
  __device__ __forceinline__ void copyv(int dst, int src) const { st(dst, ld(src)); }

  __device__ __forceinline__ double dot(const V& a, const V& b) const {
    double x = 0.0;
#pragma unroll
    for (int s = 0; s < PPL; ++s) x = fma(a.a[s], b.a[s], x);
    return wave_sum(x);
  }
  __device__ __forceinline__ double kin(const V& p, const V& minv) const {
    double x = 0.0;
#pragma unroll
    for (int s = 0; s < PPL; ++s) x += p.a[s] * minv.a[s] * p.a[s];
    return 0.5 * wave_sum(x);
  }
  // stan::mcmc::base_nuts::compute_criterion on p_sharp = minv .* p (symmetric)
  __device__ __forceinline__ bool crit(const V& pa, const V& pb, const V& rho,
                                       const V& minv) const {
    double x = 0.0, y = 0.0;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      x += minv.a[s] * pb.a[s] * rho.a[s];
      y += minv.a[s] * pa.a[s] * rho.a[s];
    }
    wave_sum2(x, y);
    return x > 0.0 && y > 0.0;
  }
  __device__ __forceinline__ bool is_log(int k) const { return k < 3 || k >= 3 + P.Nn; }

  // ---------------- model parameters for the gradient phase ----------------
  __device__ __forceinline__ double hs_lam(int j) const {
    return exp(QS[5 + P.Nn + j] + 0.5 * QS[5 + 2 * P.Nn + j]);
  }
  __device__ __forceinline__ double hs_tau() const { return exp(QS[3 + P.Nn] + 0.5 * QS[4 + P.Nn]); }

  __device__ void write_mp(const V& q) const {
#pragma unroll
    for (int s = 0; s < PPL; ++s) QS[idx(s)] = q.a[s];
    wave_fence();
    if (lane < MPW) {
      double v = 0.0;
      if (lane < 3) {
        v = exp(QS[lane]);
      } else if (lane >= 4 && lane - 4 < P.Nn) {
        const int j = lane - 4;
        v = (P.family == FAM_HORSESHOE) ? QS[3 + j] * hs_lam(j) * hs_tau() : QS[3 + j];
      }
      MP[lane] = v;
    }
    if (P.mode == MODE_POLY) {  // c_l = b_l (K^-1 yGP)_l
      wave_fence();
      const int Nn = P.Nn;
      double c = 0.0;
      if (lane < Nn) {
        for (int k = 0; k < Nn; ++k) c = fma(Kinv[lane * Nn + k], MP[4 + k], c);
        c *= bv[lane];
      }
      wave_fence();
      if (lane < Nn) MP[4 + lane] = c;
    }
  }

  // ------------- lp / grad completion from the reduced bin sums --------------
  __device__ double complete(V& g) const {
    const int D = P.D, Nn = P.Nn, fam = P.family;
    const bool lik = (P.prior_PD == 0);
    const double Sd2 = SUMS[0];
    const bool bad = lik && !(Sd2 <= DBL_MAX);
    const double u0 = QS[0], u1 = QS[1], u2 = QS[2];
    const double th0 = exp(u0), th1 = exp(u1), th2 = exp(u2);
    const double usig = QS[D - 1], sig = exp(usig), is2 = 1.0 / (sig * sig);
    const double d0 = th0 - P.theta0[0], d1 = th1 - P.theta0[1], d2 = th2 - P.theta0[2];
    const double* Si = P.S0inv;
    const double Sd0 = Si[0] * d0 + Si[1] * d1 + Si[2] * d2;
    const double Sd1 = Si[3] * d0 + Si[4] * d1 + Si[5] * d2;
    const double Sd2t = Si[6] * d0 + Si[7] * d1 + Si[8] * d2;
    const double ss = P.sigma_scale;
    const double gyf = lik ? th1 * th2 * is2 : 0.0;   // dlp/dyGP_k = gyf * SUMS[4+k]
    double lpc = 0.0;
    if (lane == 0) {
      if (lik) lpc += -0.5 * Sd2 * is2 - (double)P.N * usig;
      lpc += -0.5 * (d0 * Sd0 + d1 * Sd1 + d2 * Sd2t) + u0 + u1 + u2;
      lpc += -0.5 * (sig / ss) * (sig / ss) + usig;
    }
    double lam = 0.0, S2 = 0.0, tau = 0.0, SGy = 0.0;
    if (fam == FAM_NORMAL) {
      lam = exp(QS[3 + Nn]);
      double part_ = 0.0;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        const int k = idx(s);
        if (k >= 3 && k < 3 + Nn) part_ += QS[k] * QS[k];
      }
      S2 = wave_sum(part_);
    } else if (fam == FAM_HORSESHOE) {
      tau = hs_tau();
      double part_ = 0.0;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        const int k = idx(s);
        if (k >= 3 && k < 3 + Nn) {
          const int j = k - 3;
          part_ += gyf * SUMS[4 + j] * (QS[k] * hs_lam(j) * tau);
        }
      }
      SGy = wave_sum(part_);
    }
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double gk = 0.0;
      if (k < D) {
        if (k < 3) {
          double gl = 0.0;
          if (lik) gl = (k == 0) ? SUMS[1] * is2 : (k == 1) ? SUMS[2] * is2 : th1 * SUMS[3] * is2 / th2;
          const double thk = (k == 0) ? th0 : (k == 1) ? th1 : th2;
          const double sdk = (k == 0) ? Sd0 : (k == 1) ? Sd1 : Sd2t;
          gk = thk * (gl - sdk) + 1.0;
        } else if (k == D - 1) {
          const double gl = lik ? (Sd2 * is2 - (double)P.N) / sig : 0.0;
          gk = sig * (gl - sig / (ss * ss)) + 1.0;
        } else if (fam == FAM_NORMAL) {
          if (k < 3 + Nn) {
            const double yv = QS[k];
            gk = gyf * SUMS[4 + (k - 3)] - yv / (lam * lam);
            lpc += -yv * yv / (2.0 * lam * lam);
          } else {
            const double rate = P.lambda_rate_eff;
            gk = lam * (-(double)Nn / lam + S2 / (lam * lam * lam) - rate) + 1.0;
            lpc += -(double)Nn * QS[k] - rate * lam + QS[k];
          }
        } else if (fam == FAM_LASSO) {
          const double yv = QS[k], ls = P.lambda_scale;
          const double sg = (yv > 0.0) ? 1.0 : (yv < 0.0) ? -1.0 : 0.0;
          gk = gyf * SUMS[4 + (k - 3)] - ls * sg - 2.0 * ls * yv;
          lpc += -ls * fabs(yv) - ls * yv * yv;
        } else {  // horseshoe (Tests/horseShoePrior.stan:25-43)
          const double nu = P.nu;
          if (k < 3 + Nn) {
            const int j = k - 3;
            const double z = QS[k];
            gk = gyf * SUMS[4 + j] * hs_lam(j) * tau - z;
            lpc += -0.5 * z * z;
          } else if (k == 3 + Nn) {
            const double r1 = exp(QS[k]);
            gk = SGy - r1 * r1 + 1.0;
            lpc += -0.5 * r1 * r1 + QS[k];
          } else if (k == 4 + Nn) {
            const double r2 = exp(QS[k]);
            gk = 0.5 * SGy - 1.5 + 0.5 / r2 + 1.0;
            lpc += -1.5 * QS[k] - 0.5 / r2 + QS[k];
          } else if (k < 5 + 2 * Nn) {
            const int j = k - 5 - Nn;
            const double Gy = gyf * SUMS[4 + j] * (QS[3 + j] * hs_lam(j) * tau);
            const double r1 = exp(QS[k]);
            gk = Gy - r1 * r1 + 1.0;
            lpc += -0.5 * r1 * r1 + QS[k];
          } else {
            const int j = k - 5 - 2 * Nn;
            const double Gy = gyf * SUMS[4 + j] * (QS[3 + j] * hs_lam(j) * tau);
            const double r2 = exp(QS[k]);
            gk = 0.5 * Gy - (0.5 * nu + 1.0) + 0.5 * nu / r2 + 1.0;
            lpc += -(0.5 * nu + 1.0) * QS[k] - 0.5 * nu / r2 + QS[k];
          }
        }
      }
      g.a[s] = gk;
    }
    double lp = wave_sum(lpc);
    if (bad || !(fabs(lp) <= DBL_MAX)) lp = -INFINITY;
    return lp;
  }

  __device__ void gather_sums() const {
    if (P.prior_PD == 0 && lane < NSLOT) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += part[(w * nct + slot) * NSLOT + lane];
      SUMS[lane] = s;
    }
    wave_fence();
    if (P.prior_PD == 0 && P.mode == MODE_POLY) {  // B^T h = K^-1 (b .* M)
      const int Nn = P.Nn;
      double v = 0.0;
      if (lane < Nn)
        for (int l = 0; l < Nn; ++l) v = fma(Kinv[lane * Nn + l], bv[l] * SUMS[4 + l], v);
      wave_fence();
      if (lane < Nn) SUMS[4 + lane] = v;
      wave_fence();
    }
  }

  // ------------------------------ randomness --------------------------------
  __device__ V momentum(uint32_t tag, uint32_t c0, uint32_t c3, const V& minv) const {
    V p;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double n0, n1;
      normal_pair(key, c0, tag, (uint32_t)(k >> 1), c3, n0, n1);
      const double n = (k & 1) ? n1 : n0;
      p.a[s] = (k < P.D) ? n / sqrt(minv.a[s]) : 0.0;
    }
    return p;
  }

  // ------------------------------ init --------------------------------------
  __device__ __attribute__((noinline)) void init_state() {
    V one, zero;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      one.a[s] = ok(s) ? 1.0 : 0.0;
      zero.a[s] = 0.0;
    }
    st(V_MINV, one);
    st(V_WF_M, zero);
    st(V_WF_M2, zero);
#pragma unroll
    for (int v = 0; v < NVEC; ++v)
      if (v != V_MINV && v != V_WF_M && v != V_WF_M2) st(v, zero);
    if (lane < NSLOT) SUMS[lane] = 0.0;
    S.status = 0;
    S.leapfrogs = 0;
    S.eps = P.stepsize0;
    S.mu = log(10.0 * P.stepsize0);
    S.da_counter = 0;
    S.s_bar = 0.0;
    S.x_bar = 0.0;
    // stan::mcmc::windowed_adaptation::set_window_params + restart
    const int W = P.warmup;
    int ib = P.init_buffer, tb = P.term_buffer, bw = P.base_window;
    S.win_on = (W >= 20) ? 1 : 0;
    if (W >= 20 && ib + bw + tb > W) {
      ib = (int)(0.15 * W);
      tb = (int)(0.1 * W);
      bw = W - (ib + tb);
    }
    S.init_buf = ib;
    S.term_buf = tb;
    S.win_counter = 0;
    S.win_size = bw;
    S.win_next = ib + bw - 1;
    S.wf_n = 0;
    S.t = 0;
    S.ss_window = 0;
    S.depth = 0;
    init_start(0);
  }

  __device__ void init_start(int attempt) {
    const int Nn = P.Nn;
    V q;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double base = 0.0, w = 0.0;
      if (k < 3) {
        base = log(P.theta0[k]);
        w = 0.025;
      } else if (k < 3 + Nn) {
        w = 0.05;
      } else if (k < P.D) {
        w = 0.25;
        if (P.family == FAM_NORMAL && k == 3 + Nn) base = -log(P.lambda_rate_eff);
      }
      const double u = uniform(key, (uint32_t)attempt, TAG_INIT, (uint32_t)k, 0u);
      q.a[s] = (k < P.D) ? base + P.init_radius * w * (2.0 * u - 1.0) : 0.0;
    }
    st(V_CUR_Q, q);
    S.init_attempt = attempt;
    S.state = ST_INIT;
    write_mp(q);
  }

  __device__ __attribute__((noinline)) void init_step(double lp, const V& g, double s2) {
    double bad = 0.0;
#pragma unroll
    for (int s = 0; s < PPL; ++s)
      if (ok(s) && !(fabs(g.a[s]) <= DBL_MAX)) bad = 1.0;
    bad = wave_sum(bad);
    if (!(lp > -INFINITY) || bad != 0.0) {
      if (S.init_attempt + 1 >= 100) {
        S.status = ERR_INIT;
        finish();
        return;
      }
      init_start(S.init_attempt + 1);
      return;
    }
    copyv(V_SMP_Q, V_CUR_Q);
    st(V_SMP_G, g);
    S.smp_lp = lp;
    S.smp_s2 = s2;
    if (P.adapt) {
      ss_begin();
    } else {
      start_transition();
    }
  }

  // --------------------- leapfrog (stan expl_leapfrog) -----------------------
  __device__ void start_leapfrog(double e) {
    V q = ld(V_CUR_Q), p = ld(V_CUR_P);
    const V g = ld(V_CUR_G), minv = ld(V_MINV);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      p.a[s] = fma(0.5 * e, g.a[s], p.a[s]);     // begin_update_p: p -= e/2 dphi/dq
      q.a[s] = fma(e, minv.a[s] * p.a[s], q.a[s]);  // update_q: q += e M^-1 p
    }
    st(V_CUR_P, p);
    st(V_CUR_Q, q);
    write_mp(q);
  }
  __device__ V finish_leapfrog(double e, const V& g) const {
    V p = ld(V_CUR_P);
#pragma unroll
    for (int s = 0; s < PPL; ++s) p.a[s] = fma(0.5 * e, g.a[s], p.a[s]);  // end_update_p
    st(V_CUR_P, p);
    st(V_CUR_G, g);
    return p;
  }

  // ----------------- base_hmc::init_stepsize as a state machine --------------
  __device__ void ss_begin() {
    const double eps = S.eps;
    if (eps == 0.0 || eps > 1e7 || isnan(eps)) {  // skipped like Stan
      ss_finish();
      return;
    }
    S.ss_trial = 0;
    S.state = ST_STEPSIZE;
    ss_new_trial();
  }
  __device__ void ss_new_trial() {
    const V minv = ld(V_MINV);
    const V p = momentum(TAG_SSMOM, (uint32_t)S.ss_window, (uint32_t)S.ss_trial, minv);
    S.ss_H0 = -S.smp_lp + kin(p, minv);
    copyv(V_CUR_Q, V_SMP_Q);
    copyv(V_CUR_G, V_SMP_G);
    st(V_CUR_P, p);
    start_leapfrog(S.eps);
  }
  __device__ __attribute__((noinline)) void ss_step(double lp, const V& g) {
    const V p = finish_leapfrog(S.eps, g);
    double h = -lp + kin(p, ld(V_MINV));
    if (isnan(h)) h = INFINITY;
    const double dH = S.ss_H0 - h;
    const double L08 = -0.22314355131420976;  // log(0.8)
    if (S.ss_trial == 0) {
      S.ss_dir = (dH > L08) ? 1 : -1;
      S.ss_trial = 1;
      ss_new_trial();
      return;
    }
    if ((S.ss_dir == 1 && !(dH > L08)) || (S.ss_dir == -1 && !(dH < L08))) {
      ss_finish();
      return;
    }
    S.eps = (S.ss_dir == 1) ? 2.0 * S.eps : 0.5 * S.eps;
    if (S.eps > 1e7 || S.eps == 0.0 || S.ss_trial > 2000) {
      S.status = ERR_NUMERIC;
      finish();
      return;
    }
    S.ss_trial += 1;
    ss_new_trial();
  }
  __device__ void ss_finish() {
    if (S.ss_window == 0) {
      start_transition();
    } else {  // adapt_diag_e_nuts::transition after a metric update
      S.mu = log(10.0 * S.eps);
      S.da_counter = 0;
      S.s_bar = 0.0;
      S.x_bar = 0.0;
      next_transition();
    }
  }

  // ------------------------------ transition --------------------------------
  __device__ void start_transition() {
    S.state = ST_TREE;
    S.eps_used = S.eps;
    const V minv = ld(V_MINV);
    const V p = momentum(TAG_MOM, (uint32_t)S.t, 0u, minv);
    st(V_SMP_P, p);
    S.H0 = -S.smp_lp + kin(p, minv);
    const V q = ld(V_SMP_Q), g = ld(V_SMP_G);
    st(V_E0_Q, q); st(V_E0_P, p); st(V_E0_G, g);
    st(V_E1_Q, q); st(V_E1_P, p); st(V_E1_G, g);
    S.end_lp[0] = S.end_lp[1] = S.smp_lp;
    S.end_s2[0] = S.end_s2[1] = S.smp_s2;
    st(V_RHO, p);
    S.lsw = 0.0;
    S.n_leapfrog = 0;
    S.sum_metro = 0.0;
    S.depth = 0;
    S.divergent = 0;
    begin_subtree();
  }

  __device__ void begin_subtree() {
    const int d = S.depth;
    const double u = uniform(key, (uint32_t)S.t, TAG_DIR, (uint32_t)d, 0u);
    const int dir = (u > 0.5) ? 1 : 0;
    S.dir = dir;
    const int eq = dir ? V_E1_Q : V_E0_Q;
    const V pe = ld(eq + 1);
    st(V_PNEAR, pe);
    copyv(V_CUR_Q, eq);
    st(V_CUR_P, pe);
    copyv(V_CUR_G, eq + 2);
    S.cur_lp = S.end_lp[dir];
    S.cur_s2 = S.end_s2[dir];
    S.leaf = 0;
    start_leapfrog(dir ? S.eps_used : -S.eps_used);
  }

  __device__ void push(int l, const V& pb, const V& pe, const V& rho, double lsw, int prop) {
    gst(l, K_PBEG, pb);
    gst(l, K_PEND, pe);
    gst(l, K_RHO, rho);
    S.st_lsw[l] = lsw;
    if (prop < 0) {
      gst(l, K_PQ, ld(V_CUR_Q));
      gst(l, K_PP, ld(V_CUR_P));
      gst(l, K_PG, ld(V_CUR_G));
      S.st_lp[l] = S.cur_lp;
      S.st_s2[l] = S.cur_s2;
    } else {
      gst(l, K_PQ, gld(prop, K_PQ));
      gst(l, K_PP, gld(prop, K_PP));
      gst(l, K_PG, gld(prop, K_PG));
      S.st_lp[l] = S.st_lp[prop];
      S.st_s2[l] = S.st_s2[prop];
    }
  }

  __device__ void take_sample(int prop) {
    if (prop < 0) {
      copyv(V_SMP_Q, V_CUR_Q);
      copyv(V_SMP_P, V_CUR_P);
      copyv(V_SMP_G, V_CUR_G);
      S.smp_lp = S.cur_lp;
      S.smp_s2 = S.cur_s2;
    } else {
      st(V_SMP_Q, gld(prop, K_PQ));
      st(V_SMP_P, gld(prop, K_PP));
      st(V_SMP_G, gld(prop, K_PG));
      S.smp_lp = S.st_lp[prop];
      S.smp_s2 = S.st_s2[prop];
    }
  }

  // one leaf of base_nuts::build_tree, followed by every merge it completes
  __device__ __attribute__((noinline)) void tree_leaf(double lp, const V& g, double s2) {
    const double e = S.dir ? S.eps_used : -S.eps_used;
    const V p = finish_leapfrog(e, g);
    const V minv = ld(V_MINV);
    S.cur_lp = lp;
    S.cur_s2 = s2;
    S.n_leapfrog += 1;
    double h = -lp + kin(p, minv);
    if (isnan(h)) h = INFINITY;
    if (h - S.H0 > 1000.0) S.divergent = 1;
    const double wl = S.H0 - h;
    S.sum_metro += (wl > 0.0) ? 1.0 : exp(wl);

    V Tpb = p, Tpe = p, Trho = p;
    double Tlsw = wl;
    int Tprop = -1;
    bool valid = (S.divergent == 0);
    const int d = S.depth, j = S.leaf;
    if (valid) {
      for (int l = 0; l < d; ++l) {
        if (((j >> l) & 1) == 0) {
          push(l, Tpb, Tpe, Trho, Tlsw, Tprop);
          break;
        }
        const V Ipb = gld(l, K_PBEG), Ipe = gld(l, K_PEND), Irho = gld(l, K_RHO);
        const double Ilsw = S.st_lsw[l];
        const double lsw_sub = lse(Ilsw, Tlsw);
        if (!(Tlsw > lsw_sub)) {
          const double u = uniform(key, (uint32_t)S.t, TAG_MERGE | ((uint32_t)l << 8) | ((uint32_t)d << 16),
                                   (uint32_t)j, 0u);
          if (!(u < exp(Tlsw - lsw_sub))) Tprop = l;
        }
        V rsub, rx, ry;
#pragma unroll
        for (int s = 0; s < PPL; ++s) {
          rsub.a[s] = Irho.a[s] + Trho.a[s];
          rx.a[s] = Irho.a[s] + Tpb.a[s];
          ry.a[s] = Trho.a[s] + Ipe.a[s];
        }
        const bool okc = crit(Ipb, Tpe, rsub, minv) && crit(Ipb, Tpb, rx, minv) &&
                         crit(Ipe, Tpe, ry, minv);
        Tpb = Ipb;
        Trho = rsub;
        Tlsw = lsw_sub;
        if (!okc) {
          valid = false;
          break;
        }
      }
    }
    if (!valid) {
      end_tree();
      return;
    }
    if (j == (1 << d) - 1) {  // the subtree of depth d is complete and valid
      const int dir = S.dir;
      const int eq = dir ? V_E1_Q : V_E0_Q;
      copyv(eq, V_CUR_Q);
      st(eq + 1, p);
      st(eq + 2, g);
      S.end_lp[dir] = S.cur_lp;
      S.end_s2[dir] = S.cur_s2;
      S.depth = d + 1;
      bool take;
      if (Tlsw > S.lsw) {
        take = true;
      } else {
        const double u = uniform(key, (uint32_t)S.t, TAG_TOP, (uint32_t)d, 0u);
        take = u < exp(Tlsw - S.lsw);
      }
      if (take) take_sample(Tprop);
      S.lsw = lse(S.lsw, Tlsw);
      const V far = ld(dir ? V_E0_P : V_E1_P), near = ld(V_PNEAR), rho = ld(V_RHO);
      V rtot, rx, ry;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        rtot.a[s] = rho.a[s] + Trho.a[s];
        rx.a[s] = rho.a[s] + Tpb.a[s];
        ry.a[s] = Trho.a[s] + near.a[s];
      }
      const bool persist = crit(far, Tpe, rtot, minv) && crit(far, Tpb, rx, minv) &&
                           crit(near, Tpe, ry, minv);
      st(V_RHO, rtot);
      if (!persist || S.depth >= P.max_depth) {
        end_tree();
        return;
      }
      begin_subtree();
    } else {
      S.leaf = j + 1;
      start_leapfrog(e);
    }
  }

  __device__ void write_draw(double accept, double energy) const {
    const int t = S.t, W = P.warmup;
    if (t < W && !P.save_warmup) return;
    const int it = P.save_warmup ? t : t - W;
    double* rec = P.draws + ((size_t)lc * P.iters_saved + it) * P.ncols;
    const V q = ld(V_SMP_Q);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      if (k < P.D) rec[7 + k] = is_log(k) ? exp(q.a[s]) : q.a[s];
    }
    if (lane < 8) {
      double v;
      switch (lane) {
        case 0: v = S.smp_lp; break;
        case 1: v = accept; break;
        case 2: v = S.eps_used; break;
        case 3: v = (double)S.depth; break;
        case 4: v = (double)S.n_leapfrog; break;
        case 5: v = (double)S.divergent; break;
        case 6: v = energy; break;
        default: v = (P.prior_PD == 0) ? S.smp_s2 / (double)P.N : NAN; break;
      }
      rec[lane < 7 ? lane : 7 + P.D] = v;
    }
  }

  __device__ void end_tree() {
    const double accept = S.sum_metro / (double)S.n_leapfrog;
    const V minv = ld(V_MINV);
    const double energy = -S.smp_lp + kin(ld(V_SMP_P), minv);
    write_draw(accept, energy);
    S.leapfrogs += S.n_leapfrog;
    if (S.t < P.warmup && P.adapt) {
      learn_stepsize(accept);
      if (learn_variance()) {
        S.ss_window += 1;
        ss_begin();
        return;
      }
    }
    next_transition();
  }

  // stan::mcmc::stepsize_adaptation::learn_stepsize
  __device__ void learn_stepsize(double adapt_stat) {
    S.da_counter += 1;
    const double cnt = (double)S.da_counter;
    adapt_stat = adapt_stat > 1.0 ? 1.0 : adapt_stat;
    const double eta = 1.0 / (cnt + P.t0);
    S.s_bar = (1.0 - eta) * S.s_bar + eta * (P.adapt_delta - adapt_stat);
    const double x = S.mu - S.s_bar * sqrt(cnt) / P.gamma;
    const double x_eta = pow(cnt, -P.kappa);
    S.x_bar = (1.0 - x_eta) * S.x_bar + x_eta * x;
    S.eps = exp(x);
  }

  // stan::mcmc::var_adaptation::learn_variance + windowed_adaptation
  __device__ bool learn_variance() {
    const int W = P.warmup, cnt = S.win_counter;
    const int tb = S.term_buf;
    if (S.win_on && cnt >= S.init_buf && cnt < W - tb && cnt != W) {
      S.wf_n += 1;
      const double n = (double)S.wf_n;
      const V q = ld(V_SMP_Q);
      V m = ld(V_WF_M), m2 = ld(V_WF_M2);
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        const double delta = q.a[s] - m.a[s];
        m.a[s] += delta / n;
        m2.a[s] += (q.a[s] - m.a[s]) * delta;
      }
      st(V_WF_M, m);
      st(V_WF_M2, m2);
    }
    if (S.win_on && cnt == S.win_next && cnt != W) {
      // compute_next_window
      const int last = W - tb - 1;
      if (S.win_next != last) {
        S.win_size *= 2;
        S.win_next = cnt + S.win_size;
        if (S.win_next != last) {
          const int boundary = S.win_next + 2 * S.win_size;
          if (boundary >= W - tb) S.win_next = last;
        }
      }
      const double n = (double)S.wf_n;
      V var = ld(V_MINV);
      const V m2 = ld(V_WF_M2);
      V zero;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        zero.a[s] = 0.0;
        if (ok(s)) {
          if (S.wf_n > 1) var.a[s] = m2.a[s] / (n - 1.0);
          var.a[s] = (n / (n + 5.0)) * var.a[s] + 1e-3 * (5.0 / (n + 5.0));
        }
      }
      st(V_MINV, var);
      st(V_WF_M, zero);
      st(V_WF_M2, zero);
      S.wf_n = 0;
      S.win_counter = cnt + 1;
      return true;
    }
    S.win_counter = cnt + 1;
    return false;
  }

  __device__ void next_transition() {
    S.t += 1;
    if (S.t == P.warmup && P.adapt && P.warmup > 0) S.eps = exp(S.x_bar);  // complete_adaptation
    if (S.t >= P.warmup + P.samples) {
      finish();
      return;
    }
    start_transition();
  }

  __device__ void finish() {
    S.state = ST_DONE;
    const V q = ld(V_SMP_Q), minv = ld(V_MINV);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      if (k < P.D) {
        if (P.fin_q) P.fin_q[(size_t)lc * P.D + k] = q.a[s];
        if (P.fin_minv) P.fin_minv[(size_t)lc * P.D + k] = minv.a[s];
      }
    }
    if (lane == 0) {
      if (P.fin_eps) P.fin_eps[lc] = S.eps;
      if (P.chain_status) P.chain_status[lc] = S.status;
      if (P.leapfrogs) P.leapfrogs[lc] = S.leapfrogs;
    }
  }

  // one NUTS phase: the gradient at CUR_Q is in the partial sums
  __device__ __attribute__((noinline)) void phase() {
    if (S.state == ST_DONE) return;
    gather_sums();
    V g;
    const double lp = complete(g);
    const double s2 = (P.prior_PD == 0) ? SUMS[0] : NAN;
    switch (S.state) {
      case ST_INIT: init_step(lp, g, s2); break;
      case ST_STEPSIZE: ss_step(lp, g); break;
      default: tree_leaf(lp, g, s2); break;
    }
    wave_fence();
  }
};

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
template <int PPL>
__device__ __forceinline__ void load_kinv(const KParams& P, const Lds<PPL>& L, int tid) {
  if (P.mode == MODE_POLY) {
    const int Nn = P.Nn;
    for (int i = tid; i < Nn * Nn; i += TPB) L.kinv()[i] = P.Kinv[i];
    if (tid < Nn) L.bv()[tid] = P.bvec[tid];
  }
}

template <class R, int BPT, int NNP, int PPL, int MODE>
__global__ void __launch_bounds__(TPB, 4) nuts_kernel(const KParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds<PPL> L{smem, P.G};
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid >> 6;
  const int c0 = blockIdx.x * P.G;
  const int nct = min(P.G, P.chains - c0);
  __shared__ int act[GMAX];

  Bins<R, BPT, NNP, MODE> bins;
  bins.load(P, tid);
  load_kinv(P, L, tid);
  __syncthreads();

  if (wave < nct) {
    Chain<PPL> ch(P, L, wave, c0 + wave, lane, nct);
    ch.init_state();
    wave_fence();
  }
  __syncthreads();
  const bool lik = (P.prior_PD == 0);
  for (long long step = 0;; ++step) {
    if (tid < GMAX) act[tid] = (tid < nct) && (L.cs(tid).state != ST_DONE);
    __syncthreads();
    int nact = 0;
#pragma unroll
    for (int c = 0; c < GMAX; ++c) nact += act[c];
    if (nact == 0) break;
    if (step >= P.max_steps) {  // termination guarantee: report and drain
      if (wave < nct && lane == 0 && L.cs(wave).state != ST_DONE && P.chain_status)
        P.chain_status[c0 + wave] = -6;
      break;
    }
    if (lik)
      gradient_pass<R, BPT, NNP, MODE>(P, bins, L.mp(0), L.part(), act, nct, tid, lane, wave);
    __syncthreads();
    if (wave < nct) {
      Chain<PPL> ch(P, L, wave, c0 + wave, lane, nct);
      ch.phase();
    }
    __syncthreads();
  }
}

template <class R, int BPT, int NNP, int PPL, int MODE>
__global__ void __launch_bounds__(TPB, 4) logp_kernel(const KParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds<PPL> L{smem, P.G};
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid >> 6;
  const int c0 = blockIdx.x * P.G;
  const int nct = min(P.G, P.chains - c0);
  __shared__ int act[GMAX];
  Bins<R, BPT, NNP, MODE> bins;
  bins.load(P, tid);
  load_kinv(P, L, tid);
  if (tid < GMAX) act[tid] = (tid < nct);
  __syncthreads();
  if (wave < nct) {
    Chain<PPL> ch(P, L, wave, c0 + wave, lane, nct);
    Vd<PPL> q;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = s * WAVE + lane;
      q.a[s] = (k < P.D) ? P.q_in[(size_t)(c0 + wave) * P.D + k] : 0.0;
    }
    if (lane < NSLOT) ch.SUMS[lane] = 0.0;
    ch.write_mp(q);
    wave_fence();
  }
  __syncthreads();
  if (P.prior_PD == 0)
    gradient_pass<R, BPT, NNP, MODE>(P, bins, L.mp(0), L.part(), act, nct, tid, lane, wave);
  __syncthreads();
  if (wave < nct) {
    Chain<PPL> ch(P, L, wave, c0 + wave, lane, nct);
    ch.gather_sums();
    Vd<PPL> g;
    const double lp = ch.complete(g);
    const size_t pt = (size_t)(c0 + wave);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = s * WAVE + lane;
      if (k < P.D) P.grad_out[pt * P.D + k] = g.a[s];
    }
    if (lane == 0) {
      P.lp_out[pt] = lp;
      if (P.s2_out) P.s2_out[pt] = (P.prior_PD == 0) ? ch.SUMS[0] : NAN;
    }
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch over the template grid
// ---------------------------------------------------------------------------
int lds_bytes(int ppl, int G) { return ppl == 1 ? Lds<1>::bytes(G) : Lds<2>::bytes(G); }

template <class R, int BPT, int NNP, int PPL, int MODE>
static hipError_t launch_t(bool logp, const KParams& P, int tiles, hipStream_t st) {
  const int lds = Lds<PPL>::bytes(P.G);
  if (logp) {
    auto k = logp_kernel<R, BPT, NNP, PPL, MODE>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(tiles), dim3(TPB), lds, st, P);
  } else {
    auto k = nuts_kernel<R, BPT, NNP, PPL, MODE>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(tiles), dim3(TPB), lds, st, P);
  }
  return hipGetLastError();
}

template <int NNP, int PPL>
static hipError_t launch_n(bool logp, bool mixed, int bpt, const KParams& P, int tiles,
                           hipStream_t st) {
  if (!mixed) {
    if (P.mode == MODE_POLY) {
      switch (bpt) {
        case 1: return launch_t<double, 1, NNP, PPL, MODE_POLY>(logp, P, tiles, st);
        case 2: return launch_t<double, 2, NNP, PPL, MODE_POLY>(logp, P, tiles, st);
        case 4: return launch_t<double, 4, NNP, PPL, MODE_POLY>(logp, P, tiles, st);
        default: return hipErrorInvalidValue;
      }
    }
    return launch_t<double, 0, NNP, PPL, MODE_STREAM>(logp, P, tiles, st);
  }
  if (P.mode == MODE_BREG) {
    switch (bpt) {
      case 1: return launch_t<float, 1, NNP, PPL, MODE_BREG>(logp, P, tiles, st);
      case 2: return launch_t<float, 2, NNP, PPL, MODE_BREG>(logp, P, tiles, st);
      default: return hipErrorInvalidValue;
    }
  }
  return launch_t<float, 0, NNP, PPL, MODE_STREAM>(logp, P, tiles, st);
}

hipError_t launch(bool logp, bool mixed, int bpt, int nnp, const KParams& P, int tiles,
                  hipStream_t st) {
#ifdef FITOCT_ONE_VARIANT
  return launch_t<double, 2, 16, 1, MODE_POLY>(logp, P, tiles, st);
#else
  if (nnp == 16) return launch_n<16, 1>(logp, mixed, bpt, P, tiles, st);
  return launch_n<24, 2>(logp, mixed, bpt, P, tiles, st);
#endif
}

}  // namespace fitoct
