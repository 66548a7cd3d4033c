// Device-resident NUTS for the FitOCT ExpGP posterior (gfx950 / MI355X).
//
// Replaces rstan::sampling + Stan's base_nuts / adapt_diag_e_nuts + the
// stanc-generated model with stan-math AD.
//
// Execution model ("tile" = one 512-thread workgroup of 8 waves, persistent for the
// whole run; kernel_params.h NW / NGW / GMAX):
//   * a tile owns G <= 4 chains.  Each chain is an explicit state machine (init
//     -> step-size search -> tree building -> adaptation -> next transition)
//     that consumes one gradient per leapfrog, so a chain that finishes its
//     trajectory starts its next transition at once: no chain waits for
//     another chain's tree.
//   * the 8 waves are specialised: waves 0..3 only run the likelihood sweep,
//     waves 4..7 only run NUTS (one chain each); waves w and w+4 share SIMD
//     w mod 4, so every SIMD holds one gradient wave and one NUTS wave.  The
//     roles meet in a dataflow pipeline through LDS: a NUTS wave enqueues its
//     chain's next position in a ring, the gradient waves drain the ring in
//     order and count their completions per chain, the NUTS wave resumes when
//     all 4 sweeps are in.  No barrier after start-up: each chain's sampler
//     latency hides behind the sweeps of the tile's other chains.
//   * gradient waves: the N depth bins are strided over 256 lanes; each lane
//     keeps its bins' data resident in VGPRs for the whole run (read from HBM
//     once per tile, shared by all G chains; up to 8 bins per lane, or 16 in
//     the compact layout for arithmetic depth grids).  For the
//     built-in uniform-grid SE basis (MODE_POLY) the GP basis factorises as
//     K(x~_i, g_l) = a_i t_i^l b_l, so a bin needs 5 registers (c*x, y, 1/uy,
//     t, a) instead of a 16-wide basis row: dL_i = a_i P(t_i) by Horner on the
//     chain's coefficients c = b .* K^-1 yGP, and B^T h = K^-1 (b .* M) from
//     the moments M_l = sum_i h_i a_i t_i^l.  A user-supplied basis keeps its
//     rows in registers (MODE_ROWS, fp32) or streams them (MODE_STREAM).
//     Per chain a lane accumulates 4+NNP partial sums; a transposed butterfly
//     built from v_permlane32_swap / v_permlane16_swap / DPP row mirrors
//     reduces them across the wave (no LDS round trips), and 4 per-wave
//     partials land in LDS.
//   * NUTS phase (wave 4+c drives chain c): lane k holds parameter k.  The wave
//     sums the 4 partials, completes lp / grad with the priors and the
//     log-Jacobians, and advances the chain's state machine.  Stan's recursive
//     build_tree is replayed iteratively, one leaf per step: the U-turn records
//     (p_beg, p_end, rho) of each tree level live in LDS, the multinomial
//     proposals (q, grad; the momentum only as its energy) in a per-chain HBM pool addressed by slot index, so
//     a proposal is written once when its leaf is pushed and read only when it
//     becomes the sample.  Wave reductions are DPP/permlane butterflies.
//   * workgroups communicate only to hand whole chains between tiles at transition
//     boundaries (chain migration, the MIG instantiation).
//   * a tile of one chain (fewer chains than CUs) puts its three spare NUTS waves to work:
//     two producers leapfrog the trajectory's backward and forward ends at once and a
//     helper books the leaves in Stan's tree order ("Two-ended trajectories" below).
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

// Explicit address spaces: LDS (3), global (1), constant (4).  Generic pointers
// would compile to FLAT instructions, which count in both vmcnt and lgkmcnt --
// every LDS wait would then also wait for the sampler's outstanding HBM stores.
#define AS_LDS __attribute__((address_space(3)))
#define AS_GLB __attribute__((address_space(1)))
#define AS_CST __attribute__((address_space(4)))
using KPc = const AS_CST KParams;

enum { FAM_NORMAL = 0, FAM_LASSO = 1, FAM_HORSESHOE = 2, FAM_MONO = 3 };
// (round 6: the A/B switches measured "off" or "rejected" in DESIGN.md §4 are gone from
// the kernel; what is left compiles to the measured defaults.  The only remaining build
// switches are the ordering fallbacks FITOCT_LOCAL_FENCE / FITOCT_LDS_INORDER and the
// profiling build FITOCT_PROFILE.)
// 16 bins per lane (config 4): moments are formed per group of 8 bins
constexpr int BPT16_GROUP = 8;

// Cycle stamps (FITOCT_STAMPS) exist only in a profiling build
// (FITOCT_PROFILE=1 python -m fitoct_amd.build): the production kernels carry
// no per-action timing code at all.
#ifndef FITOCT_PROFILE
#define FITOCT_PROFILE 0
#endif
constexpr bool kProfile = FITOCT_PROFILE != 0;
// -DFITOCT_ASM_MARKS: assembly comments at action boundaries, for per-action
// instruction counts in a -S listing (scripts/asm_actions.py); no code otherwise
#ifdef FITOCT_ASM_MARKS
#define FITOCT_MARK(name) asm volatile(";MARK " #name)
#else
#define FITOCT_MARK(name)
#endif
enum { ERR_INIT = -4, ERR_NUMERIC = -5, ERR_TIMEOUT = -6, ERR_CANCELLED = -8 };

// vectors kept in LDS per chain (lane-private elements)
enum VecId : int {
  V_CUR_Q, V_CUR_P, V_CUR_G,
  V_E0_Q, V_E0_P, V_E0_G,      // backward end of the trajectory
  V_E1_Q, V_E1_P, V_E1_G,      // forward end
  V_SMP_Q, V_SMP_G,            // z_sample (its momentum enters only the energy: smp_h)
  V_MINV, V_WF_M, V_WF_M2,     // metric + Welford
  V_RHO, V_PNEAR,              // trajectory momentum sum, near end of old trajectory
  V_QS, V_QE,                  // staged q and its constrained values (exp on positive params)
  V_PG, V_CA,                  // prior part of grad, likelihood coefficient (prior_part)
  NVEC
};
// U-turn record of one tree level (LDS)
enum LvlId : int { K_PBEG = 0, K_PEND = 1, K_RHO = 2, NLVL = 3 };
// proposal pool slot (HBM): q and g of a candidate sample.  Its momentum is dead once it is
// a candidate (the next transition draws a fresh one) except in the energy__ diagnostic,
// H(z_sample), which is the candidate leaf's own Hamiltonian h: kept as a scalar (pool_h)
enum PoolId : int { P_Q = 0, P_G = 1, NPOOL = POOL_VECS };
constexpr int NAUX = 96;   // per chain: yGP[32] | horseshoe lambda_j*tau [32] | FW_j [32]

struct ChainScalars {
  int state, t, depth, leaf, dir, n_leapfrog, divergent, init_attempt;
  int da_counter, win_counter, win_size, win_next, wf_n, ss_trial, ss_dir, ss_window;
  int status, win_on, init_buf, term_buf, pool_used, lsw_e, spec_we, pad2;
  int st_prop[MAXDEPTH];
  int st_w_e[MAXDEPTH];
  double H0, lsw_m, sum_metro, eps, eps_used, mu, s_bar, x_bar, ss_H0, lf_e;
  double cur_lp, cur_s2, smp_lp, smp_s2;
  double pr_lp, pr_is2, u_top, spec_wm;   // spec_wm, spec_we, spec_h: the speculative
                                          // path's booked leaf weight and energy
  int u_blk[MAXDEPTH];     // which block of 64 merge uniforms each level's ring holds (-1: none)
  double end_lp[2], end_s2[2];
  double st_w_m[MAXDEPTH];
  double pool_lp[MAXDEPTH + 1], pool_s2[MAXDEPTH + 1];
  long long leapfrogs;
  double spec_h;
  // Hamiltonian -lp + K(p) of each pool candidate and of the sample (energy__)
  double pool_h[MAXDEPTH + 1], smp_h;
  // the running subtree's sum of the leaves' acceptance terms (added to sum_metro when the
  // subtree ends, so two-ended trajectories can sum per subtree and stay bitwise equal)
  double sub_metro, pad_sm;
  long long prof[2][32];   // diagnostic build: cycles and calls per action
};
static_assert(sizeof(ChainScalars) % 16 == 0, "LDS carve alignment");

// two-ended trajectories (P.bidi): the tile's hand-off words in LDS.  BD_GEN: the transition
// (1..BD_GEN_MASK, -1: the chain has finished); BD_PROD + s: stream s's published leaves as
// (gen << 16) | count; BD_CONS + s: leaves of stream s the helper has booked; BD_END: the
// transition whose tree the helper has ended; BD_EXIT: producers that have left
// TW_*: who grows the ends -- the producers' NUTS slots (TW_SLOT, TW_SLOT + 1; a tile of
// one chain: 1, 2), the chain's slot and index (TW_CHAIN, TW_LC; written by bidi_begin);
// migrating tiles recruit producers at run time (TW_CLAIM: role bits claimed, TW_JOIN:
// producers in place; see receive_chain)
enum BdWord : int {
  BD_GEN = 0, BD_PROD = 1, BD_CONS = 3, BD_END = 5, BD_EXIT = 6,
  TW_CLAIM = 7, TW_JOIN = 8, TW_SLOT = 9, TW_CHAIN = 11, TW_LC = 12, TW_BUSY = 13, BD_N = 16
};
constexpr int BD_GEN_MASK = (1 << 15) - 1;
// BD_GEN | BD_ENDED: a migrating tile's chain has booked transition BD_GEN's tree to its end
// (its producers stop, and wait for the next transition or the launch's end)
constexpr int BD_ENDED = 1 << 20;
// a producer runs at most this many doublings past the booked one (lookahead 1 / 2 / 5
// measured -1.0 / -0.2 / +-0 % on config 2, profiles/r05_ab_stage.txt)
constexpr int BIDI_LOOK = 3;

constexpr long long SPIN_LIMIT = 1LL << 26;   // polls (~2 s) before a wait reads the clock
constexpr unsigned long long TICKS_PER_S = 100000000ULL;   // s_memrealtime: 100 MHz
// a wait for one leaf's work (a sweep, a booking, a producer's record): far above any real
// leaf (microseconds; a deep tree's whole trajectory is bounded separately, MIG_WAIT_TICKS)
constexpr unsigned long long LEAF_WAIT_TICKS = 30ULL * TICKS_PER_S;

// The hang guard of every wait in the kernel.  The first SPIN_LIMIT polls read no clock;
// past them the wait is bounded in REAL time (s_memrealtime), not in polls, so a slow
// sweep, a profiler or a deep tree never fails a healthy chain with ERR_TIMEOUT, and a
// fault still ends the launch.  expired(T) is true once T ticks passed since poll SPIN_LIMIT.
struct Patience {
  long long n = 0;
  unsigned long long t0 = 0;
  __device__ __forceinline__ bool expired(unsigned long long ticks) {
    if (++n <= SPIN_LIMIT) return false;
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (n == SPIN_LIMIT + 1) t0 = t;
    __builtin_amdgcn_s_sleep(32);
    return t - t0 > ticks;
  }
};

__device__ __forceinline__ void wave_fence() {
  // orders this wave's LDS traffic: every earlier ds_* op has completed and the
  // compiler may not move memory accesses across this point.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
// A wave reading back what its own lanes just stored to LDS: the DS operations of one
// wave are performed in issue order (the AMDGPU memory model), so only the compiler must
// keep the order -- no wait for the stores to complete (FITOCT_LOCAL_FENCE=0: the full wait)
#ifndef FITOCT_LOCAL_FENCE
#define FITOCT_LOCAL_FENCE 1
#endif
__device__ __forceinline__ void wave_order() {
#if FITOCT_LOCAL_FENCE
  asm volatile("" ::: "memory");
#else
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
}
// A wave publishing LDS data to another wave of the tile by a later LDS store or atomic (a
// sweep's partial sums before grad_cnt, a position's MP before its ring entry, a leaf record
// before its count): the LDS performs one wave's DS operations in issue order, so a reader
// that sees the count and then reads the data sees the data.  FITOCT_LDS_INORDER=0: wait for
// the data stores to complete first (s_waitcnt lgkmcnt(0)).
#ifndef FITOCT_LDS_INORDER
#define FITOCT_LDS_INORDER 1
#endif
__device__ __forceinline__ void wave_publish() {
#if FITOCT_LDS_INORDER
  asm volatile("" ::: "memory");
#else
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
}

// ---------------------------------------------------------------------------
// chain migration between tiles: agent-scope atomics on global memory (the
// tiles of a launch sit on different XCDs, each with its own L2; release /
// acquire at agent scope write back / invalidate L2 as the gfx950 memory model
// requires).  Rare operations (at most one per transition), so generic pointers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int g_load(AS_GLB int* p) {
  return __hip_atomic_load((int*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_add(AS_GLB int* p, int v) {
  return __hip_atomic_fetch_add((int*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_or(AS_GLB int* p, int v) {
  return __hip_atomic_fetch_or((int*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_and(AS_GLB int* p, int v) {
  return __hip_atomic_fetch_and((int*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// run-time progress / cancellation: host-pinned fine-grained memory, read by the
// host while the kernel runs (system scope; at most one access per transition)
__device__ __forceinline__ void sys_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int sys_load(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool g_cas(AS_GLB int* p, int expect, int v) {
  return __hip_atomic_compare_exchange_strong((int*)p, &expect, v, __ATOMIC_RELAXED,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct MigView {   // KParams::mig carved per MigCtrl
  AS_GLB int* hdr;
  AS_GLB int* load;
  AS_GLB int* fmask;
  AS_GLB int* mbox;
  __device__ MigView(int* base, int tiles)
      : hdr((AS_GLB int*)base), load((AS_GLB int*)base + MIG_HDR), fmask(load + tiles),
        mbox(fmask + tiles) {}
};
constexpr unsigned long long MIG_WAIT_TICKS = 120ULL * TICKS_PER_S;

// ---------------------------------------------------------------------------
// paired tiles (KParams::pair): the forward end of a one-chain tile's two-ended trajectories
// grows in a partner tile, with its own four gradient waves.  Everything crossing between
// the two workgroups is a write-through (sc1) agent-scope store, drained by the storing wave
// (s_waitcnt vmcnt(0)) before the one word that publishes it, and read with sc1 loads only
// (relaxed agent-scope atomics: global_load / global_store ... sc1, no L1 copy on either
// side), so no L2 write-back or invalidation is needed whichever XCDs the two tiles sit on.
// Per pair: PAIR_HDR_INTS hand-off words (zeroed before every launch), then in pair_buf
// the transition's start and one subtree record of the forward end.
// ---------------------------------------------------------------------------
enum PairHdr : int {
  // primary -> partner: the transition (its start is in pair_buf; -1: the chain finished),
  // the booking's records taken of the forward end and the booked depth, each (gen << 16) | v;
  // the chain's index and the transition's number t
  PH_GEN = 0, PH_CONS = 1, PH_DEPTH = 2, PH_LC = 3, PH_T = 4,
  PH_COUNT = 32,   // partner -> primary: (gen << 16) | forward-end subtree records published
  PH_STATE = 48    // PairState bits (both, atomics); PAIR_HDR_INTS words per pair (kernel_params.h)
};
// The pair's hand-shake: the primary marks START when it begins; the partner joins (START ->
// START | JOIN) only if the primary has begun, else marks LOCAL and leaves; the primary decides
// at its chain's first transition (START -> START | LOCAL unless the partner has joined).  So
// a partner that is not resident (a busy GPU) never holds up its primary, and a primary only
// ever waits for a partner that is running: the unpaired tile grows both ends itself.
enum PairState : int { PS_START = 1, PS_JOIN = 2, PS_LOCAL = 4 };
constexpr unsigned long long PAIR_JOIN_TICKS = 10000;   // 100 us (s_memrealtime: 100 MHz)
__device__ __forceinline__ void x_st(AS_GLB double* p, double v) {
  __hip_atomic_store((AS_GLB unsigned long long*)p, __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double x_ld(const AS_GLB double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((AS_GLB unsigned long long*)p,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void x_sti(AS_GLB int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int x_ldi(AS_GLB int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every sc1 store of this wave has reached memory (before the word that publishes them)
__device__ __forceinline__ void x_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------
// cross-lane moves of doubles without LDS (DPP row ops, gfx950 permlane swaps)
// ---------------------------------------------------------------------------
constexpr int DPP_XOR1 = 0xB1;         // quad_perm(1,0,3,2)
constexpr int DPP_XOR2 = 0x4E;         // quad_perm(2,3,0,1)
constexpr int DPP_QREV = 0x1B;         // quad_perm(3,2,1,0): flip bits 0,1
constexpr int DPP_HALF_MIRROR = 0x141; // lane i <-> 7-i within 8: flip bits 0..2
constexpr int DPP_MIRROR = 0x140;      // lane i <-> 15-i within 16: flip bits 0..3

// (bound_ctrl: a disabled source lane reads 0, as the zero 'old' operand of update_dpp
// gave, without a v_mov of that zero before every DPP move)
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// v_readlane of a double (lane index wave-uniform)
__device__ __forceinline__ double rl(double x, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// a' = a with rows {1,3} (lanes 16-31, 48-63) replaced by b's rows {0,2};
// b' = b with rows {0,2} replaced by a's rows {1,3}.  Returns a' + b'.
__device__ __forceinline__ double swap16_add(double a, double b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  const double a2 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
  const double b2 = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  return a2 + b2;
}
// same across the two 32-lane halves
__device__ __forceinline__ double swap32_add(double a, double b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  const double a2 = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
  const double b2 = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
  return a2 + b2;
}

// butterfly sum over the wave; every lane ends with the bitwise-identical value
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp<DPP_XOR1>(x);
  x += dpp<DPP_XOR2>(x);
  x += dpp<DPP_HALF_MIRROR>(x);
  x += dpp<DPP_MIRROR>(x);
  x = swap16_add(x, x);
  return swap32_add(x, x);
}
__device__ __forceinline__ void wave_sum2(double& a, double& b) {
  a += dpp<DPP_XOR1>(a);
  b += dpp<DPP_XOR1>(b);
  a += dpp<DPP_XOR2>(a);
  b += dpp<DPP_XOR2>(b);
  a += dpp<DPP_HALF_MIRROR>(a);
  b += dpp<DPP_HALF_MIRROR>(b);
  a += dpp<DPP_MIRROR>(a);
  b += dpp<DPP_MIRROR>(b);
  a = swap16_add(a, a);
  b = swap16_add(b, b);
  a = swap32_add(a, a);
  b = swap32_add(b, b);
}

// N independent butterfly sums, stage by stage (the DPP / permlane moves of the
// N values overlap instead of serialising N reductions)
template <int N>
__device__ __forceinline__ void wave_sum_n(double (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] += dpp<DPP_XOR1>(x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] += dpp<DPP_XOR2>(x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] += dpp<DPP_HALF_MIRROR>(x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] += dpp<DPP_MIRROR>(x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = swap16_add(x[i], x[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = swap32_add(x[i], x[i]);
}

// exp on the sampler side: reduction by ln2 (hi/lo), Taylor degree 12 on
// |r| <= ln2/2, n = round(x log2 e) from the 1.5*2^52 shifter fed straight to
// v_ldexp_f64 (<= 2 ulp from the library exp, scripts/micro/acc.hip; no special
// cases: x is clamped to [-746, 710], where exp is 0 / inf either way).
// v_fma_f64 with all three operands in VGPRs.  In the sampler's code the compiler keeps
// fexp's coefficients in VGPRs (its SGPRs are spent) and forms p * r + c as a copy of c into
// the destination plus a v_fmac_f64: two VALU instructions per Horner step.  Same operation.
__device__ __forceinline__ double fma_v(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
template <bool V3>
__device__ __forceinline__ double fmac3(double a, double b, double c) {
  if constexpr (V3) return fma_v(a, b, c);
  else return fma(a, b, c);
}
// V3: Horner steps as fma_v (the samplers where that form compiles without spills, Chain::FV3)
template <bool V3 = false>
__device__ __forceinline__ double fexp(double x) {
  x = fmin(fmax(x, -746.0), 710.0);
  const double SH = 6755399441055744.0;   // 1.5 * 2^52
  const double t = fma(x, 1.4426950408889634, SH);
  const double n = t - SH;
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
  double r = fma(-n, 6.93147180369123816490e-01, x);
  r = fma(-n, 1.90821492927058770002e-10, r);
  double p = 2.08767569878680989792e-09;   // 1/12!
  p = fmac3<V3>(p, r, 2.50521083854417187751e-08);
  p = fmac3<V3>(p, r, 2.75573192239858906526e-07);
  p = fmac3<V3>(p, r, 2.75573192239858906526e-06);
  p = fmac3<V3>(p, r, 2.48015873015873015873e-05);
  p = fmac3<V3>(p, r, 1.98412698412698412698e-04);
  p = fmac3<V3>(p, r, 1.38888888888888888889e-03);
  p = fmac3<V3>(p, r, 8.33333333333333333333e-03);
  p = fmac3<V3>(p, r, 4.16666666666666666667e-02);
  p = fmac3<V3>(p, r, 1.66666666666666666667e-01);
  p = fmac3<V3>(p, r, 0.5);
  p = fmac3<V3>(p, r, 1.0);
  p = fmac3<V3>(p, r, 1.0);
  return ldexp(p, ni);
}
// 1/x to <= 1 ulp: v_rcp_f64 and one Newton step (x finite, nonzero)
__device__ __forceinline__ double frcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}

// Multinomial trajectory weights exp(H0 - H) as extended-exponent floats
// m * 2^e (m in [1/2, 1) or 0): the merges of base_nuts (log_sum_exp of log
// weights, then u < exp(lsw_final - lsw_subtree)) become an add and a multiply,
// with no exp / log1p per merge and no overflow for any energy change.  The
// oracle (oracle/fitoct_oracle.c) uses the same representation.
struct XF {
  double m;
  int e;
};
__device__ __forceinline__ XF xf_norm(double m, int e) {
  int k;
  const double f = frexp(m, &k);
  return XF{f, f == 0.0 ? 0 : e + k};
}
template <bool V3 = false>
__device__ __forceinline__ XF xf_exp(double x) {   // exp(x), x <= +inf; -inf -> 0
  if (x > -700.0 && x < 700.0) return xf_norm(fexp<V3>(x), 0);
  // above 1e8 (an energy drop no trajectory of a finite start reaches) the weight
  // saturates: the exponent stays within int, and so does the exponent difference of
  // two weights in xf_u_below (>= -1.45e9 - 1.45e8)
  if (!(x < 1.0e8)) x = 1.0e8;
  // below -1e9 (a divergent leaf: its weight is never merged) the exponent would not fit
  // an int; the weight is 0 to every digit the merges can resolve
  if (!(x > -1.0e9)) return XF{0.0, 0};
  const double k = floor(x * 1.4426950408889634);   // log2(e)
  return xf_norm(fexp<V3>(fma(-k, 0.6931471805599453, x)), (int)k);
}
__device__ __forceinline__ XF xf_add(XF a, XF b) {
  if (a.m == 0.0) return b;
  if (b.m == 0.0) return a;
  const int e = a.e > b.e ? a.e : b.e;
  return xf_norm(ldexp(a.m, a.e - e) + ldexp(b.m, b.e - e), e);
}
__device__ __forceinline__ bool xf_gt(XF a, XF b) {   // a > b (both >= 0)
  if (a.m == 0.0) return false;
  if (b.m == 0.0) return true;
  return a.e != b.e ? a.e > b.e : a.m > b.m;
}
__device__ __forceinline__ bool xf_u_below(double u, XF a, XF b) {   // u < a / b
  if (b.m == 0.0) return false;   // Stan: u < exp(-inf - -inf) = NaN is false
  return ldexp(u * b.m, b.e - a.e) < a.m;
}
__device__ __forceinline__ double xf_val(XF a) { return ldexp(a.m, a.e); }


__device__ __forceinline__ void normal_pair(RngKey k, uint32_t c0, uint32_t c1, uint32_t c2,
                                            uint32_t c3, double& n0, double& n1) {
  U4 c = {c0, c1, c2, c3};
  U4 r = philox4x32_10(c, k.k0, k.k1);
  const double u1 = u53(r.x, r.y), u2 = u53(r.z, r.w);
  const double rad = sqrt(-2.0 * log(1.0 - u1));
  double sn, cs;
  sincospi(2.0 * u2, &sn, &cs);   // angle 2*pi*u2; sinpi/cospi need no Payne-Hanek reduction
  n0 = rad * cs;
  n1 = rad * sn;
}

// The sweep's arithmetic is contracted only where the source writes a * b + c as one
// expression (or calls fma): HIP's default, fast contraction across statements, let the
// backend fuse the same sweep differently in two kernel instantiations (the migrating and
// the plain sampler at 4 bins per lane, round 5), which broke the bitwise equality of
// their draws.  1 + a P(t) is written as an FMA (measured: hand-fusing the four per-bin sums
// as well costs config 5 7 %, scripts/gpu_r5_variants.sh); config 5 runs 1.7 % below the
// fast contraction, config 3 0.5 % (profiles/r05_ab_contract.txt).
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------
// per-bin arithmetic (the likelihood sweep)
// ---------------------------------------------------------------------------
template <class R> __device__ __forceinline__ R rcp_(R x);
template <> __device__ __forceinline__ double rcp_<double>(double x) {
  const double r = __builtin_amdgcn_rcp(x);    // v_rcp_f64 (quarter rate)
  const double e = fma(-x, r, 1.0);
  return fma(r, e, r);   // one Newton step: <= 1 ulp from 1/x (scripts/micro/acc.hip)
}
template <> __device__ __forceinline__ float rcp_<float>(float x) {
  return __builtin_amdgcn_rcpf(x);
}
template <class R> __device__ __forceinline__ R exp_(R x);
// exp for the sweep: reduction by ln2 (hi/lo), Taylor degree 12 on |r| <= ln2/2,
// ldexp.  n = round(x log2 e) comes from the 1.5*2^52 shifter (its low word is n
// as an int, fed straight to v_ldexp_f64: no v_rndne / v_cvt_i32_f64, the latter
// half rate).  x is clamped at -746 (below it exp is 0 either way, and the shifter
// needs |x log2 e| < 2^51); arguments here are <= 0, underflow ends in 0 via ldexp.
template <> __device__ __forceinline__ double exp_<double>(double x) {
  x = fmax(x, -746.0);
  const double SH = 6755399441055744.0;   // 1.5 * 2^52
  const double t = fma(x, 1.4426950408889634, SH);
  const double n = t - SH;
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
  double r = fma(-n, 6.93147180369123816490e-01, x);
  r = fma(-n, 1.90821492927058770002e-10, r);
  double p = 2.08767569878680989792e-09;   // 1/12!
  p = fma(p, r, 2.50521083854417187751e-08);
  p = fma(p, r, 2.75573192239858906526e-07);
  p = fma(p, r, 2.75573192239858906526e-06);
  p = fma(p, r, 2.48015873015873015873e-05);
  p = fma(p, r, 1.98412698412698412698e-04);
  p = fma(p, r, 1.38888888888888888889e-03);
  p = fma(p, r, 8.33333333333333333333e-03);
  p = fma(p, r, 4.16666666666666666667e-02);
  p = fma(p, r, 1.66666666666666666667e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, ni);
}
template <> __device__ __forceinline__ float exp_<float>(float x) { return __expf(x); }

// Estrin's scheme for sum_k c[k] t^k (k < N): pairs c[2j] + c[2j+1] t, then pairs of those
// with t^2, t^4, ...: dependency depth ceil(log2 N) + 1 FMAs instead of N - 1.
template <int N>
__device__ __forceinline__ double estrin(const double* c, double t) {
  constexpr int M = (N + 1) / 2;
  double v[M];
#pragma unroll
  for (int j = 0; j < M; ++j) v[j] = (2 * j + 1 < N) ? fma(c[2 * j + 1], t, c[2 * j]) : c[2 * j];
  double x = t * t;
#pragma unroll
  for (int n = M; n > 1; n = (n + 1) / 2) {
#pragma unroll
    for (int j = 0; j < n / 2; ++j) v[j] = fma(v[2 * j + 1], x, v[2 * j]);
    if (n & 1) v[n / 2] = v[n - 1];
    x = x * x;
  }
  return v[0];
}
// exp_<double>'s reduction and Taylor-12 polynomial, the polynomial by Estrin
__device__ __forceinline__ double exp_lat(double x) {
  x = fmax(x, -746.0);
  const double SH = 6755399441055744.0;   // 1.5 * 2^52
  const double t = fma(x, 1.4426950408889634, SH);
  const double n = t - SH;
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
  double r = fma(-n, 6.93147180369123816490e-01, x);
  r = fma(-n, 1.90821492927058770002e-10, r);
  constexpr double c[13] = {1.0, 1.0, 0.5, 1.66666666666666666667e-01,
                            4.16666666666666666667e-02, 8.33333333333333333333e-03,
                            1.38888888888888888889e-03, 1.98412698412698412698e-04,
                            2.48015873015873015873e-05, 2.75573192239858906526e-06,
                            2.75573192239858906526e-07, 2.50521083854417187751e-08,
                            2.08767569878680989792e-09};
  return ldexp(estrin<13>(c, r), ni);
}
// exp_ with a degree-11 polynomial: same reduction, one FMA fewer
__device__ __forceinline__ double exp11_(double x) {
  x = fmax(x, -746.0);
  const double SH = 6755399441055744.0;
  const double t = fma(x, 1.4426950408889634, SH);
  const double n = t - SH;
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, t);
  double r = fma(-n, 6.93147180369123816490e-01, x);
  r = fma(-n, 1.90821492927058770002e-10, r);
  // degree-11 Chebyshev fit on |r| <= ln2/2 (scripts/micro/exp_fit.py): <= 1 ulp from the
  // correctly rounded exp, one FMA fewer than Taylor-12
  double p = 2.5110037605963777e-08;
  p = fma(p, r, 2.763263963904103e-07);
  p = fma(p, r, 2.755724091857897e-06);
  p = fma(p, r, 2.4801485482328494e-05);
  p = fma(p, r, 0.00019841269890047113);
  p = fma(p, r, 0.0013888888952314775);
  p = fma(p, r, 0.008333333333319601);
  p = fma(p, r, 0.0416666666664881);
  p = fma(p, r, 0.1666666666666668);
  p = fma(p, r, 0.5000000000000019);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, ni);
}

// Likelihood terms of one bin given its modulation dL (shared by every mode).
// acc: [0] sum d^2, [1] sum a, [2] sum a e, [3] sum w; returns h (adjoint seed of dL).
// yi = y / uy is staged per bin (fitoct_api.cpp stage), so d = (y - m) / uy is one FMA,
// and c x / L is formed once for the exponent and the theta3 weight.
// The non-physical guard (1 + dL <= 0 -> lp = -inf) is a per-lane running min
// (umin), applied once after the lane's bins (no per-bin selects).
template <class R, class A, int NA>
__device__ __forceinline__ R bin_tail(R iL, R cx, R yi, R isu, R th1, R th2, A (&acc)[NA]) {
  const R ciL = cx * iL;                                         // c x / L
  R e;                                                           // exp(-c x / L)
  if constexpr (sizeof(R) == 8) e = exp11_(-ciL);
  else e = exp_<R>(-ciL);
  const R m = fma(th2, e, th1);                                  // ui.R:88
  const R d = fma(-m, isu, yi);                                  // (y-m)/uy
  const R a = d * isu;                                           // dlp/dm * sigma^2
  const R ae = a * e;
  const R w = ae * ciL;
  acc[0] += (A)(d * d);
  acc[1] += (A)a;
  acc[2] += (A)ae;
  acc[3] += (A)w;
  return w * iL;                                                 // dlp/ddL / (th2 th3) * sigma^2
}
template <class R, class A, int NA, bool LAT = false>
__device__ __forceinline__ R bin_core(R u, R cx, R yi, R isu, R th1, R th2, R th3, A (&acc)[NA],
                                      R& umin) {   // u = 1 + dL
  umin = fmin(umin, u);
  const R L = th3 * u;                                           // decay length theta3*(1+dL)
  const R iL = rcp_<R>(L);
  const R ciL = cx * iL;                                         // c x / L
  R e;                                                           // exp(-c x / L)
  if constexpr (LAT && sizeof(R) == 8) e = exp_lat(-ciL);
  else e = exp_<R>(-ciL);
  const R m = fma(th2, e, th1);                                  // ui.R:88
  const R d = fma(-m, isu, yi);                                  // (y-m)/uy
  const R a = d * isu;                                           // dlp/dm * sigma^2
  const R ae = a * e;
  const R w = ae * ciL;
  acc[0] += (A)(d * d);
  acc[1] += (A)a;
  acc[2] += (A)ae;
  acc[3] += (A)w;
  return w * iL;                                                 // dlp/ddL / (th2 th3) * sigma^2
}

// MODE_POLY: dL = a P(t) with P = sum_l c_l t^l ; moments M_l += h a t^l
template <class R, int NNP, class A>
__device__ __forceinline__ void bin_poly(R cx, R y, R isu, R t, R av, R th1, R th2, R th3,
                                         const R (&cf)[NNP], A (&acc)[4 + NNP], R& umin) {
  R P = cf[NNP - 1];
#pragma unroll
  for (int k = NNP - 2; k >= 0; --k) P = fma(P, t, cf[k]);
  const R h = bin_core<R, A, 4 + NNP>(fma(av, P, R(1)), cx, y, isu, th1, th2, th3, acc, umin);
  R p = h * av;
  acc[4] += (A)p;
#pragma unroll
  for (int l = 1; l < NNP; ++l) {
    p *= t;
    acc[4 + l] += (A)p;
  }
}

// MODE_POLY on a uniform grid: the forward half of bin_poly; returns w = h a,
// the bin's weight in the moments (accumulated per lane by moments_geo).
template <class R, int NNP, class A, bool LAT = false>
__device__ __forceinline__ R bin_poly_fwd(R cx, R y, R isu, R t, R av, R th1, R th2, R th3,
                                          const R (&cf)[NNP], A (&acc)[4 + NNP], R& umin) {
  R P;
  if constexpr (LAT && sizeof(R) == 8) {
    P = estrin<NNP>(cf, t);
  } else {
    P = cf[NNP - 1];
#pragma unroll
    for (int k = NNP - 2; k >= 0; --k) P = fma(P, t, cf[k]);
  }
  return bin_core<R, A, 4 + NNP, LAT>(fma(av, P, R(1)), cx, y, isu, th1, th2, th3, acc, umin) * av;
}

// Two bins of bin_poly_fwd sharing one reciprocal: 1/L0 = L1 / (L0 L1), 1/L1 = L0 / (L0 L1)
// (one quarter-rate v_rcp_f64 and its Newton step for two bins, <= 3 ulp).
template <class R, int NNP, class A>
__device__ __forceinline__ void bin_poly_fwd2(R cx0, R y0, R isu0, R t0, R a0, R cx1, R y1,
                                              R isu1, R t1, R a1, R th1, R th2, R th3,
                                              const R (&cf)[NNP], A (&acc)[4 + NNP], R& umin,
                                              R& w0, R& w1) {
  R P0 = cf[NNP - 1], P1 = cf[NNP - 1];
#pragma unroll
  for (int k = NNP - 2; k >= 0; --k) {
    P0 = fma(P0, t0, cf[k]);
    P1 = fma(P1, t1, cf[k]);
  }
  const R u0 = R(1) + a0 * P0, u1 = R(1) + a1 * P1;
  umin = fmin(umin, fmin(u0, u1));
  const R L0 = th3 * u0, L1 = th3 * u1;
  const R ip = rcp_<R>(L0 * L1);
  w0 = bin_tail<R, A, 4 + NNP>(ip * L1, cx0, y0, isu0, th1, th2, acc) * a0;
  w1 = bin_tail<R, A, 4 + NNP>(ip * L0, cx1, y1, isu1, th1, th2, acc) * a1;
}

// Moments of one lane's BPT bins t_b = t0 R^b:  M_l = t0^l sum_b w_b (R^l)^b.
// BPT-1 FMAs + 2 multiplies per moment instead of 2 operations per bin and moment.
template <int BPT, int NNP>
__device__ __forceinline__ void moments_geo(KPc& P, double t0, const double (&w)[BPT],
                                            double (&acc)[4 + NNP]) {
  double pw = 1.0;
#pragma unroll
  for (int l = 0; l < NNP; ++l) {
    const double X = P.geo_R[l];
    double S = w[BPT - 1];
#pragma unroll
    for (int b = BPT - 2; b >= 0; --b) S = fma(S, X, w[b]);
    acc[4 + l] = pw * S;
    pw *= t0;
  }
}

// The same for one 8-bin half of a 16-bin lane (BPT 16): M_l += t0^l sum_b w_b (R^l)^b.
template <int NB, int NNP>
__device__ __forceinline__ void moments_geo_add(KPc& P, double t0, const double (&w)[NB],
                                                double (&acc)[4 + NNP]) {
  double pw = 1.0;
#pragma unroll
  for (int l = 0; l < NNP; ++l) {
    const double X = P.geo_R[l];
    double S = w[NB - 1];
#pragma unroll
    for (int b = NB - 2; b >= 0; --b) S = fma(S, X, w[b]);
    acc[4 + l] = fma(pw, S, acc[4 + l]);
    pw *= t0;
  }
}

// MODE_ROWS / MODE_STREAM: dL = B_i . yGP ; (B^T h)_k += B_ik h
// LAT (f64, 1-2 bins per lane: a latency-bound sweep): exp by Estrin's scheme (config 5 at
// one GPU +7 %, config 2 +-0; the dot product in three FMA chains as well measured config 5
// +10 % but config 2 -1.8 %, alone config 5 -8 %: profiles/r06_ab_rows.txt)
template <class R, int NNP, class A, bool LAT = false>
__device__ __forceinline__ void bin_rows(R cx, R y, R isu, const R (&Brow)[NNP], R th1, R th2,
                                         R th3, const R (&yg)[NNP], A (&acc)[4 + NNP], R& umin) {
  R dL = R(0);
#pragma unroll
  for (int k = 0; k < NNP; ++k) dL = fma(Brow[k], yg[k], dL);
  const R h = bin_core<R, A, 4 + NNP, LAT>(R(1) + dL, cx, y, isu, th1, th2, th3, acc, umin);
#pragma unroll
  for (int k = 0; k < NNP; ++k) acc[4 + k] = fma((A)Brow[k], (A)h, acc[4 + k]);
}

// Transposed butterfly over the wave: 32 values x 64 lanes -> lane l holds the
// full sum of value (l >> 1).  Each step halves the live values: lanes whose
// step bit is set keep the upper half.  Bits 5 and 4 use the gfx950 permlane
// swaps (no select needed), bits 3..1 DPP row mirrors (partner differs in the
// step bit and below), the final pair a quad swap.
template <int H, int CTRL, int NV>
__device__ __forceinline__ void tr_dpp(double (&v)[NV], bool up) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const double send = up ? v[i] : v[i + H];
    const double keep = up ? v[i + H] : v[i];
    v[i] = keep + dpp<CTRL>(send);
  }
}
// The same transposed butterfly for 8 values (U-turn criteria): after it every
// lane of each 8-lane group holds the full sum of one value; returns whether all
// 8 sums are > 0 (one ballot).  ~3x fewer cross-lane steps than 8 butterflies.
__device__ __forceinline__ bool transpose_all_positive8(double (&v)[8], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = swap32_add(v[i], v[i + 4]);
#pragma unroll
  for (int i = 0; i < 2; ++i) v[i] = swap16_add(v[i], v[i + 2]);
  tr_dpp<1, DPP_MIRROR>(v, (lane & 8) != 0);
  double x = v[0];
  x += dpp<DPP_XOR1>(x);
  x += dpp<DPP_XOR2>(x);
  x += dpp<DPP_HALF_MIRROR>(x);
  const uint64_t ok = __builtin_amdgcn_ballot_w64(x > 0.0);
  return ok == __builtin_amdgcn_read_exec();
}

// The transposed butterfly for any NV <= 32 values: halves the live values per
// step (ceil), a missing partner counts as zero.  Returns the lane's total and,
// in idx, which value it is (-1: a padding lane).
template <int H, int N, int CTRL, int NV>
__device__ __forceinline__ void tr_dpp_n(double (&v)[NV], bool up) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    double send, keep;
    if (i + H < N) {
      send = up ? v[i] : v[i + H];
      keep = up ? v[i + H] : v[i];
    } else {
      send = up ? v[i] : 0.0;
      keep = up ? 0.0 : v[i];
    }
    v[i] = keep + dpp<CTRL>(send);
  }
}
template <int NV>
__device__ __forceinline__ double transpose_reduce(double (&v)[NV], int lane, int& idx) {
  constexpr int c1 = (NV + 1) / 2, c2 = (c1 + 1) / 2, c3 = (c2 + 1) / 2, c4 = (c3 + 1) / 2;
  constexpr int c5 = (c4 + 1) / 2;
  static_assert(NV <= 32 && c5 == 1, "transpose_reduce: at most 32 values");
#pragma unroll
  for (int i = 0; i < c1; ++i) v[i] = swap32_add(v[i], i + c1 < NV ? v[i + c1] : 0.0);
#pragma unroll
  for (int i = 0; i < c2; ++i) v[i] = swap16_add(v[i], i + c2 < c1 ? v[i + c2] : 0.0);
  tr_dpp_n<c3, c2, DPP_MIRROR>(v, (lane & 8) != 0);
  tr_dpp_n<c4, c3, DPP_HALF_MIRROR>(v, (lane & 4) != 0);
  tr_dpp_n<c5, c4, DPP_QREV>(v, (lane & 2) != 0);
  int i = (lane & 2) ? c5 : 0;
  bool ok = i < c4;
  i += (lane & 4) ? c4 : 0;
  ok = ok && i < c3;
  i += (lane & 8) ? c3 : 0;
  ok = ok && i < c2;
  i += (lane & 16) ? c2 : 0;
  ok = ok && i < c1;
  i += (lane & 32) ? c1 : 0;
  ok = ok && i < NV;
  idx = ok ? i : -1;
  return v[0] + dpp<DPP_XOR1>(v[0]);
}

// per-lane resident bin data
template <class R, int BPT, int NNP, int MODE>
struct Bins {
  static constexpr int NB = BPT > 0 ? BPT : 1;
  static constexpr int NR = MODE == MODE_POLY ? 2 : NNP;
  R cx[NB], y[NB], isu[NB];
  R row[NB][NR];
  __device__ void load(KPc& P, int tid) {
    if constexpr (BPT > 0) {
      const AS_GLB R* pcx = (const AS_GLB R*)P.cx;
      const AS_GLB R* py = (const AS_GLB R*)P.y;
      const AS_GLB R* pisu = (const AS_GLB R*)P.isu;
      const AS_GLB R* pB = (const AS_GLB R*)P.B;
      if constexpr (BPT == 16) {   // compact: y, 1/uy, a per bin; c*x and t of bin 0 only
        cx[0] = pcx[tid];
        row[0][0] = pB[2 * (size_t)tid];
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
          const int i = tid + b * GT;
          y[b] = py[i];
          isu[b] = pisu[i];
          row[b][1] = pB[2 * (size_t)i + 1];
        }
      } else {
#pragma unroll
        for (int b = 0; b < BPT; ++b) {
          const int i = tid + b * GT;
          cx[b] = pcx[i];
          y[b] = py[i];
          isu[b] = pisu[i];
#pragma unroll
          for (int k = 0; k < NR; ++k) row[b][k] = pB[(size_t)i * NR + k];
        }
      }
    }
  }
};

// LDS carve -----------------------------------------------------------------
// [ K^-1 (KMAX x KMAX, row stride NNP) | b (KMAX) | MP[GMAX][MPW] | PART[G][NGW][NSLOT] |
//   G x chain{ ChainScalars | NVEC vectors | SUMS[NSLOT] | AUX[NAUX] | levels[max_depth][NLVL] } ]
template <int PPL>
struct Lds {
  static constexpr int VLEN = WAVE * PPL;
  static constexpr int KBYTES = (KMAX * KMAX + KMAX) * 8;
  static __host__ __device__ constexpr int head_bytes(int G) {
    return KBYTES + (GMAX * MPW + NGW * G * NSLOT) * 8;
  }
  static __host__ __device__ constexpr int chain_bytes(int max_depth) {
    // ... | levels[max_depth][NLVL][VLEN] | merge-uniform rings[max_depth][WAVE]
    return (int)sizeof(ChainScalars) +
           (NVEC * VLEN + NSLOT + NAUX + max_depth * NLVL * VLEN + max_depth * WAVE) * 8;
  }
  // tiles of one or two chains (deep speculation): per chain, the booked leaf's q,
  // end-updated p, g, lp and sum r^2, handed from the chain's wave to its helper wave
  static constexpr int HX_BYTES = ((3 * VLEN + 2) * 8 + 15) / 16 * 16;
  // two-ended trajectories (G = 3 areas: the chain's, two producers'): per producer, two
  // slots for the leaves it hands its booking helper (q, end-updated p, g, lp, sum r^2, depth,
  // leaf, transition)
  static constexpr int PX_BYTES = ((3 * VLEN + 8) * 8 + 15) / 16 * 16;
  // ... and per end, two slots for its subtree records (Chain::rvec): 5 vectors, 16 scalars
  // (one parameter per lane; at two, whose chain areas leave less room, one record slot per
  // end in the producer's own area)
  static constexpr int QX_DOUBLES = 5 * VLEN + 16;
  static constexpr int QX_SLOTS = PPL == 1 ? 4 : 0;
  static __host__ __device__ constexpr int bytes(int G, int max_depth) {
    return head_bytes(G) + G * chain_bytes(max_depth) +
           (G <= 2 ? G * HX_BYTES : G == 3 ? 4 * PX_BYTES + QX_SLOTS * QX_DOUBLES * 8 : 0);
  }
  AS_LDS char* base;
  int G, cb;
  __device__ AS_LDS double* kinv() const { return (AS_LDS double*)base; }
  __device__ AS_LDS double* bv() const { return (AS_LDS double*)base + KMAX * KMAX; }
  __device__ AS_LDS double* mp(int c) const { return (AS_LDS double*)(base + KBYTES) + c * MPW; }
  __device__ AS_LDS double* part() const { return (AS_LDS double*)(base + KBYTES) + GMAX * MPW; }
  __device__ AS_LDS char* chain(int c) const { return base + head_bytes(G) + c * cb; }
  __device__ AS_LDS ChainScalars& cs(int c) const { return *(AS_LDS ChainScalars*)chain(c); }
  __device__ AS_LDS double* vecs(int c) const {
    return (AS_LDS double*)(chain(c) + sizeof(ChainScalars));
  }
  __device__ AS_LDS double* sums(int c) const { return vecs(c) + NVEC * VLEN; }
  __device__ AS_LDS double* aux(int c) const { return sums(c) + NSLOT; }
  __device__ AS_LDS double* lvls(int c) const { return aux(c) + NAUX; }
  // chain c's hand-off block (G <= 2)
  __device__ AS_LDS double* hx(int c = 0) const {
    return (AS_LDS double*)(base + head_bytes(G) + G * cb + c * HX_BYTES);
  }
  // producer s's hand-off slot k (two-ended trajectories, G = 3)
  __device__ AS_LDS double* px(int s, int k) const {
    return (AS_LDS double*)(base + head_bytes(G) + G * cb + (2 * s + k) * PX_BYTES);
  }
  // the record slots (end s, slot k = 2 s + k), after the hand-off slots
  __device__ AS_LDS double* qx0() const {
    return (AS_LDS double*)(base + head_bytes(G) + G * cb + 4 * PX_BYTES);
  }
};

// The likelihood sweep of chains [cb, ce) of the tile (gradient waves only).
// PART[c][wave][0 .. 4+NNP) receives this wave's partial sums of chain c.
// LATR: the row-mode sweep's latency form (bin_rows LAT); every sampler and the logp kernel
// use it, so all paths keep computing the same gradient bit for bit.
template <class R, int BPT, int NNP, int MODE, bool LATR = false>
__device__ void gradient_pass(KPc& P, const Bins<R, BPT, NNP, MODE>& bins,
                              const AS_LDS double* mpall, AS_LDS double* part, const int* done,
                              int cb, int ce,
                              int tid, int lane, int wave) {
  FITOCT_MARK(gradient_pass);
  for (int c = cb; c < ce; ++c) {
    if (done[c]) continue;   // wave-uniform (LDS broadcast)
    const AS_LDS double* mp = mpall + c * MPW;
    const R th1 = (R)mp[0], th2 = (R)mp[1], th3 = (R)mp[2];
    R cf[NNP];   // POLY: c_l = b_l (K^-1 yGP)_l ; ROWS: yGP_k
#pragma unroll
    for (int k = 0; k < NNP; ++k) cf[k] = (R)mp[4 + k];
    double acc[4 + NNP];
#pragma unroll
    for (int k = 0; k < 4 + NNP; ++k) acc[k] = 0.0;
    R umin = R(1);
    if constexpr (BPT == 16) {   // MODE_POLY f64 on an arithmetic grid (host-checked)
      double cx0 = bins.cx[0], t0 = bins.row[0][0];
      const double tmax = P.geo_tmax;
      // opaque per sweep: c*x_b and t_b are formed inside the sweep, as the compact layout
      // intends, instead of being hoisted out of the sweep loop (32 more live doubles)
      asm volatile("" : "+v"(cx0), "+v"(t0));
      // the lane's bins in groups of NQ (moments per group: NQ weights live at a time);
      // one reciprocal per bin (pairs sharing one measured 3 % slower here)
      constexpr int NQ = BPT16_GROUP;
#pragma unroll
      for (int q = 0; q < 16 / NQ; ++q) {
        double w[NQ];
#pragma unroll
        for (int b = 0; b < NQ; ++b) {
          const int bb = q * NQ + b;
          const double cxb = cx0 + P.geo_dcx[bb];
          const double tb = fmin(t0 * P.geo_R[bb], tmax);
          w[b] = bin_poly_fwd<R, NNP, double>(cxb, bins.y[bb], bins.isu[bb], tb,
                                              bins.row[bb][1], th1, th2, th3, cf, acc, umin);
        }
        moments_geo_add<NQ, NNP>(P, q ? t0 * P.geo_R[q * NQ] : t0, w, acc);
      }
    } else if constexpr (BPT > 0 && MODE == MODE_POLY && sizeof(R) == 8) {
      if (P.geo) {
        double w[BPT];
        // 8 bins per lane (the headline shape, N = 2048): bins in pairs sharing one
        // reciprocal, exp by a degree-11 polynomial (A/B: config 3 +1.7 %, configs 2 / 5
        // within noise; at 16 bins the pairs spill)
        if constexpr (BPT == 8) {
#pragma unroll
          for (int b = 0; b < BPT; b += 2)
            bin_poly_fwd2<R, NNP, double>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b][0],
                                          bins.row[b][1], bins.cx[b + 1], bins.y[b + 1],
                                          bins.isu[b + 1], bins.row[b + 1][0], bins.row[b + 1][1],
                                          th1, th2, th3, cf, acc, umin, w[b], w[b + 1]);
        } else {
          // sweeps of at most 2 bins per lane (N <= 512: configs 2 and 5) are latency-bound:
          // the basis polynomial and exp by Estrin's scheme (config 5 +1.8 %)
          constexpr bool LAT = BPT <= 2;
#pragma unroll
          for (int b = 0; b < BPT; ++b)
            w[b] = bin_poly_fwd<R, NNP, double, LAT>(bins.cx[b], bins.y[b], bins.isu[b],
                                                     bins.row[b][0], bins.row[b][1], th1, th2,
                                                     th3, cf, acc, umin);
        }
        moments_geo<BPT, NNP>(P, bins.row[0][0], w, acc);
      } else {
#pragma unroll
        for (int b = 0; b < BPT; ++b)
          bin_poly<R, NNP, double>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b][0],
                                   bins.row[b][1], th1, th2, th3, cf, acc, umin);
      }
    } else if constexpr (BPT > 0 && MODE == MODE_POLY) {
#pragma unroll
      for (int b = 0; b < BPT; ++b)
        bin_poly<R, NNP, double>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b][0],
                                 bins.row[b][1], th1, th2, th3, cf, acc, umin);
    } else if constexpr (BPT > 0) {
      // the few bins of one lane accumulate in R, the lane totals in f64
      constexpr bool ROWS_LAT = LATR && sizeof(R) == 8 && BPT <= 2;
      R racc[4 + NNP];
#pragma unroll
      for (int k = 0; k < 4 + NNP; ++k) racc[k] = R(0);
#pragma unroll
      for (int b = 0; b < BPT; ++b)
        bin_rows<R, NNP, R, ROWS_LAT>(bins.cx[b], bins.y[b], bins.isu[b], bins.row[b], th1, th2,
                                      th3, cf, racc, umin);
#pragma unroll
      for (int k = 0; k < 4 + NNP; ++k) acc[k] = (double)racc[k];
    } else {
      const AS_GLB R* pcx = (const AS_GLB R*)P.cx;
      const AS_GLB R* py = (const AS_GLB R*)P.y;
      const AS_GLB R* pisu = (const AS_GLB R*)P.isu;
      const AS_GLB R* pB = (const AS_GLB R*)P.B;
      for (int i = tid; i < P.n_pad; i += GT) {
        if constexpr (MODE == MODE_POLY) {
          bin_poly<R, NNP, double>(pcx[i], py[i], pisu[i], pB[2 * (size_t)i], pB[2 * (size_t)i + 1],
                                   th1, th2, th3, cf, acc, umin);
        } else {
          R row[NNP];
#pragma unroll
          for (int k = 0; k < NNP; ++k) row[k] = pB[(size_t)i * NNP + k];
          bin_rows<R, NNP, double>(pcx[i], py[i], pisu[i], row, th1, th2, th3, cf, acc, umin);
        }
      }
    }
    if (!(umin > R(0))) acc[0] = INFINITY;   // some bin has 1 + dL <= 0: lp = -inf
    int idx;
    FITOCT_MARK(sweep_reduce);
    const double r = transpose_reduce<4 + NNP>(acc, lane, idx);
    if (!(lane & 1) && idx >= 0) part[(c * NGW + wave) * NSLOT + idx] = r;
  }
}

// (end of the sweep's arithmetic: the sampler's code below keeps HIP's default contraction)
#pragma clang fp contract(fast)

// ---------------------------------------------------------------------------
// the chain (one wave; lane = parameter)
// ---------------------------------------------------------------------------
template <int PPL>
struct Vd {
  double a[PPL];
};

// MIG = false: a sampler built without chain migration (plans where it cannot
// run: one chain per tile, batch mode, FITOCT_NO_MIGRATE), so the receive loop
// and the donor check cost no registers in the NUTS waves
// SPEC = true: speculative leaves with a helper wave (one chain per tile, no migration)
// MODE_: the kernel's basis mode (MODE_POLY / MODE_ROWS) as a constant, or -1: read P.mode
template <int PPL, int NNP, int FAM, bool MIG = true, bool SPEC = false, int MODE_ = -1>
struct Chain {
  using V = Vd<PPL>;
  static constexpr int VLEN = WAVE * PPL;
  KPc* pp;   // laundered once per action: no kernarg load is hoisted across actions
  AS_LDS ChainScalars* Sp;
  AS_LDS double* Vb;
  AS_LDS double* SUMS;
  AS_LDS double* AUX;   // [0,32): yGP ; [32,64): horseshoe lambda_j * tau
  AS_LDS double* LV;    // [max_depth][NLVL][VLEN]
  AS_LDS double* RNG;   // [max_depth][WAVE]: level l's merge uniforms, one block of 64 merges
  AS_LDS double* MP;
  AS_LDS double* part;
  const AS_LDS double* Kinv;
  // this lane's row of K^-1 (lanes < NNP) held in VGPRs for the two K^-1 matvecs
  // of every leaf (write_mp, finish_grad): same arithmetic, no LDS reads on the
  // NUTS wave's critical path (configs 2 / 5 +2 %).  Not at NNP = 24 (it would spill).
  static constexpr bool KROW = NNP <= 16 && !MIG && MODE_ != MODE_ROWS;
  // fexp's Horner steps as three-VGPR FMAs (fma_v) in the non-migrating samplers: bitwise
  // the same, configs 2 / 5 +2 / +0.6 %.  The migrating samplers then spill a VGPR (the
  // headline horseshoe one loses 2.2 %, profiles/r03_ab_fmav.txt): they keep the compiler's form
  static constexpr bool FV3 = !MIG;
  double krow[KROW ? NNP : 1];
  const AS_LDS double* bv;
  int lane, slot, lc, gid, nct;
  int pix;   // proposal pool region: the chain's (lc); a two-ended producer's own (produce)
  // speculative leaves (the SPEC sampler): always in a tile of one chain (with a helper
  // wave), else while the tile hosts <= P.spec_live live chains (the tail of a launch, when
  // the sweep no longer hides the sampler's latency; this wave then does the helper's part)
  static constexpr bool spec = SPEC;
  bool helped;   // ... with a helper wave (tiles of one or two chains, no migration)
  const AS_LDS int* live = nullptr;   // the tile's live-chain count (kernel-maintained)
  // a speculated leaf's values, kept from leaf_spec to act_spec_book (across the hand-off)
  // (the metric and the next subtree's start are re-read from LDS.)  The migrating
  // sampler, whose migration paths leave no registers to spare, also parks the leaf itself
  // in LDS, in slots dead from leaf_spec to the end of the bookkeeping: q in V_PG and g in
  // V_CA (there is no helper wave, so the next prior part is written only after the
  // bookkeeping), the end-updated p in V_CUR_G (where spec_weight reads it anyway).  No
  // LDS is added: the tile's LDS carve decides how many chains fit (G = 4 at depth 12).
  static constexpr bool KLDS = MIG;
  V k_q, k_pe, k_g;
  // (its lp / sum r^2 stay in Sp->cur_lp / cur_s2 until the bookkeeping)
  int k_dirn, k_dn, k_jn;
  uint32_t k_t;
  // deep speculation (tiles of one or two chains, helped): the helper books leaf k
  // (deep_book) while this wave completes gradient k + 1; this wave waits for booking k
  // (book_done >= book_want) only before it stages leaf k + 2, and reads its outcome from
  // book_res
  bool deep = false;
  AS_LDS double* HX = nullptr;
  volatile AS_LDS int* book_done = nullptr;
  volatile AS_LDS int* book_res = nullptr;
  int book_want = 0;
  // two-ended trajectories (P.bidi, deep tiles): the producer waves' chain areas (slots 1, 2:
  // backward, forward) and the tile's hand-off words BD_*
  // Compiled where it can run: tiles of one chain (deep speculation, spare waves from the
  // start), and migrating tiles in the launch's tail (a chain alone in its tile, with two
  // idle receivers recruited as producers: kernel and receive_chain, P.tail_bidi)
  static constexpr bool kTwoEnded = SPEC;
  bool bidi = false;
  volatile AS_LDS int* bd = nullptr;
  RngKey key;

  __device__ __forceinline__ Chain(KPc& P_, const Lds<PPL>& L, int slot_, int lc_, int lane_, int nct_)
      : pp(&P_), Sp(&L.cs(slot_)), Vb(L.vecs(slot_)), SUMS(L.sums(slot_)), AUX(L.aux(slot_)),
        LV(L.lvls(slot_)), RNG(L.lvls(slot_) + (size_t)P_.max_depth * NLVL * VLEN), MP(L.mp(slot_)),
        part(L.part()), Kinv(L.kinv()), bv(L.bv()),
        lane(lane_), slot(slot_), lc(lc_), nct(nct_) {
    gid = Pr().chain_offset + lc;
    pix = lc;
    // tiles of G <= 2 chains: NUTS wave G + c helps chain slot c (tile of one chain: wave 1)
    helped = SPEC && !MIG && P_.G <= 2;
    deep = helped;
    HX = L.hx(L.G <= 2 ? slot_ : 0);
    if (L.G == 3) QX0 = L.qx0();
    bidi = kTwoEnded && !MIG && deep && P_.bidi != 0;
    key = make_key(Pr().seed, (uint32_t)gid);
    if constexpr (KROW) {
      const int r = lane < NNP ? lane : 0;
#pragma unroll
      for (int k = 0; k < NNP; ++k) krow[k] = Kinv[r * NNP + k];
    }
  }
  __device__ __forceinline__ double kinv_row(int k) const {
    if constexpr (KROW) return krow[k];
    else return Kinv[lane * NNP + k];
  }

  __device__ __forceinline__ KPc& Pr() const { return *pp; }
  __device__ __forceinline__ bool is_poly() const {
    return MODE_ >= 0 ? MODE_ == MODE_POLY : Pr().mode == MODE_POLY;
  }
  // two-ended trajectories: producer k's chain area (NUTS slot bd[TW_SLOT + k] of this
  // tile: the chain areas are consecutive, chain_bytes apart), its scalars and vectors
  __device__ __forceinline__ AS_LDS char* parea(int k) const {
    const int sl = __builtin_amdgcn_readfirstlane(bd[TW_SLOT + k]);
    return (AS_LDS char*)Sp + (sl - slot) * Lds<PPL>::chain_bytes(Pr().max_depth);
  }
  __device__ __forceinline__ AS_LDS ChainScalars* psp(int k) const {
    return (AS_LDS ChainScalars*)parea(k);
  }
  __device__ __forceinline__ AS_LDS double* pvb(int k) const {
    return (AS_LDS double*)(parea(k) + sizeof(ChainScalars));
  }
  __device__ __forceinline__ int idx(int s) const { return s * WAVE + lane; }
  __device__ __forceinline__ bool ok(int s) const { return idx(s) < Pr().D; }
  __device__ __forceinline__ AS_LDS double* vec(int v) const { return Vb + v * VLEN; }
  __device__ __forceinline__ const AS_LDS double* QS() const { return Vb + V_QS * VLEN; }
  __device__ __forceinline__ const AS_LDS double* QE() const { return Vb + V_QE * VLEN; }
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
  __device__ __forceinline__ void copyv(int dst, int src) const { st(dst, ld(src)); }
  __device__ __forceinline__ AS_LDS double* lvl(int level, int which) const {
    return LV + ((size_t)level * NLVL + which) * VLEN;
  }
  __device__ __forceinline__ V lld(int level, int which) const {
    V r;
    const AS_LDS double* p = lvl(level, which);
#pragma unroll
    for (int s = 0; s < PPL; ++s) r.a[s] = p[idx(s)];
    return r;
  }
  __device__ __forceinline__ void lst(int level, int which, const V& x) const {
    AS_LDS double* p = lvl(level, which);
#pragma unroll
    for (int s = 0; s < PPL; ++s) p[idx(s)] = x.a[s];
  }
  __device__ __forceinline__ AS_GLB double* pslot(int sl, int which) const {
    // HBM [chain][max_depth+1][NPOOL][VLEN]; recomputed from the parameter block
    // on use (scalar ops) instead of holding a 64-bit pointer across actions
    const size_t base = ((size_t)pix * (Pr().max_depth + 1) + sl) * NPOOL + which;
    return (AS_GLB double*)Pr().stack + base * VLEN;
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
  // three compute_criterion calls of one merge, reduced together (6 dot products
  // in one interleaved butterfly; the conjunction is order-independent)
  __device__ __forceinline__ bool crit3(const V& a1, const V& b1, const V& r1, const V& a2,
                                        const V& b2, const V& r2, const V& a3, const V& b3,
                                        const V& r3, const V& minv) const {
    // slots 6, 7 pad the transposed reduction with a positive constant (lane 0)
    double x[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, lane == 0 ? 1.0 : 0.0, lane == 0 ? 1.0 : 0.0};
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      x[0] += minv.a[s] * b1.a[s] * r1.a[s];
      x[1] += minv.a[s] * a1.a[s] * r1.a[s];
      x[2] += minv.a[s] * b2.a[s] * r2.a[s];
      x[3] += minv.a[s] * a2.a[s] * r2.a[s];
      x[4] += minv.a[s] * b3.a[s] * r3.a[s];
      x[5] += minv.a[s] * a3.a[s] * r3.a[s];
    }
    return transpose_all_positive8(x, lane);
  }
  __device__ __forceinline__ bool is_log(int k) const { return k < 3 || k >= 3 + Pr().Nn; }

  // ---------------- the point handed to the gradient phase ------------------
  // Stages q, caches its constrained values (QE) and, per family, yGP and the
  // horseshoe scales (AUX), then writes the gradient phase's parameters MP:
  // theta[3] and, per basis mode, yGP (rows) or c = b .* K^-1 yGP (poly).
  // (LDS exchange: on gfx950 a v_readlane assembly of yGP measured 3x slower.)
  __device__ void write_mp(const V& q) const {
    FITOCT_MARK(write_mp);
    long long ts = stamp0();
    const int Nn = Pr().Nn, D = Pr().D;
    const bool poly = is_poly();
    AS_LDS double* qs = vec(V_QS);
    AS_LDS double* qe = vec(V_QE);
#pragma unroll
    for (int s = 0; s < PPL; ++s) qs[idx(s)] = q.a[s];
    wave_order();   // q of every lane visible: the yGP lanes start at once, in parallel with
                    // the constrained values below
    double yv = 0.0, hl = 0.0, u = 0.0;
    const int jl = lane < Nn ? lane : 0;
    if (FAM == FAM_HORSESHOE) {
      // Tests/horseShoePrior.stan:30-32 in the exponent: lambda_j tau =
      // r1_l sqrt(r2_l) r1_g sqrt(r2_g) = exp(u1_l + u2_l/2 + u1_g + u2_g/2)
      const double a1 = qs[5 + Nn + jl], a2 = qs[5 + 2 * Nn + jl];
      const double g1 = qs[3 + Nn], g2 = qs[4 + Nn];
      u = qs[3 + jl];
      hl = fexp<FV3>(fma(0.5, a2, a1) + fma(0.5, g2, g1));
    } else {
      u = qs[3 + jl];
    }
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      const double ev = (k < D && is_log(k)) ? fexp<FV3>(q.a[s]) : q.a[s];
      qe[k] = ev;
      if (s == 0 && lane < 3) MP[lane] = ev;   // theta for the gradient waves
    }
    yv = (FAM == FAM_HORSESHOE) ? u * hl : u;
    if (lane >= Nn) yv = hl = 0.0;
    if (lane < NNP) {
      AUX[lane] = yv;
      AUX[32 + lane] = hl;
      if (!poly) MP[4 + lane] = yv;
    }
    sub(5, ts);
    if (poly) {  // c_l = b_l (K^-1 yGP)_l ; K^-1 padded to NNP x NNP
      wave_order();
      if (lane < NNP) {
        double c0 = 0.0, c1 = 0.0;   // two chains of FMAs: half the dependent latency
#pragma unroll
        for (int k = 0; k + 1 < NNP; k += 2) {
          c0 = fma(kinv_row(k), AUX[k], c0);
          c1 = fma(kinv_row(k + 1), AUX[k + 1], c1);
        }
        if constexpr ((NNP & 1) != 0) c0 = fma(kinv_row(NNP - 1), AUX[NNP - 1], c0);
        MP[4 + lane] = (c0 + c1) * bv[lane];
      }
    }
    sub(6, ts);
  }

  // The lp / grad completion is split so that everything depending only on the
  // staged position runs while the gradient waves sweep the bins (prior_part,
  // off the critical path), and only a few FMAs per lane remain once the bin
  // sums arrive (lik_part):
  //   grad_k = PG_k + CA_k * S[sidx(k)] + CB_k * famsum,   lp = pr_lp - 0.5 S0 pr_is2
  // with S = the bin sums after finish_grad's transform and famsum = sum_j FW_j S[4+j].
  __device__ __forceinline__ int sidx(int k) const {   // which bin sum lane k's gradient needs
    const int D = Pr().D, Nn = Pr().Nn;
    if (k < 3) return 1 + k;
    if (k == D - 1) return 0;
    if (k < 3 + Nn) return 4 + (k - 3);
    if (FAM == FAM_HORSESHOE && k >= 5 + Nn) return 4 + ((k - 5 - Nn) % Nn);
    return 0;
  }

  __device__ void prior_part() const {
    FITOCT_MARK(prior_part);
    const int D = Pr().D, Nn = Pr().Nn;
    constexpr int fam = FAM;
    const AS_LDS double* qs = QS();
    const AS_LDS double* qe = QE();
    const bool lik = (Pr().prior_PD == 0);
    constexpr bool mono = FAM == FAM_MONO;   // flat theta prior, sigma = 1 (fitMonoExp)
    const double th0 = qe[0], th1 = qe[1], th2 = qe[2];
    const double usig = mono ? 0.0 : qs[D - 1], sig = mono ? 1.0 : qe[D - 1];
    const double is2 = mono ? 1.0 : frcp(sig * sig);
    const double d0 = mono ? 0.0 : th0 - Pr().theta0[0], d1 = mono ? 0.0 : th1 - Pr().theta0[1],
                 d2 = mono ? 0.0 : th2 - Pr().theta0[2];
    const AS_CST double* Si = Pr().S0inv;
    const double Sd0 = Si[0] * d0 + Si[1] * d1 + Si[2] * d2;
    const double Sd1 = Si[3] * d0 + Si[4] * d1 + Si[5] * d2;
    const double Sd2t = Si[6] * d0 + Si[7] * d1 + Si[8] * d2;
    const double iss = Pr().sigma_scale_inv;   // 1 / sigma_scale (host division)
    const double gyf = lik ? th1 * th2 * is2 : 0.0;   // dlp/dyGP_k = gyf * S[4+k]
    // mono-exp with theta_prior = 1: theta_k ~ exponential(tr) (Tests/testGamma.R's model)
    const double tr = mono ? Pr().theta_rate : 0.0;
    double lpc = 0.0;
    if (lane == 0) {
      if (lik) lpc += -(double)Pr().N * usig;
      lpc += -0.5 * (d0 * Sd0 + d1 * Sd1 + d2 * Sd2t) + qs[0] + qs[1] + qs[2];
      if (mono) lpc += -tr * (th0 + th1 + th2);
      if (!mono) lpc += -0.5 * (sig * iss) * (sig * iss) + usig;
    }
    double ysum = 0.0;   // normal family: sum yGP^2
    if (fam == FAM_NORMAL) ysum = wave_sum(lane < Nn ? AUX[lane] * AUX[lane] : 0.0);
    if (fam == FAM_HORSESHOE && lane < Nn) AUX[64 + lane] = gyf * AUX[lane];   // FW_j
    V pg, ca;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double gk = 0.0, ck = 0.0;
      if (k < D) {
        const double qk = qs[k];
        if (k < 3) {
          const double thk = (k == 0) ? th0 : (k == 1) ? th1 : th2;
          const double sdk = (k == 0) ? Sd0 : (k == 1) ? Sd1 : Sd2t;
          gk = 1.0 - thk * sdk;
          if (mono) gk -= tr * thk;
          if (lik) ck = (k == 2) ? th1 * is2 : thk * is2;
        } else if (mono) {
          // no other parameter
        } else if (k == D - 1) {
          gk = (lik ? -(double)Pr().N : 0.0) - (sig * iss) * (sig * iss) + 1.0;
          if (lik) ck = is2;
        } else if (fam == FAM_NORMAL) {
          // one reciprocal for the wave (lambda is the same on every lane) instead of an
          // IEEE division per term: no division latency on the sampler's path
          const double lam = qe[3 + Nn], il2 = frcp(lam * lam);
          if (k < 3 + Nn) {
            gk = -qk * il2;
            ck = gyf;
            lpc += -0.5 * qk * qk * il2;
          } else {  // lambda: lam * (-Nn / lam + ysum / lam^3 - rate) + 1
            const double rate = Pr().lambda_rate_eff;
            gk = -(double)Nn + ysum * il2 - rate * lam + 1.0;
            lpc += -(double)Nn * qk - rate * lam + qk;
          }
        } else if (fam == FAM_LASSO) {
          const double ls = Pr().lambda_scale;
          const double sg = (qk > 0.0) ? 1.0 : (qk < 0.0) ? -1.0 : 0.0;
          gk = -ls * sg - 2.0 * ls * qk;
          ck = gyf;
          lpc += -ls * fabs(qk) - ls * qk * qk;
        } else {  // horseshoe (Tests/horseShoePrior.stan:25-43), straight-line over lanes:
          //   z_j      : grad -q              lp -q^2/2
          //   r1 (g, l): grad 1 - e^2         lp -e^2/2 + q          (half-normal + log-Jacobian)
          //   r2 (g, l): grad c (1/e - 1)     lp -c (q + 1/e)        (InvGamma(c, c) + log-Jacobian,
          //                                                         c = 1/2 global, nu/2 local)
          const double ek = qe[k];
          const bool tz = k < 3 + Nn;
          const bool r1l = k >= 5 + Nn && k < 5 + 2 * Nn, r2l = k >= 5 + 2 * Nn;
          const bool tr1 = k == 3 + Nn || r1l;
          const double cc = (k == 4 + Nn) ? 0.5 : 0.5 * Pr().nu;
          const double e2 = ek * ek, ie = frcp(ek);
          gk = tz ? -qk : tr1 ? 1.0 - e2 : cc * ie - cc;
          lpc += tz ? -0.5 * qk * qk : tr1 ? fma(-0.5, e2, qk) : -cc * (qk + ie);
          const int ai = tz ? 32 + (k - 3) : r1l ? k - 5 - Nn : r2l ? k - 5 - 2 * Nn : 0;
          const double aw = (tz || r1l) ? 1.0 : r2l ? 0.5 : 0.0;
          ck = aw * gyf * AUX[ai];
        }
      }
      pg.a[s] = gk;
      ca.a[s] = ck;
    }
    st(V_PG, pg);
    st(V_CA, ca);
    const double lp = wave_sum(lpc);
    if (lane == 0) {
      Sp->pr_lp = lp;
      Sp->pr_is2 = lik ? is2 : 0.0;
    }
  }

  // After the sweep: reduce the 8 waves' partial sums and complete lp / grad from
  // what prior_part left in LDS.  s0 = sum of squared residuals.  Two LDS round
  // trips: bin sums out (-> the K^-1 transform), transformed sums out (-> every
  // parameter lane); famsum is reduced straight from the transform's lanes.
  __device__ double finish_grad(V& g, double& s0) const {
    FITOCT_MARK(finish_grad);
    const int Nn = Pr().Nn, D = Pr().D;
    const bool lik = (Pr().prior_PD == 0), poly = is_poly();
    const V pg = ld(V_PG), ca = ld(V_CA);   // issued up front, used last
    const double pr_lp = Sp->pr_lp, pr_is2 = Sp->pr_is2;
    const double fw = (FAM == FAM_HORSESHOE && lane < Nn) ? AUX[64 + lane] : 0.0;
    double famsum = 0.0, S0 = 0.0;
    double srow[PPL];   // basis rows (MODE_ROWS): the bin sum each lane's gradient needs
#pragma unroll
    for (int s = 0; s < PPL; ++s) srow[s] = 0.0;
    if (lik && !poly) {
      // each lane sums the partials of the sums it needs itself, in the SUMS path's order
      // (bitwise the same values): no store / wait / read-back before the gradient
      const AS_LDS double* pw = part + slot * NGW * NSLOT;
      double v = 0.0;
      const int jv = lane < NNP ? 4 + lane : 0;
#pragma unroll
      for (int w = 0; w < NGW; ++w) {
        S0 += pw[w * NSLOT];
        if (FAM == FAM_HORSESHOE) v += pw[w * NSLOT + jv];
#pragma unroll
        for (int s = 0; s < PPL; ++s) srow[s] += pw[w * NSLOT + sidx(idx(s))];
      }
      if (FAM == FAM_HORSESHOE) famsum = wave_sum(lane < Nn ? fw * v : 0.0);
    } else if (lik) {
      double sl = 0.0;
      if (lane < 4 + NNP) {
#pragma unroll
        for (int w = 0; w < NGW; ++w) sl += part[(slot * NGW + w) * NSLOT + lane];
        if (poly && lane >= 4) sl *= bv[lane - 4];   // b .* M  (B^T h = K^-1 (b .* M))
        SUMS[lane] = sl;
      }
      S0 = rl(sl, 0);
      wave_order();
      double v = 0.0;
      if (lane < NNP) {
        if (poly) {
          double v1 = 0.0;
#pragma unroll
          for (int m = 0; m + 1 < NNP; m += 2) {
            v = fma(kinv_row(m), SUMS[4 + m], v);
            v1 = fma(kinv_row(m + 1), SUMS[4 + m + 1], v1);
          }
          if constexpr ((NNP & 1) != 0) v = fma(kinv_row(NNP - 1), SUMS[4 + NNP - 1], v);
          v += v1;
          SUMS[4 + lane] = v;   // every lane's reads above precede this store
        } else {
          v = SUMS[4 + lane];
        }
      }
      if (FAM == FAM_HORSESHOE) famsum = wave_sum(lane < Nn ? fw * v : 0.0);
      wave_order();
    }
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double gk = pg.a[s];
      if (lik && k < D) {
        gk = fma(ca.a[s], poly ? SUMS[sidx(k)] : srow[s], gk);
        if (FAM == FAM_HORSESHOE && (k == 3 + Nn || k == 4 + Nn))
          gk = fma(k == 3 + Nn ? 1.0 : 0.5, famsum, gk);
      }
      g.a[s] = gk;
    }
    s0 = lik ? S0 : NAN;
    double lp = fma(-0.5 * S0, pr_is2, pr_lp);
    if ((lik && !(S0 <= DBL_MAX)) || !(fabs(lp) <= DBL_MAX)) lp = -INFINITY;
    return lp;
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
      p.a[s] = (k < Pr().D) ? n / sqrt(minv.a[s]) : 0.0;
    }
    return p;
  }

  // =========================================================================
  // The sampler as a flat action machine.  Every action appears once in the
  // code and returns the next action; A_YIELD hands the position staged by
  // A_WRITE_MP to the gradient waves.  Values crossing actions live in LDS.
  // =========================================================================
  enum Act : int {
    A_YIELD = 0, A_GRAD, A_INIT_STATE, A_INIT_START, A_INIT_STEP, A_SS_BEGIN, A_SS_TRIAL,
    A_SS_STEP, A_SS_FINISH, A_START_TRANSITION, A_BEGIN_SUBTREE, A_LEAF, A_END_TREE,
    A_NEXT_TRANSITION, A_FINISH, A_LEAPFROG, A_WRITE_MP, A_PRIOR,
    // the speculative path (leaf_spec): A_SPEC_STAGED yields a staged position for the
    // kernel to enqueue and hand to the helper wave, A_SPEC_BOOK then does the leaf's
    // bookkeeping and yields A_SPEC_WAIT (wait for the sweep and the helper, then A_GRAD)
    // or A_SPEC_DISCARD (the trajectory ended: drain both, then A_END_TREE)
    A_SPEC_STAGED, A_SPEC_BOOK, A_SPEC_WAIT, A_SPEC_DISCARD,
    // two-ended trajectories: the producers and the helper grow and book the whole tree;
    // the chain's wave waits for its end, then A_END_TREE
    A_BIDI_TREE
  };
  enum LeafBook : int { LB_MID = 0, LB_NEXT = 1, LB_END = 2 };

  __device__ __forceinline__ int uni(int x) const { return __builtin_amdgcn_readfirstlane(x); }
  // diagnostic sub-action stamps (profiling build + FITOCT_STAMPS): cycles since t
  // into prof[0][20 + i]
  __device__ __forceinline__ void sub(int i, long long& t) const {
    if (kProfile && Pr().stamps) {
      wave_fence();
      const long long n = (long long)__builtin_amdgcn_s_memtime();
      if (lane == 0) Sp->prof[0][20 + i] += n - t;
      t = n;
    }
  }
  __device__ __forceinline__ long long stamp0() const {
    return (kProfile && Pr().stamps) ? (long long)__builtin_amdgcn_s_memtime() : 0;
  }

  // runs while the gradient waves sweep the staged position: the position-only
  // part of lp / grad, and the uniforms the coming leaf's merges will consume
  __device__ int act_prior() {
    FITOCT_MARK(act_prior);
    const bool tree = uni(Sp->state) == ST_TREE;
    if (deep) {   // the tree uniforms are the booking helper's (it owns the rings and Sp->leaf)
      prior_part();
      return A_YIELD;
    }
    prior_and_uniforms(tree, uni(Sp->depth), uni(Sp->leaf), (uint32_t)uni(Sp->t));
    return A_YIELD;
  }
  // The position-only part of lp / grad, and (tree building, leaf j of the subtree of
  // depth d) the uniforms that leaf's merges will consume.  Run by the chain's NUTS
  // wave (A_PRIOR) or, for a speculated leaf, by the tile's helper wave.
  __device__ void prior_and_uniforms(const bool tree, const int d, const int j,
                                     const uint32_t t) const {
    long long ts = stamp0();
    prior_part();
    sub(7, ts);
    if (tree) tree_uniforms(d, j, t);
  }
  // the uniforms leaf j of the subtree of depth d will consume in its merges (and the
  // top-level merge's, for the subtree's last leaf)
  __device__ void tree_uniforms(const int d, const int j, const uint32_t t) const {
    {
      // Leaf j completes the merges of levels l < nm (trailing ones of j).
      // The k-th level-l merge of a subtree sits at leaf (k + 1) 2^(l+1) - 1; each
      // level keeps a ring of the uniforms of 64 consecutive merges, refilled a block
      // at a time by one Philox per lane (same counters as one draw per merge, so the
      // same numbers), i.e. one Philox pass per 64 merges instead of per leaf.
      const int nm = min(d, (int)__builtin_ctz(~(unsigned)j));
      for (int l = 0; l < nm; ++l) {
        const int blk = (j >> (l + 1)) >> 6;
        if (uni(Sp->u_blk[l]) != blk) {
          const int jj = ((((blk << 6) + lane) + 1) << (l + 1)) - 1;   // may pass the subtree's end: unused
          RNG[l * WAVE + lane] = uniform(key, t, TAG_MERGE | ((uint32_t)l << 8) | ((uint32_t)d << 16),
                                         (uint32_t)jj, 0u);
          if (lane == 0) Sp->u_blk[l] = blk;
        }
      }
      if (lane == WAVE - 1 && j == (1 << d) - 1)
        Sp->u_top = uniform(key, t, TAG_TOP, (uint32_t)d, 0u);
    }
  }

  // a gradient arrived for CUR_Q: complete lp / grad, store them, dispatch
  __device__ int act_grad() {
    FITOCT_MARK(act_grad);
    long long ts = stamp0();
    const int stt = uni(Sp->state);
    V g;
    double s0;
    if (stt == ST_TREE) {
      // the leaf's position, momentum and the metric are read while the bin sums reduce
      const V q = ld(V_CUR_Q), p = ld(V_CUR_P), minv = ld(V_MINV);
      const double lp = finish_grad(g, s0);
      sub(4, ts);
      st(V_CUR_G, g);
      Sp->cur_lp = lp;
      Sp->cur_s2 = s0;
      if constexpr (spec) {   // per leaf: plain and speculative leaves leave the same state
        if (deep) {
          // leaf k - 1 is being booked by the helper: its outcome decides whether this leaf
          // belongs to the trajectory, and it sets the tree coordinates this leaf continues from
          const int w = wait_booking();
          if (w < 0) return A_FINISH;
          if (w == LB_END) return A_END_TREE;   // this (speculated) leaf is discarded
          return leaf_spec(q, p, g, minv, lp, s0);
        }
        if (helped || uni(__atomic_load_n(live, __ATOMIC_RELAXED)) <= Pr().spec_live)
          return leaf_spec(q, p, g, minv, lp, s0);
      }
      return leaf(q, p, g, minv, lp, s0);
    }
    const double lp = finish_grad(g, s0);
    sub(4, ts);
    st(V_CUR_G, g);
    Sp->cur_lp = lp;
    Sp->cur_s2 = s0;
    return stt == ST_STEPSIZE ? A_SS_STEP : A_INIT_STEP;
  }

  __device__ int act_init_state() {
    FITOCT_MARK(act_init_state);
    V one, zero;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      one.a[s] = ok(s) ? 1.0 : 0.0;
      zero.a[s] = 0.0;
    }
    Sp->prof[lane >> 5][lane & 31] = 0;
#pragma unroll 1
    for (int v = 0; v < NVEC; ++v) st(v, zero);
    if (Pr().init_minv) {   // warm restart (fitoct_plan_set_init): the chain's metric
      V m;
#pragma unroll
      for (int s = 0; s < PPL; ++s)
        m.a[s] = ok(s) ? Pr().init_minv[(size_t)lc * Pr().D + idx(s)] : 0.0;
      st(V_MINV, m);
    } else {
      st(V_MINV, one);
    }
    if (lane < NSLOT) SUMS[lane] = 0.0;
    AUX[lane] = 0.0;
    Sp->status = 0;
    Sp->leapfrogs = 0;
    const double eps0 = Pr().init_eps ? Pr().init_eps[lc] : Pr().stepsize0;
    Sp->eps = eps0;
    Sp->mu = log(10.0 * eps0);
    Sp->da_counter = 0;
    Sp->s_bar = 0.0;
    Sp->x_bar = 0.0;
    // stan::mcmc::windowed_adaptation::set_window_params + restart
    const int W = Pr().warmup;
    int ib = Pr().init_buffer, tb = Pr().term_buffer, bw = Pr().base_window;
    Sp->win_on = (W >= 20) ? 1 : 0;
    if (W >= 20 && ib + bw + tb > W) {
      ib = (int)(0.15 * W);
      tb = (int)(0.1 * W);
      bw = W - (ib + tb);
    }
    Sp->init_buf = ib;
    Sp->term_buf = tb;
    Sp->win_counter = 0;
    Sp->win_size = bw;
    Sp->win_next = ib + bw - 1;
    Sp->wf_n = 0;
    Sp->t = 0;
    Sp->ss_window = 0;
    Sp->depth = 0;
    Sp->pool_used = 0;
    Sp->init_attempt = 0;
    return A_INIT_START;
  }

  __device__ int act_init_start() {
    FITOCT_MARK(act_init_start);
    const int Nn = Pr().Nn, attempt = uni(Sp->init_attempt);
    V q;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      double base = 0.0, w = 0.0;
      if (k < 3) {
        base = log(Pr().theta0[k]);
        w = 0.025;
      } else if (k < 3 + Nn) {
        w = 0.05;
      } else if (k < Pr().D) {
        w = 0.25;
        if (FAM == FAM_NORMAL && k == 3 + Nn) base = -log(Pr().lambda_rate_eff);
      }
      const double u = uniform(key, (uint32_t)attempt, TAG_INIT, (uint32_t)k, 0u);
      q.a[s] = (k < Pr().D) ? base + Pr().init_radius * w * (2.0 * u - 1.0) : 0.0;
      if (Pr().init_q && k < Pr().D) q.a[s] = Pr().init_q[(size_t)lc * Pr().D + k];   // warm restart
    }
    st(V_CUR_Q, q);
    Sp->state = ST_INIT;
    return A_WRITE_MP;
  }

  __device__ int act_init_step() {
    FITOCT_MARK(act_init_step);
    const V g = ld(V_CUR_G);
    double bad = 0.0;
#pragma unroll
    for (int s = 0; s < PPL; ++s)
      if (ok(s) && !(fabs(g.a[s]) <= DBL_MAX)) bad = 1.0;
    bad = wave_sum(bad);
    if (!(Sp->cur_lp > -INFINITY) || bad != 0.0) {
      if (Sp->init_attempt + 1 >= 100 || Pr().init_q) {   // a given start is not retried
        Sp->status = ERR_INIT;
        return A_FINISH;
      }
      Sp->init_attempt += 1;
      return A_INIT_START;
    }
    copyv(V_SMP_Q, V_CUR_Q);
    st(V_SMP_G, g);
    Sp->smp_lp = Sp->cur_lp;
    Sp->smp_s2 = Sp->cur_s2;
    return Pr().adapt ? A_SS_BEGIN : A_START_TRANSITION;
  }

  // --------------------- leapfrog (stan expl_leapfrog) -----------------------
  // A_LEAPFROG: begin_update_p + update_q from CUR with step Sp->lf_e
  __device__ int act_leapfrog() {
    FITOCT_MARK(act_leapfrog);
    return leapfrog_stage(ld(V_CUR_Q), ld(V_CUR_P), ld(V_CUR_G), ld(V_MINV), Sp->lf_e);
  }
  // begin_update_p + update_q from (q, p, g) in registers, then stage the new position
  // for the gradient waves (write_mp): the whole path to the next sweep without an LDS
  // round trip or an action dispatch
  __device__ int leapfrog_stage(V q, V p, const V& g, const V& minv, const double e) const {
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      p.a[s] = fma(0.5 * e, g.a[s], p.a[s]);        // p -= e/2 dphi/dq
      q.a[s] = fma(e, minv.a[s] * p.a[s], q.a[s]);  // q += e M^-1 p
    }
    st(V_CUR_P, p);
    st(V_CUR_Q, q);
    write_mp(q);
    return A_YIELD;
  }
  __device__ int act_write_mp() {
    FITOCT_MARK(act_write_mp);
    long long ts = stamp0();
    write_mp(ld(V_CUR_Q));
    return A_YIELD;
  }
  // end_update_p with the gradient that just arrived
  __device__ V finish_leapfrog(double e) const {
    V p = ld(V_CUR_P);
    const V g = ld(V_CUR_G);
#pragma unroll
    for (int s = 0; s < PPL; ++s) p.a[s] = fma(0.5 * e, g.a[s], p.a[s]);
    st(V_CUR_P, p);
    return p;
  }

  // ----------------- base_hmc::init_stepsize as actions ----------------------
  __device__ int act_ss_begin() {
    FITOCT_MARK(act_ss_begin);
    const double eps = Sp->eps;
    if (eps == 0.0 || eps > 1e7 || isnan(eps)) return A_SS_FINISH;  // skipped like Stan
    Sp->ss_trial = 0;
    Sp->state = ST_STEPSIZE;
    return A_SS_TRIAL;
  }
  __device__ int act_ss_trial() {
    FITOCT_MARK(act_ss_trial);
    const V minv = ld(V_MINV);
    const V p = momentum(TAG_SSMOM, (uint32_t)uni(Sp->ss_window), (uint32_t)uni(Sp->ss_trial), minv);
    Sp->ss_H0 = -Sp->smp_lp + kin(p, minv);
    copyv(V_CUR_Q, V_SMP_Q);
    copyv(V_CUR_G, V_SMP_G);
    st(V_CUR_P, p);
    Sp->lf_e = Sp->eps;
    return A_LEAPFROG;
  }
  __device__ int act_ss_step() {
    FITOCT_MARK(act_ss_step);
    const V p = finish_leapfrog(Sp->eps);
    double h = -Sp->cur_lp + kin(p, ld(V_MINV));
    if (isnan(h)) h = INFINITY;
    const double dH = Sp->ss_H0 - h;
    const double L08 = -0.22314355131420976;  // log(0.8)
    if (Sp->ss_trial == 0) {
      Sp->ss_dir = (dH > L08) ? 1 : -1;
      Sp->ss_trial = 1;
      return A_SS_TRIAL;
    }
    if ((Sp->ss_dir == 1 && !(dH > L08)) || (Sp->ss_dir == -1 && !(dH < L08))) return A_SS_FINISH;
    Sp->eps = (Sp->ss_dir == 1) ? 2.0 * Sp->eps : 0.5 * Sp->eps;
    if (Sp->eps > 1e7 || Sp->eps == 0.0 || Sp->ss_trial > 2000) {
      Sp->status = ERR_NUMERIC;
      return A_FINISH;
    }
    Sp->ss_trial += 1;
    return A_SS_TRIAL;
  }
  __device__ int act_ss_finish() {
    FITOCT_MARK(act_ss_finish);
    if (uni(Sp->ss_window) == 0) return A_START_TRANSITION;
    // adapt_diag_e_nuts::transition after a metric update
    Sp->mu = log(10.0 * Sp->eps);
    Sp->da_counter = 0;
    Sp->s_bar = 0.0;
    Sp->x_bar = 0.0;
    return A_NEXT_TRANSITION;
  }

  // ------------------------------ transition --------------------------------
  __device__ int act_start_transition() {
    FITOCT_MARK(act_start_transition);
    Sp->state = ST_TREE;
    Sp->eps_used = Sp->eps;
    const V minv = ld(V_MINV);
    const V p = momentum(TAG_MOM, (uint32_t)uni(Sp->t), 0u, minv);
    Sp->H0 = -Sp->smp_lp + kin(p, minv);
    Sp->smp_h = Sp->H0;   // energy__ if no leaf replaces the initial point
    const V q = ld(V_SMP_Q), g = ld(V_SMP_G);
    st(V_E0_Q, q); st(V_E0_P, p); st(V_E0_G, g);
    st(V_E1_Q, q); st(V_E1_P, p); st(V_E1_G, g);
    Sp->end_lp[0] = Sp->end_lp[1] = Sp->smp_lp;
    Sp->end_s2[0] = Sp->end_s2[1] = Sp->smp_s2;
    st(V_RHO, p);
    Sp->lsw_m = 0.5;   // weight of the initial point: exp(0) = 0.5 * 2^1
    Sp->lsw_e = 1;
    Sp->n_leapfrog = 0;
    Sp->sum_metro = 0.0;
    Sp->depth = 0;
    Sp->divergent = 0;
    Sp->pool_used = 0;
    return A_BEGIN_SUBTREE;
  }

  __device__ int act_begin_subtree() {
    FITOCT_MARK(act_begin_subtree);
    if constexpr (kTwoEnded) {
      if (bidi) return bidi_begin();   // reached at depth 0 only: the helper books from there on
      if (MIG && tail_ready() && tail_claim()) return bidi_begin();   // (the chain's own wave books, kernel)
    }
    const int d = uni(Sp->depth);
    const double u = uniform(key, (uint32_t)uni(Sp->t), TAG_DIR, (uint32_t)d, 0u);
    const int dir = (u > 0.5) ? 1 : 0;
    Sp->dir = dir;
    const int eq = dir ? V_E1_Q : V_E0_Q;
    const V qe = ld(eq), pe = ld(eq + 1), ge = ld(eq + 2), minv = ld(V_MINV);
    st(V_PNEAR, pe);
    st(V_CUR_G, ge);
    Sp->cur_lp = Sp->end_lp[dir];
    Sp->cur_s2 = Sp->end_s2[dir];
    Sp->leaf = 0;
    Sp->sub_metro = 0.0;
    if (lane < MAXDEPTH) Sp->u_blk[lane] = -1;   // merge uniforms are per subtree (depth d)
    const double e = dir ? Sp->eps_used : -Sp->eps_used;
    Sp->lf_e = e;
    return leapfrog_stage(qe, pe, ge, minv, e);   // act_leapfrog + act_write_mp
  }

  // proposal pool: at most max_depth + 1 live slots (stack records + the running
  // subtree).  `used` is the slot bitmask, kept in registers by the caller.
  __device__ int pool_put(unsigned& used, const V& q, const V& g, double lp, double s2,
                          double h) const {
    const int sl = __builtin_ctz(~used);
    used |= 1u << sl;
    AS_GLB double* dq = pslot(sl, P_Q);
    AS_GLB double* dg = pslot(sl, P_G);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {   // HBM stores, never waited on; D lanes only (the
      if (ok(s)) {                    // padding lanes of q, g are 0: top_merge reads 0)
        dq[idx(s)] = q.a[s];
        dg[idx(s)] = g.a[s];
      }
    }
    Sp->pool_lp[sl] = lp;
    Sp->pool_s2[sl] = s2;
    Sp->pool_h[sl] = h;
    return sl;
  }

  // one leaf of base_nuts::build_tree, followed by every merge it completes and,
  // when the subtree of depth d is complete, the top-level merge of the transition.
  // Chain scalars are read once into registers and written back once, so the
  // action costs a handful of LDS round trips instead of one per field.
  // Reached from act_grad (state ST_TREE) with the leaf's q, p (begin-updated), the
  // gradient just completed, the metric, lp and sum r^2 in registers.  A leaf inside
  // the subtree continues straight into the next leapfrog and stages its position
  // (act_leapfrog + act_write_mp with the same arithmetic, no LDS round trip or
  // dispatch between them).
  __device__ int leaf(const V& q, V p, const V& g, const V& minv, const double cur_lp,
                      const double cur_s2) {
    const double e = Sp->lf_e;
#pragma unroll
    for (int s = 0; s < PPL; ++s) p.a[s] = fma(0.5 * e, g.a[s], p.a[s]);   // end_update_p
    switch (leaf_book(q, p, g, minv, cur_lp, cur_s2)) {
      case LB_MID: return leapfrog_stage(q, p, g, minv, e);   // act_leapfrog + act_write_mp
      case LB_NEXT: return A_BEGIN_SUBTREE;
      default: return A_END_TREE;
    }
  }

  // Speculative leaf (tiles hosting one chain, with a helper wave): the next leaf's
  // position depends only on this leaf's (q, p, g) -- or, after the last leaf of a
  // subtree, on the trajectory end the next subtree grows from, whose direction is a
  // pre-addressed uniform -- not on the merges and U-turn checks.  So the next position
  // is staged and handed to the gradient waves first; the helper wave computes its prior
  // part while this wave does the bookkeeping of leaf j.  If the bookkeeping ends the
  // trajectory, the speculated sweep is drained and discarded.  Same arithmetic on the
  // same values as the plain path: draws are bitwise identical.
  __device__ int leaf_spec(const V& q, const V& p, const V& g, const V& minv, const double cur_lp,
                           const double cur_s2) {
    const double e = Sp->lf_e;
    const int d = uni(Sp->depth), j = uni(Sp->leaf);
    const bool last = j == (1 << d) - 1;
    if (last && d + 1 >= Pr().max_depth) {   // the tree ends here at the latest: no speculation
      if (deep) tree_uniforms(d, j, (uint32_t)uni(Sp->t));   // the helper did not draw them
      return leaf(q, p, g, minv, cur_lp, cur_s2);
    }
    V pe;
#pragma unroll
    for (int s = 0; s < PPL; ++s) pe.a[s] = fma(0.5 * e, g.a[s], p.a[s]);   // end_update_p
    const int dir = uni(Sp->dir);
    int dirn = dir, dn = d, jn = j + 1;
    double en = e;
    V qs = q, ps = pe, gs = g;
    const uint32_t t = (uint32_t)uni(Sp->t);
    if (last) {   // act_begin_subtree of depth d + 1
      dn = d + 1;
      jn = 0;
      dirn = (uniform(key, t, TAG_DIR, (uint32_t)dn, 0u) > 0.5) ? 1 : 0;
      if (dirn != dir) {
        const int eq = dirn ? V_E1_Q : V_E0_Q;
        qs = ld(eq);
        ps = ld(eq + 1);
        gs = ld(eq + 2);
      }
      en = dirn ? Sp->eps_used : -Sp->eps_used;
    }
    leapfrog_stage(qs, ps, gs, minv, en);
    if (deep) {   // hand leaf k to the booking helper (deep_book)
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        HX[idx(s)] = q.a[s];
        HX[VLEN + idx(s)] = pe.a[s];
        HX[2 * VLEN + idx(s)] = g.a[s];
      }
      if (lane == 0) {
        HX[3 * VLEN] = cur_lp;
        HX[3 * VLEN + 1] = cur_s2;
      }
      return A_SPEC_STAGED;
    }
    // for the helper (spec_weight): the booked leaf's end-updated momentum, in CUR_G's
    // slot (while a tree grows nothing reads CUR_G; begin_subtree rewrites it)
    st(V_CUR_G, pe);   // (its lp is Sp->cur_lp, set by act_grad)
    if constexpr (KLDS) {
      st(V_PG, q);
      st(V_CA, g);
    } else {
      k_q = q; k_pe = pe; k_g = g;
    }

    k_dirn = dirn; k_dn = dn; k_jn = jn; k_t = t;
    return A_SPEC_STAGED;   // the kernel enqueues the position and posts the helper
  }
  // the bookkeeping of the speculated leaf, while its successor is being swept
  __device__ int act_spec_book() {
    FITOCT_MARK(act_spec_book);
    spec_weight();   // (act_spec_book runs only without a helper wave: tiles of several chains)
    const int r = KLDS ? leaf_book_split(ld(V_PG), ld(V_CUR_G), ld(V_CA), ld(V_MINV), Sp->cur_lp,
                                         Sp->cur_s2)
                       : leaf_book_split(k_q, k_pe, k_g, ld(V_MINV), Sp->cur_lp, Sp->cur_s2);
    if (r == LB_NEXT) {   // the rest of act_begin_subtree (the top merge set depth d + 1)
      // the next subtree grows from trajectory end k_dirn: the far end if the direction
      // changed (untouched by the top merge), else the end the top merge just set to this
      // leaf -- in both cases the (p, g) leaf_spec staged the next leapfrog from
      Sp->dir = k_dirn;
      const int eq = k_dirn ? V_E1_Q : V_E0_Q;
      st(V_PNEAR, ld(eq + 1));
      st(V_CUR_G, ld(eq + 2));
      Sp->cur_lp = Sp->end_lp[k_dirn];
      Sp->cur_s2 = Sp->end_s2[k_dirn];
      Sp->leaf = 0;
      Sp->sub_metro = 0.0;
      if (lane < MAXDEPTH) Sp->u_blk[lane] = -1;
      Sp->lf_e = k_dirn ? Sp->eps_used : -Sp->eps_used;
    }
    // without a helper, the next position's prior part follows the bookkeeping here
    if (r != LB_END) prior_and_uniforms(true, k_dn, k_jn, k_t);
    return r == LB_END ? A_SPEC_DISCARD : A_SPEC_WAIT;
  }

  // Deep speculation, run by the helper wave: the whole bookkeeping of the leaf the chain's
  // wave handed over in HX (act_spec_book's work with the weight computed here), with the
  // coordinates (depth, leaf, direction, step) in Sp advanced for the next leaf exactly as
  // act_spec_book advances them -- the chain's wave reads them only after waiting for this
  // booking.  Same operations on the same values as the plain path: same draws.
  __device__ __forceinline__ int deep_book() {
    V q, pe, g;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      q.a[s] = HX[idx(s)];
      pe.a[s] = HX[VLEN + idx(s)];
      g.a[s] = HX[2 * VLEN + idx(s)];
    }
    return book_leaf(q, pe, g, HX[3 * VLEN], HX[3 * VLEN + 1]);
  }
  // ... of a leaf given by value (deep_book: from HX; bidi_book: from a producer's ring)
  __device__ __forceinline__ int book_leaf(const V& q, const V& pe, const V& g, const double lp, const double s2) {
    const int d = uni(Sp->depth), j = uni(Sp->leaf);
    const uint32_t t = (uint32_t)uni(Sp->t);
    tree_uniforms(d, j, t);
    const V minv = ld(V_MINV);
    double h = -lp + kin(pe, minv);
    if (isnan(h)) h = INFINITY;
    const XF w = xf_exp<FV3>(Sp->H0 - h);
    Sp->spec_h = h;
    Sp->spec_wm = w.m;
    Sp->spec_we = w.e;
    const int r = leaf_book_split(q, pe, g, minv, lp, s2);
    if (r == LB_NEXT) {   // act_begin_subtree's bookkeeping for the subtree of depth d + 1
      const int dirn = (uniform(key, t, TAG_DIR, (uint32_t)(d + 1), 0u) > 0.5) ? 1 : 0;
      Sp->dir = dirn;
      st(V_PNEAR, ld((dirn ? V_E1_Q : V_E0_Q) + 1));
      Sp->leaf = 0;
      Sp->sub_metro = 0.0;
      if (lane < MAXDEPTH) Sp->u_blk[lane] = -1;
      Sp->lf_e = dirn ? Sp->eps_used : -Sp->eps_used;
    }
    return r;
  }
  // the chain's wave: wait for the booking of the previous leaf (if one is outstanding);
  // its LB_* outcome, or -1 on a timeout (status set)
  __device__ int wait_booking() {
    if (book_want == 0) return LB_MID;
    long long ts = stamp0();   // profiling build: sub-stamp 8 = this wave's stall on the booking
    Patience w;
    while (*book_done < book_want) {
      if (w.expired(LEAF_WAIT_TICKS)) {
        Sp->status = ERR_TIMEOUT;
        return -1;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    wave_fence();   // the booking's LDS writes are visible from here
    sub(8, ts);
    const int r = uni(*book_res);
    book_want = 0;
    return r;
  }

  // ---------------- two-ended trajectories (P.bidi; tiles of one chain) ----------------
  // Stan's trajectory grows by doublings in directions drawn per depth (TAG_DIR); a doubling of
  // depth d builds a subtree of 2^d leaves from the trajectory end in its direction, and the
  // subtrees grown in one direction form one unbroken leapfrog chain from the transition's
  // start.  Everything base_nuts::build_tree does inside a subtree -- each leaf's weight and
  // divergence test, the multinomial merges, the U-turn checks of its levels, the subtree's
  // proposal -- depends only on that subtree's leaves.  So two producer waves (one per
  // direction, slots 1 and 2) build the subtrees of their direction whole, each in its own
  // chain area (levels, merge uniforms, proposal pool), at most BIDI_LOOK doublings past the
  // one booked, and the chain's wave books the trajectory level only, in tree order, from one
  // record per subtree (sub_publish): the top-level multinomial merge, the new end, the
  // trajectory-level U-turn checks.  The same operations on the same values as the one-ended
  // path (the acceptance statistic is summed per subtree on every path), so the same draws;
  // a transition takes about as long as its longer end, and the booking no longer paces it.
  enum SubRes : int { SL_MID = 0, SL_DONE = 1, SL_END = 2 };
  enum SubFlag : int { SR_VALID = 1, SR_DIVERGENT = 2 };
  // A subtree record: RVEC vectors -- the proposal's q and g, the end's (last leaf's)
  // momentum, the subtree's begin momentum and momentum sum -- and scalars RS_*.  Record m of
  // end s sits in slot m % RSLOTS: in a tile of one chain two slots per end (Lds::qx0, after
  // the hand-off slots), in a migrating tile (or at two parameters per lane) one, in vectors of
  // the producer's own area that a producer never uses (V_E1_Q .. V_SMP_G; the scalars in
  // V_RHO's).  Record m is written once the booking has taken record m - RSLOTS.
  static constexpr int RVEC = 5, RSLOTS = (MIG || PPL > 1) ? 1 : 2;
  enum RecVec : int { RV_SQ = 0, RV_SG, RV_EP, RV_PB, RV_RHO };
  enum RecSc : int { RS_SLP = 0, RS_SS2, RS_SH, RS_TWM, RS_METRO, RS_TWE, RS_N, RS_FLAGS, RS_DEPTH,
                     RS_N_ };
  AS_LDS double* QX0 = nullptr;   // the tile's record slots (tiles of one chain)
  __device__ __forceinline__ AS_LDS double* rvec(int s, int m) const {
    if constexpr (RSLOTS == 1) return pvb(s) + V_E1_Q * VLEN;
    else return QX0 + (size_t)(2 * s + (m & 1)) * Lds<PPL>::QX_DOUBLES;
  }
  __device__ __forceinline__ AS_LDS double* rsc(int s, int m) const {
    if constexpr (RSLOTS == 1) return pvb(s) + V_RHO * VLEN;
    else return rvec(s, m) + RVEC * VLEN;
  }
  __device__ __forceinline__ V pld(const AS_LDS double* base, int v) const {
    V r;
#pragma unroll
    for (int s = 0; s < PPL; ++s) r.a[s] = base[v * VLEN + idx(s)];
    return r;
  }
  // a migrating tile's chain, at the start of a transition (depth 0): two-ended when the tile
  // hosts one live chain, two idle receivers of the tile have become
  // producers and no other chain of the tile is growing a tree with them (TW_BUSY, claimed
  // by tail_claim, released when the tree is booked)
  __device__ __forceinline__ bool tail_ready() const {
    const int lv = uni(__atomic_load_n(live, __ATOMIC_RELAXED));
    return Pr().tail_bidi != 0 && uni(Sp->depth) == 0 && uni(bd[TW_JOIN]) >= 2 && lv == 1 &&
           uni(bd[TW_BUSY]) == 0;
  }
  __device__ __forceinline__ bool tail_claim() const {
    int ok = 0;
    if (lane == 0) ok = atomicCAS((int*)&bd[TW_BUSY], 0, 1) == 0;
    return uni(__shfl(ok, 0)) != 0;
  }
  // The chain's wave: book transition g's trajectory level in Stan's tree order from the
  // producers' subtree records (base_nuts::transition: the loop over depths; top_merge and
  // leaf_book's trajectory check on the record's values).  LB_END, with the status
  // ERR_TIMEOUT if a producer's record never came (a fault)
  // profiling build: this wave's cycles waiting for records / booking, subtrees booked
  long long pf_wait = 0, pf_busy = 0, pf_n = 0;
  template <class Idle>
  __device__ __forceinline__ int bidi_book_tree(const int g, Idle&& idle) {
    const uint32_t t = (uint32_t)uni(Sp->t);
    const V minv = ld(V_MINV);
    int m0 = 0, m1 = 0;
    for (;;) {
      const long long pt0 = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
      const int d = uni(Sp->depth);
      const int s = (uniform(key, t, TAG_DIR, (uint32_t)d, 0u) > 0.5) ? 1 : 0;
      const int m = s ? m1 : m0;
      bool lost = false;
      Patience wl;   // one subtree of the longer end: bounded by the whole tree's bound
      for (;;) {     // record m of end s published for this transition
        const int w = bd[BD_PROD + s];
        if ((w >> 16) == g && (w & 0xFFFF) > m) break;
        if (bd[BD_GEN] != g || wl.expired(MIG_WAIT_TICKS)) {   // never, short of a fault
          lost = true;
          break;
        }
        if (!idle()) __builtin_amdgcn_s_sleep(1);
      }
      if (lost) {
        Sp->status = ERR_TIMEOUT;
        return LB_END;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // the record after its count
      const long long pt1 = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
      const AS_LDS double* RV = rvec(s, m);
      const AS_LDS double* SC = rsc(s, m);
      const int fl = uni((int)SC[RS_FLAGS]);
      Sp->n_leapfrog = uni(Sp->n_leapfrog) + uni((int)SC[RS_N]);
      Sp->sum_metro = Sp->sum_metro + SC[RS_METRO];
      if (fl & SR_DIVERGENT) Sp->divergent = 1;
      bool persist = false;
      if (fl & SR_VALID) {
        // top_merge: the sample, the trajectory's weight, the end, the depth
        const XF Tw{SC[RS_TWM], uni((int)SC[RS_TWE])};
        const XF Ww{Sp->lsw_m, Sp->lsw_e};
        const double u_top = uniform(key, t, TAG_TOP, (uint32_t)d, 0u);
        const bool take = xf_gt(Tw, Ww) || xf_u_below(u_top, Tw, Ww);
        if (take) {
          st(V_SMP_Q, pld(RV, RV_SQ));
          st(V_SMP_G, pld(RV, RV_SG));
          Sp->smp_lp = SC[RS_SLP];
          Sp->smp_s2 = SC[RS_SS2];
          Sp->smp_h = SC[RS_SH];
        }
        const XF Wn = xf_add(Ww, Tw);
        Sp->lsw_m = Wn.m;
        Sp->lsw_e = Wn.e;
        Sp->depth = d + 1;
        // the trajectory-level U-turn checks (leaf_book's, at the subtree's last leaf)
        const V pend = pld(RV, RV_EP), Tpb = pld(RV, RV_PB), Trho = pld(RV, RV_RHO);
        const int ef = s ? V_E1_P : V_E0_P;
        const V far = ld(s ? V_E0_P : V_E1_P), near = ld(ef), rho = ld(V_RHO);
        V rtot, rx, ry;
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
          rtot.a[k] = rho.a[k] + Trho.a[k];
          rx.a[k] = rho.a[k] + Tpb.a[k];
          ry.a[k] = Trho.a[k] + near.a[k];
        }
        persist = crit3(far, pend, rtot, far, Tpb, rx, near, pend, ry, minv);
        st(ef, pend);
        st(V_RHO, rtot);
      }
      if (s) ++m1;
      else ++m0;
      wave_publish();   // the record's reads are done before the slot is released
      if (lane == 0) bd[BD_CONS + s] = m + 1;
      if (kProfile) {
        pf_wait += pt1 - pt0;
        pf_busy += (long long)__builtin_amdgcn_s_memtime() - pt1;
        ++pf_n;
      }
      if (!persist || d + 1 >= Pr().max_depth) return LB_END;
    }
  }
  // the chain's wave, at depth 0 of a transition: the start to both producers' slots, then
  // the transition's number (BD_GEN) releases them
  __device__ int bidi_begin() {
    const uint32_t t = (uint32_t)uni(Sp->t);
    const V q = ld(V_E0_Q), p = ld(V_E0_P), g = ld(V_E0_G), minv = ld(V_MINV);   // E0 = E1 = start
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      AS_LDS double* const pv = pvb(k);
      AS_LDS ChainScalars* const ps = psp(k);
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        pv[V_E0_Q * VLEN + idx(s)] = q.a[s];
        pv[V_E0_P * VLEN + idx(s)] = p.a[s];
        pv[V_E0_G * VLEN + idx(s)] = g.a[s];
        pv[V_MINV * VLEN + idx(s)] = minv.a[s];
      }
      if (lane == 0) {
        ps->eps_used = Sp->eps_used;
        ps->t = (int)t;
        ps->H0 = Sp->H0;
      }
    }
    if (lane == 0) {
      bd[BD_CONS] = 0;
      bd[BD_CONS + 1] = 0;
      bd[TW_CHAIN] = slot;   // the producers read the booked depth and the key from these
      bd[TW_LC] = lc;
    }
    wave_publish();   // every store above lands before the transition's number
    if (lane == 0) {
      bd[BD_GEN] = (bd[BD_GEN] & BD_GEN_MASK) % BD_GEN_MASK + 1;
      atomicAdd(Pr().bidi_count, 1ULL);
    }
    return A_BIDI_TREE;
  }
  // ---- the producer's side (run on the producer's own chain area) ----
  // a subtree of depth d begins (act_begin_subtree's bookkeeping, counts of this subtree)
  __device__ void sub_begin(const int d) {
    Sp->depth = d;
    Sp->leaf = 0;
    Sp->sub_metro = 0.0;
    Sp->n_leapfrog = 0;
    Sp->pool_used = 0;
    Sp->divergent = 0;
    if (lane < MAXDEPTH) Sp->u_blk[lane] = -1;
  }
  // One leaf of the producer's subtree (base_nuts::build_tree below the trajectory level):
  // leaf_book's weight, divergence test, merges, U-turn checks and push -- the same operations
  // on the same values.  At the subtree's last leaf (SL_DONE) its weight, proposal, begin
  // momentum and momentum sum are returned for sub_publish.  (q, p, g): the leaf with its
  // end-updated momentum.
  __device__ __forceinline__ int sub_leaf(const V& q, const V& p, const V& g, const V& minv, const double cur_lp,
                          const double cur_s2, XF& Tw_o, int& Tprop_o, V& Tpb_o, V& Trho_o,
                          double& h_o) {
    const double H0 = Sp->H0;
    const double sub_metro0 = Sp->sub_metro;
    const int d = uni(Sp->depth), j = uni(Sp->leaf), nlf = uni(Sp->n_leapfrog);
    unsigned used = (unsigned)uni(Sp->pool_used);
    Sp->n_leapfrog = nlf + 1;
    tree_uniforms(d, j, (uint32_t)uni(Sp->t));   // this leaf's merge uniforms
    double h = -cur_lp + kin(p, minv);
    if (isnan(h)) h = INFINITY;
    const double wl = H0 - h;
    const XF wleaf = xf_exp<FV3>(wl);
    Sp->sub_metro = sub_metro0 + ((wl > 0.0) ? 1.0 : xf_val(wleaf));
    if (h - H0 > 1000.0) {   // divergent: the transition ends here
      Sp->divergent = 1;
      return SL_END;
    }
    V Tpb = p, Trho = p;
    XF Tw = wleaf;
    int Tprop = -1;   // -1: the current leaf; else a pool slot
#pragma unroll 1
    for (int l = 0; l < d; ++l) {
      if (((j >> l) & 1) == 0) {   // push T as the init subtree of level l+1
        lst(l, K_PBEG, Tpb);
        lst(l, K_PEND, p);
        lst(l, K_RHO, Trho);
        Sp->st_w_m[l] = Tw.m;
        Sp->st_w_e[l] = Tw.e;
        Sp->st_prop[l] = (Tprop < 0) ? pool_put(used, q, g, cur_lp, cur_s2, h) : Tprop;
        break;
      }
      // merge init I = level l with final T (base_nuts::build_tree at depth l+1)
      const V Ipb = lld(l, K_PBEG), Ipe = lld(l, K_PEND), Irho = lld(l, K_RHO);
      const XF Iw{Sp->st_w_m[l], Sp->st_w_e[l]};
      const double um = RNG[l * WAVE + ((j >> (l + 1)) & (WAVE - 1))];
      const int Iprop = uni(Sp->st_prop[l]);
      const XF Sw = xf_add(Iw, Tw);
      const bool take_final = xf_gt(Tw, Sw) || xf_u_below(um, Tw, Sw);
      if (take_final) {
        used &= ~(1u << Iprop);
      } else {
        if (Tprop >= 0) used &= ~(1u << Tprop);
        Tprop = Iprop;
      }
      V rsub, rx, ry;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        rsub.a[s] = Irho.a[s] + Trho.a[s];
        rx.a[s] = Irho.a[s] + Tpb.a[s];
        ry.a[s] = Trho.a[s] + Ipe.a[s];
      }
      const bool okc = crit3(Ipb, p, rsub, Ipb, Tpb, rx, Ipe, p, ry, minv);
      Tpb = Ipb;
      Trho = rsub;
      Tw = Sw;
      if (!okc) {
        Sp->pool_used = (int)used;
        return SL_END;
      }
    }
    Sp->pool_used = (int)used;
    if (j != (1 << d) - 1) {
      Sp->leaf = j + 1;
      return SL_MID;
    }
    Tw_o = Tw;
    Tprop_o = Tprop;
    Tpb_o = Tpb;
    Trho_o = Trho;
    h_o = h;
    return SL_DONE;
  }
  // record m of end s for the booking (its slot free: record m - RSLOTS was booked).
  // flags 0 / SR_DIVERGENT: an invalid subtree (only its counts matter)
  __device__ __forceinline__ void sub_publish(const int s, const int m, const int flags,
                                              const XF Tw, const int Tprop, const V& Tpb,
                                              const V& Trho, const V& q, const V& pe,
                                              const V& g, const double lp, const double s2,
                                              const double h) {
    AS_LDS double* const RV = rvec(s, m);
    AS_LDS double* const SC = rsc(s, m);
    if (flags & SR_VALID) {
      V sq = q, sg = g;
      double slp = lp, ss2 = s2, sh = h;
      if (Tprop >= 0) {   // the proposal is a pool slot (top_merge's read)
        const AS_GLB double* pq = pslot(Tprop, P_Q);
        const AS_GLB double* pg = pslot(Tprop, P_G);
#pragma unroll
        for (int k = 0; k < PPL; ++k) {
          sq.a[k] = ok(k) ? pq[idx(k)] : 0.0;
          sg.a[k] = ok(k) ? pg[idx(k)] : 0.0;
        }
        slp = Sp->pool_lp[Tprop];
        ss2 = Sp->pool_s2[Tprop];
        sh = Sp->pool_h[Tprop];
      }
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        RV[RV_SQ * VLEN + idx(k)] = sq.a[k];
        RV[RV_SG * VLEN + idx(k)] = sg.a[k];
        RV[RV_EP * VLEN + idx(k)] = pe.a[k];
        RV[RV_PB * VLEN + idx(k)] = Tpb.a[k];
        RV[RV_RHO * VLEN + idx(k)] = Trho.a[k];
      }
      if (lane == 0) {
        SC[RS_SLP] = slp;
        SC[RS_SS2] = ss2;
        SC[RS_SH] = sh;
        SC[RS_TWM] = Tw.m;
        SC[RS_TWE] = (double)Tw.e;
      }
    }
    if (lane == 0) {
      SC[RS_METRO] = Sp->sub_metro;
      SC[RS_N] = (double)Sp->n_leapfrog;
      SC[RS_FLAGS] = (double)flags;
      SC[RS_DEPTH] = (double)Sp->depth;
    }
  }

  // run by the helper wave for the leaf being booked: its Hamiltonian and multinomial
  // weight, the same operations as leaf_book's first lines
  __device__ void spec_weight() const {
    const V pe = ld(V_CUR_G), minv = ld(V_MINV);   // leaf_spec staged the momentum there
    double h = -Sp->cur_lp + kin(pe, minv);
    if (isnan(h)) h = INFINITY;
    const XF w = xf_exp<FV3>(Sp->H0 - h);
    Sp->spec_h = h;
    Sp->spec_wm = w.m;
    Sp->spec_we = w.e;
  }

  // base_nuts::transition's merge of the completed subtree of depth d (final weight Tw,
  // proposal Tprop: -1 = the leaf (q, p, g) itself, else a pool slot) into the trajectory
  // grown in direction dir: the new trajectory end, depth d + 1, the multinomial choice
  // of the sample (u_top drawn by act_prior) and the trajectory weight.  Shared by
  // leaf_book and leaf_book_split.
  __device__ __forceinline__ void top_merge(const V& q, const V& p, const V& g, const double cur_lp,
                                            const double cur_s2, const double h, const XF Tw,
                                            const int Tprop, unsigned used, const int dir,
                                            const int d) const {
    const XF Ww{Sp->lsw_m, Sp->lsw_e};
    const double u_top = Sp->u_top;
    const int eq = dir ? V_E1_Q : V_E0_Q;
    st(eq, q);
    st(eq + 1, p);
    st(eq + 2, g);
    Sp->end_lp[dir] = cur_lp;
    Sp->end_s2[dir] = cur_s2;
    Sp->depth = d + 1;
    const bool take = xf_gt(Tw, Ww) || xf_u_below(u_top, Tw, Ww);
    if (take) {
      if (Tprop < 0) {
        st(V_SMP_Q, q);
        st(V_SMP_G, g);
        Sp->smp_lp = cur_lp;
        Sp->smp_s2 = cur_s2;
        Sp->smp_h = h;
      } else {
        const AS_GLB double* sq = pslot(Tprop, P_Q);
        const AS_GLB double* sg = pslot(Tprop, P_G);
        V q2, g2;
#pragma unroll
        for (int s = 0; s < PPL; ++s) {
          q2.a[s] = ok(s) ? sq[idx(s)] : 0.0;
          g2.a[s] = ok(s) ? sg[idx(s)] : 0.0;
        }
        st(V_SMP_Q, q2);
        st(V_SMP_G, g2);
        Sp->smp_lp = Sp->pool_lp[Tprop];
        Sp->smp_s2 = Sp->pool_s2[Tprop];
        Sp->smp_h = Sp->pool_h[Tprop];
      }
    }
    if (Tprop >= 0) used &= ~(1u << Tprop);
    Sp->pool_used = (int)used;
    const XF Wn = xf_add(Ww, Tw);
    Sp->lsw_m = Wn.m;
    Sp->lsw_e = Wn.e;
  }

  // leaf_book for the speculative path, split so that the weight can come from the
  // helper wave: first every U-turn check the leaf completes (they need momenta only:
  // the running subtree's begin momentum and momentum sum follow the levels'
  // records whatever the multinomial choices), including the trajectory-level check
  // when the subtree ends; then, with the helper's weight, the divergence test, the
  // multinomial merges up to the first failing check, the push and the top-level
  // merge.  Same operations on the same values as leaf_book, so the same outcome.
  __device__ int leaf_book_split(const V& q, const V& p, const V& g, const V& minv,
                                 const double cur_lp, const double cur_s2) {
    FITOCT_MARK(act_leaf_split);
    long long ts = stamp0();
    const double H0 = Sp->H0;
    const double sub_metro0 = Sp->sub_metro;
    const int d = uni(Sp->depth), j = uni(Sp->leaf), nlf = uni(Sp->n_leapfrog);
    unsigned used = (unsigned)uni(Sp->pool_used);
    Sp->n_leapfrog = nlf + 1;
    const int nm = min(d, (int)__builtin_ctz(~(unsigned)j));   // merges this leaf completes
    const bool last = j == (1 << d) - 1;
    // phase A: U-turn checks
    V Tpb = p, Trho = p;
    int fail = nm;
#pragma unroll 1
    for (int l = 0; l < nm; ++l) {
      const V Ipb = lld(l, K_PBEG), Ipe = lld(l, K_PEND), Irho = lld(l, K_RHO);
      V rsub, rx, ry;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        rsub.a[s] = Irho.a[s] + Trho.a[s];
        rx.a[s] = Irho.a[s] + Tpb.a[s];
        ry.a[s] = Trho.a[s] + Ipe.a[s];
      }
      const bool okc = crit3(Ipb, p, rsub, Ipb, Tpb, rx, Ipe, p, ry, minv);
      Tpb = Ipb;
      Trho = rsub;
      if (!okc) {
        fail = l;
        break;
      }
    }
    const int dir = uni(Sp->dir);
    V rtot;
    bool persist = false;
    if (last && fail == nm) {
      const V far = ld(dir ? V_E0_P : V_E1_P), near = ld(V_PNEAR), rho = ld(V_RHO);
      V rx, ry;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        rtot.a[s] = rho.a[s] + Trho.a[s];
        rx.a[s] = rho.a[s] + Tpb.a[s];
        ry.a[s] = Trho.a[s] + near.a[s];
      }
      persist = crit3(far, p, rtot, far, Tpb, rx, near, p, ry, minv);
    }
    sub(2, ts);
    // phase B: the leaf's weight (book_leaf's, or this wave's own: act_spec_book)
    const double h = Sp->spec_h, wl = H0 - h;
    const XF wleaf{Sp->spec_wm, uni(Sp->spec_we)};
    const double sm = sub_metro0 + ((wl > 0.0) ? 1.0 : xf_val(wleaf));
    Sp->sub_metro = sm;
    sub(1, ts);
    if (h - H0 > 1000.0) {   // divergent: the transition ends here
      Sp->divergent = 1;
      Sp->sum_metro += sm;
      return LB_END;
    }
    XF Tw = wleaf;
    int Tprop = -1;   // -1: the current leaf (CUR); else a pool slot
    const int nmerge = fail < nm ? fail + 1 : nm;
#pragma unroll 1
    for (int l = 0; l < nmerge; ++l) {
      const XF Iw{Sp->st_w_m[l], Sp->st_w_e[l]};
      const double um = RNG[l * WAVE + ((j >> (l + 1)) & (WAVE - 1))];
      const int Iprop = uni(Sp->st_prop[l]);
      const XF Sw = xf_add(Iw, Tw);
      const bool take_final = xf_gt(Tw, Sw) || xf_u_below(um, Tw, Sw);
      if (take_final) {
        used &= ~(1u << Iprop);
      } else {
        if (Tprop >= 0) used &= ~(1u << Tprop);
        Tprop = Iprop;
      }
      Tw = Sw;
    }
    if (fail < nm) {
      Sp->pool_used = (int)used;
      Sp->sum_metro += sm;
      return LB_END;
    }
    if (nm < d) {   // push the running subtree as the init subtree of level nm + 1
      lst(nm, K_PBEG, Tpb);
      lst(nm, K_PEND, p);
      lst(nm, K_RHO, Trho);
      Sp->st_w_m[nm] = Tw.m;
      Sp->st_w_e[nm] = Tw.e;
      Sp->st_prop[nm] = (Tprop < 0) ? pool_put(used, q, g, cur_lp, cur_s2, h) : Tprop;
    }
    sub(0, ts);
    if (!last) {
      Sp->pool_used = (int)used;
      Sp->leaf = j + 1;
      return LB_MID;
    }
    // the subtree of depth d is complete and valid: top-level merge (base_nuts::transition)
    top_merge(q, p, g, cur_lp, cur_s2, h, Tw, Tprop, used, dir, d);
    Sp->sum_metro += sm;
    st(V_RHO, rtot);
    sub(3, ts);
    if (!persist || d + 1 >= Pr().max_depth) return LB_END;
    return LB_NEXT;
  }

  // one leaf of base_nuts::build_tree with the momentum already end-updated: weight,
  // divergence, every merge it completes and, when the subtree of depth d is complete,
  // the top-level merge of the transition.  Returns LB_MID (leaf j + 1 of this subtree
  // is next), LB_NEXT (a subtree of depth d + 1 is next) or LB_END.
  __device__ int leaf_book(const V& q, const V& p, const V& g, const V& minv, const double cur_lp,
                           const double cur_s2) {
    FITOCT_MARK(act_leaf);
    long long ts = stamp0();
    const double H0 = Sp->H0;
    const double sub_metro0 = Sp->sub_metro;
    const int d = uni(Sp->depth), j = uni(Sp->leaf), nlf = uni(Sp->n_leapfrog);
    unsigned used = (unsigned)uni(Sp->pool_used);
    Sp->n_leapfrog = nlf + 1;
    double h = -cur_lp + kin(p, minv);
    if (isnan(h)) h = INFINITY;
    sub(0, ts);
    const double wl = H0 - h;
    const XF wleaf = xf_exp<FV3>(wl);
    // (Stan sums these over the trajectory's leaves in order; here per subtree, then the
    // subtrees' sums in tree order: a reassociation of the same terms, so that two-ended
    // trajectories, whose subtrees are booked by their producers, give the same bits)
    const double sm = sub_metro0 + ((wl > 0.0) ? 1.0 : xf_val(wleaf));
    Sp->sub_metro = sm;
    sub(1, ts);
    if (h - H0 > 1000.0) {   // divergent: the transition ends here
      Sp->divergent = 1;
      Sp->sum_metro += sm;
      return LB_END;
    }

    V Tpb = p, Trho = p;
    XF Tw = wleaf;
    int Tprop = -1;   // -1: the current leaf (CUR); else a pool slot
#pragma unroll 1
    for (int l = 0; l < d; ++l) {
      if (((j >> l) & 1) == 0) {   // push T as the init subtree of level l+1
        lst(l, K_PBEG, Tpb);
        lst(l, K_PEND, p);
        lst(l, K_RHO, Trho);
        Sp->st_w_m[l] = Tw.m;
        Sp->st_w_e[l] = Tw.e;
        Sp->st_prop[l] = (Tprop < 0) ? pool_put(used, q, g, cur_lp, cur_s2, h) : Tprop;
        break;
      }
      // merge init I = level l with final T (base_nuts::build_tree at depth l+1)
      const V Ipb = lld(l, K_PBEG), Ipe = lld(l, K_PEND), Irho = lld(l, K_RHO);
      const XF Iw{Sp->st_w_m[l], Sp->st_w_e[l]};
      const double um = RNG[l * WAVE + ((j >> (l + 1)) & (WAVE - 1))];   // drawn by act_prior
      const int Iprop = uni(Sp->st_prop[l]);
      const XF Sw = xf_add(Iw, Tw);
      const bool take_final = xf_gt(Tw, Sw) || xf_u_below(um, Tw, Sw);
      if (take_final) {
        used &= ~(1u << Iprop);
      } else {
        if (Tprop >= 0) used &= ~(1u << Tprop);
        Tprop = Iprop;
      }
      V rsub, rx, ry;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        rsub.a[s] = Irho.a[s] + Trho.a[s];
        rx.a[s] = Irho.a[s] + Tpb.a[s];
        ry.a[s] = Trho.a[s] + Ipe.a[s];
      }
      const bool okc = crit3(Ipb, p, rsub, Ipb, Tpb, rx, Ipe, p, ry, minv);
      Tpb = Ipb;
      Trho = rsub;
      Tw = Sw;
      if (!okc) {
        Sp->pool_used = (int)used;
        Sp->sum_metro += sm;
        return LB_END;
      }
    }
    sub(2, ts);
    if (j != (1 << d) - 1) {
      Sp->pool_used = (int)used;
      Sp->leaf = j + 1;
      return LB_MID;
    }
    // the subtree of depth d is complete and valid: top-level merge (base_nuts::transition)
    const int dir = uni(Sp->dir);
    top_merge(q, p, g, cur_lp, cur_s2, h, Tw, Tprop, used, dir, d);
    Sp->sum_metro += sm;
    const V far = ld(dir ? V_E0_P : V_E1_P), near = ld(V_PNEAR), rho = ld(V_RHO);
    V rtot, rx, ry;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      rtot.a[s] = rho.a[s] + Trho.a[s];
      rx.a[s] = rho.a[s] + Tpb.a[s];
      ry.a[s] = Trho.a[s] + near.a[s];
    }
    const bool persist = crit3(far, p, rtot, far, Tpb, rx, near, p, ry, minv);
    st(V_RHO, rtot);
    sub(3, ts);
    if (!persist || d + 1 >= Pr().max_depth) return LB_END;
    return LB_NEXT;
  }

  // Draw records are written once and never read by the kernel: streaming (non-temporal)
  // stores, so the draws stream through L2 instead of evicting the proposal pools, whose
  // lines are rewritten at every other leaf (config 3: L2->memory writes 6.6x the draws
  // with ordinary stores, profiles/r03_pmc_traffic_config3.json).
  static __device__ __forceinline__ void st_draw(AS_GLB double* p, double v) {
    __builtin_nontemporal_store(v, p);
  }
  __device__ void write_draw(double accept, double energy) const {
    const int t = Sp->t, W = Pr().warmup;
    if (t < W && !Pr().save_warmup) return;
    const int it = Pr().save_warmup ? t : t - W;
    AS_GLB double* rec = (AS_GLB double*)Pr().draws + ((size_t)lc * Pr().iters_saved + it) * Pr().ncols;
    const V q = ld(V_SMP_Q);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      if (k < Pr().D) st_draw(&rec[7 + k], is_log(k) ? exp(q.a[s]) : q.a[s]);
    }
    if (lane < 8) {
      double v;
      switch (lane) {
        case 0: v = Sp->smp_lp; break;
        case 1: v = accept; break;
        case 2: v = Sp->eps_used; break;
        case 3: v = (double)Sp->depth; break;
        case 4: v = (double)Sp->n_leapfrog; break;
        case 5: v = (double)Sp->divergent; break;
        case 6: v = energy; break;
        default: v = (Pr().prior_PD == 0) ? Sp->smp_s2 / (double)Pr().N : NAN; break;
      }
      st_draw(&rec[lane < 7 ? lane : 7 + Pr().D], v);
    }
  }

  __device__ int act_end_tree() {
    FITOCT_MARK(act_end_tree);
    const double accept = Sp->sum_metro / (double)Sp->n_leapfrog;
    // energy__ = H(z_sample) (base_nuts::transition), the sample leaf's own -lp + K(p):
    // the same operations on the same values as -smp_lp + kin(p_sample)
    const double energy = Sp->smp_h;
    write_draw(accept, energy);
    Sp->leapfrogs += Sp->n_leapfrog;
    if (uni(Sp->t) < Pr().warmup && Pr().adapt) {
      learn_stepsize(accept);
      if (learn_variance()) {
        Sp->ss_window += 1;
        return A_SS_BEGIN;
      }
    }
    return A_NEXT_TRANSITION;
  }

  // stan::mcmc::stepsize_adaptation::learn_stepsize
  __device__ void learn_stepsize(double adapt_stat) {
    Sp->da_counter += 1;
    const double cnt = (double)Sp->da_counter;
    adapt_stat = adapt_stat > 1.0 ? 1.0 : adapt_stat;
    const double eta = 1.0 / (cnt + Pr().t0);
    Sp->s_bar = (1.0 - eta) * Sp->s_bar + eta * (Pr().adapt_delta - adapt_stat);
    const double x = Sp->mu - Sp->s_bar * sqrt(cnt) / Pr().gamma;
    const double x_eta = pow(cnt, -Pr().kappa);
    Sp->x_bar = (1.0 - x_eta) * Sp->x_bar + x_eta * x;
    Sp->eps = exp(x);
  }

  // stan::mcmc::var_adaptation::learn_variance + windowed_adaptation
  __device__ bool learn_variance() {
    const int W = Pr().warmup, cnt = uni(Sp->win_counter);
    const int tb = Sp->term_buf;
    if (Sp->win_on && cnt >= Sp->init_buf && cnt < W - tb && cnt != W) {
      Sp->wf_n += 1;
      const double n = (double)Sp->wf_n;
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
    if (Sp->win_on && cnt == Sp->win_next && cnt != W) {
      // compute_next_window
      const int last = W - tb - 1;
      if (Sp->win_next != last) {
        Sp->win_size *= 2;
        Sp->win_next = cnt + Sp->win_size;
        if (Sp->win_next != last) {
          const int boundary = Sp->win_next + 2 * Sp->win_size;
          if (boundary >= W - tb) Sp->win_next = last;
        }
      }
      const double n = (double)Sp->wf_n;
      V var = ld(V_MINV);
      const V m2 = ld(V_WF_M2);
      V zero;
#pragma unroll
      for (int s = 0; s < PPL; ++s) {
        zero.a[s] = 0.0;
        if (ok(s)) {
          if (Sp->wf_n > 1) var.a[s] = m2.a[s] / (n - 1.0);
          var.a[s] = (n / (n + 5.0)) * var.a[s] + 1e-3 * (5.0 / (n + 5.0));
        }
      }
      st(V_MINV, var);
      st(V_WF_M, zero);
      st(V_WF_M2, zero);
      Sp->wf_n = 0;
      Sp->win_counter = cnt + 1;
      return true;
    }
    Sp->win_counter = cnt + 1;
    return false;
  }

  __device__ int act_next_transition() {
    FITOCT_MARK(act_next_transition);
    Sp->t += 1;
    const int t = uni(Sp->t);
    // transitions done, for fitoct_plan_poll (replaces rstan's stan.log progress)
    if (Pr().progress != nullptr && lane == 0) sys_store(Pr().progress + lc, t);
    if (t == Pr().warmup && Pr().adapt && Pr().warmup > 0) Sp->eps = exp(Sp->x_bar);  // complete_adaptation
    if (t >= Pr().warmup + Pr().samples) return A_FINISH;
    // fitoct_plan_cancel: stop at a transition boundary (checked every 8th transition)
    if (Pr().cancel != nullptr && (t & 7) == 0 && uni(sys_load(Pr().cancel)) != 0) {
      Sp->status = ERR_CANCELLED;
      return A_FINISH;
    }
    // a transition boundary: the chain's whole state is its LDS image (current
    // sample, metric, adaptation); hand it to an idle tile if this one is crowded
    if (MIG && Pr().mig != nullptr && t + 2 < Pr().warmup + Pr().samples && try_donate()) {
      Sp->state = ST_MOVED;
      return A_YIELD;
    }
    return A_START_TRANSITION;
  }

  // Work balance (the kernel ends with its slowest tile): a chain in a tile
  // hosting L chains moves to a posted free slot of a tile hosting <= L-2, if
  // any.  Its draws do not change: a chain's arithmetic is the same in every
  // tile of the launch (same bin-to-lane layout) and its random numbers are
  // addressed by (global chain id, iteration).
  __device__ bool try_donate() {
    KPc& P = Pr();
    const MigView M(P.mig, P.mig_tiles);
    if (uni(g_load(&M.hdr[MIG_WAITING])) <= 0) return false;
    const int me = blockIdx.x, T = P.mig_tiles;
    const int my = uni(g_load(&M.load[me]));
    if (my < 2) return false;
    int best = 0x7FFFFFFF;
    for (int i = lane; i < T; i += WAVE)
      if (g_load(&M.fmask[i]) != 0) best = min(best, (g_load(&M.load[i]) << 16) | i);
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) best = min(best, __shfl_xor(best, o));
    best = uni(best);
    if (best == 0x7FFFFFFF || (best >> 16) > my - 2) return false;
    const int tt = best & 0xFFFF;
    int slot = -1;
    if (lane == 0) {
      const int f = g_load(&M.fmask[tt]);
      if (f != 0) {
        const int b = __builtin_ctz(f);
        if (g_cas(&M.fmask[tt], f, f & ~(1 << b))) slot = b;
      }
    }
    slot = __shfl(slot, 0);
    slot = uni(slot);
    if (slot < 0) return false;
    if (lane == 0) {
      g_add(&M.load[tt], 1);
      g_add(&M.load[me], -1);
      g_add(&M.hdr[MIG_WAITING], -1);
      g_add(&M.hdr[MIG_MOVES], 1);
    }
    image_out(P.mig_img + (size_t)(tt * GMAX + slot) * P.mig_img_words);
    // one wave-wide release (the L2 write-back of every lane's image stores) publishes
    // the image to the receiver's XCD; the mailbox store itself is then relaxed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0)
      __hip_atomic_store((int*)&M.mbox[tt * GMAX + slot], lc + 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  // the chain's LDS state at a transition boundary (scalars, vectors, sums, aux;
  // the tree levels are dead between transitions) <-> a global image
  __device__ void image_out(double* dst) const {
    const AS_LDS double* src = (const AS_LDS double*)Sp;
    for (int i = lane; i < Pr().mig_img_words; i += WAVE) ((AS_GLB double*)dst)[i] = src[i];
  }

  __device__ int act_finish() {
    FITOCT_MARK(act_finish);
    Sp->state = ST_DONE;
    const V q = ld(V_SMP_Q), minv = ld(V_MINV);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = idx(s);
      if (k < Pr().D) {
        if (Pr().fin_q) ((AS_GLB double*)Pr().fin_q)[(size_t)lc * Pr().D + k] = q.a[s];
        if (Pr().fin_minv) ((AS_GLB double*)Pr().fin_minv)[(size_t)lc * Pr().D + k] = minv.a[s];
      }
    }
    if (lane == 0) {
      if (Pr().fin_eps) ((AS_GLB double*)Pr().fin_eps)[lc] = Sp->eps;
      if (Pr().chain_status) ((AS_GLB int*)Pr().chain_status)[lc] = Sp->status;
      if (Pr().leapfrogs) ((AS_GLB long long*)Pr().leapfrogs)[lc] = Sp->leapfrogs;
    }
    return A_YIELD;
  }

  // run actions until the chain yields a position to the gradient waves (or finishes)
  __device__ __forceinline__ int run(int a) {
    for (;;) {
      FITOCT_MARK(dispatch);
      a = uni(a);
      // opaque per action: no jump threading across actions, and no address or
      // kernarg load hoisted out of the action loop (keeps register pressure local)
      {   // keep the block pointer provably wave-uniform (SGPRs) in every variant
        const uint64_t pv = (uint64_t)pp;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pv);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(pv >> 32));
        pp = (KPc*)(((uint64_t)hi << 32) | lo);
      }
      asm volatile("" : "+s"(a), "+s"(pp));
      if (a == A_YIELD || a == A_SPEC_STAGED || a == A_SPEC_WAIT || a == A_SPEC_DISCARD ||
          (kTwoEnded && a == A_BIDI_TREE))
        break;
      const bool prof = kProfile && Pr().stamps != nullptr;
      const long long t0 = prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
      const int a0 = a;
      switch (a) {
        case A_GRAD: a = act_grad(); break;
        case A_INIT_STATE: a = act_init_state(); break;
        case A_INIT_START: a = act_init_start(); break;
        case A_INIT_STEP: a = act_init_step(); break;
        case A_SS_BEGIN: a = act_ss_begin(); break;
        case A_SS_TRIAL: a = act_ss_trial(); break;
        case A_SS_STEP: a = act_ss_step(); break;
        case A_SS_FINISH: a = act_ss_finish(); break;
        case A_START_TRANSITION: a = act_start_transition(); break;
        case A_BEGIN_SUBTREE: a = act_begin_subtree(); break;
        case A_END_TREE: a = act_end_tree(); break;
        case A_NEXT_TRANSITION: a = act_next_transition(); break;
        case A_FINISH: a = act_finish(); break;
        case A_LEAPFROG: a = act_leapfrog(); break;
        case A_WRITE_MP: a = act_write_mp(); break;
        case A_PRIOR: a = act_prior(); break;
        case A_SPEC_BOOK: a = act_spec_book(); break;
        default: a = A_YIELD; break;
      }
      if (prof) {
        wave_fence();
        const int ai = (a0 == A_SPEC_BOOK) ? A_LEAF : a0;   // slot 11: the leaf's bookkeeping
        Sp->prof[0][ai] += (long long)__builtin_amdgcn_s_memtime() - t0;
        Sp->prof[1][ai] += 1;
      }
    }
    wave_publish();   // (the yielded position's MP before the kernel's ring entry)
    return a;
  }
};

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
template <int PPL, int NNP>
__device__ __forceinline__ void load_kinv(KPc& P, const Lds<PPL>& L, int tid) {
  if (P.mode == MODE_POLY) {  // zero-padded to NNP x NNP so the device loops are fixed-size
    const int Nn = P.Nn;
    for (int i = tid; i < KMAX * KMAX; i += TPB) {   // whole tile: no stale LDS is ever read
      const int r = i / NNP, c = i % NNP;
      L.kinv()[i] = (i < NNP * NNP && r < Nn && c < Nn) ? P.Kinv[r * Nn + c] : 0.0;
    }
    if (tid < NNP) L.bv()[tid] = (tid < Nn) ? P.bvec[tid] : 0.0;
  }
}

// LDS hand-off primitives between the waves of one tile (one CU: LDS is a
// single coherent memory, so a writer's ds ops completed under lgkmcnt(0) are
// visible to every later read of any wave).
__device__ __forceinline__ int lds_load(const int* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
__device__ __forceinline__ unsigned long long lds_load64(const unsigned long long* p) {
  return __atomic_load_n(p, __ATOMIC_RELAXED);
}
constexpr int RINGN = 16;                 // hand-off ring: >= 2 * GMAX entries

// Migration receiver: post NUTS slot c of this tile as free and wait until a
// crowded tile hands a chain over (returns its chain index, image loaded into
// the slot's LDS) or every chain of the launch has finished (returns -1).
// Receivers wait only once every tile of the launch has started: then no tile
// is waiting for a CU, so waiting cannot starve one.  An idle wait longer than
// MIG_WAIT_TICKS withdraws the post (if no donor claimed it meanwhile).
// The launch's tail (P.tail_bidi; at most P.tail_left chains left unfinished): a receiver
// whose tile hosts exactly one live chain withdraws its post and becomes one of that chain's
// two producers of two-ended trajectories (returns -2 - end; one claim bit per end in
// TW_CLAIM, the slot in TW_SLOT + end, TW_JOIN counts producers in place).  A tile whose
// claims are taken keeps its other free slots posted.
template <int PPL>
__device__ int receive_chain(KPc& P, const Lds<PPL>& L, int c, int lane, volatile AS_LDS int* bd,
                             const AS_LDS int* live) {
  const MigView M(P.mig, P.mig_tiles);
  const int me = blockIdx.x;
  if (__builtin_amdgcn_readfirstlane(g_load(&M.hdr[MIG_STARTED])) < P.mig_tiles) return -1;
  if (lane == 0) {
    g_or(&M.fmask[me], 1 << c);
    g_add(&M.hdr[MIG_WAITING], 1);
  }
  AS_GLB int* box = &M.mbox[me * GMAX + c];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int m = 0;
  // Poll with relaxed loads and acquire once the mailbox is set: an agent-scope acquire
  // invalidates this XCD's L2, and up to hundreds of receivers wait at the end of a launch
  // (each poll an invalidation would evict every tile's proposal pools on the XCD).
  for (;;) {
    m = __builtin_amdgcn_readfirstlane(g_load(box));
    if (m != 0) break;
    const int done = __builtin_amdgcn_readfirstlane(g_load(&M.hdr[MIG_DONE]));
    if (done >= P.chains) return -1;
    const int lv = __builtin_amdgcn_readfirstlane(*(volatile const AS_LDS int*)live);
    if (P.tail_bidi && P.chains - done <= P.tail_left && lv == 1 &&
        __builtin_amdgcn_readfirstlane(bd[TW_CLAIM]) != 3) {
      int r = -1;
      if (lane == 0) {
        for (int k = 0; k < 2 && r < 0; ++k)
          if (((atomicOr((int*)&bd[TW_CLAIM], 1 << k) >> k) & 1) == 0) r = k;
        if (r >= 0) {
          if ((g_and(&M.fmask[me], ~(1 << c)) >> c) & 1) {   // withdrawn: no migrant comes here
            g_add(&M.hdr[MIG_WAITING], -1);
            bd[TW_SLOT + r] = c;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            atomicAdd((int*)&bd[TW_JOIN], 1);
          } else {   // a donor claimed this slot first: receive its chain, free the end
            atomicAnd((int*)&bd[TW_CLAIM], ~(1 << r));
            r = -1;
          }
        }
      }
      r = __builtin_amdgcn_readfirstlane(__shfl(r, 0));
      if (r >= 0) return -2 - r;
    }
      if (__builtin_amdgcn_s_memrealtime() - t0 > MIG_WAIT_TICKS) {
      int still = 0;   // withdraw the post unless a donor already claimed it
      if (lane == 0) {
        still = (g_and(&M.fmask[me], ~(1 << c)) >> c) & 1;
        if (still) g_add(&M.hdr[MIG_WAITING], -1);
      }
      if (__shfl(still, 0)) return -1;
      while ((m = __builtin_amdgcn_readfirstlane(g_load(box))) == 0) __builtin_amdgcn_s_sleep(8);
      break;
    }
    __builtin_amdgcn_s_sleep(32);
  }
  // pairs with the donor's release store of the mailbox: the image is visible from here
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (lane == 0) __hip_atomic_store((int*)box, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const AS_GLB double* src =
      (const AS_GLB double*)P.mig_img + (size_t)(me * GMAX + c) * P.mig_img_words;
  AS_LDS double* dst = (AS_LDS double*)L.chain(c);
  for (int i = lane; i < P.mig_img_words; i += WAVE) dst[i] = src[i];
  wave_fence();
  return m - 1;
}

// Dataflow pipeline inside a tile.  The NUTS wave of chain c writes the next
// position's parameters to MP[c] and enqueues c in an LDS ring (64-bit entries
// {sequence number, chain}); the gradient waves drain the ring in order, each
// sweeping its bins for that chain and bumping grad_cnt[c]; the NUTS wave waits
// until grad_cnt[c] reaches NGW * epoch and runs the sampler until it yields
// the next position.  Chains cycle independently (no barrier after start-up),
// so the sampler latency of one chain hides behind the sweeps of the others.
//
// Batch mode (fitoct_batch_*, FitOCT.R's loop over files): Pg is an array of
// parameter blocks, one per problem, and tile_map[2*tile] = {problem, first
// chain} places each tile; a tile never mixes problems, so every tile still
// keeps one problem's bins in registers.  tile_map == nullptr: one problem.
//
// Paired tiles (P.pair, one-chain tiles with two-ended trajectories, 2 x tiles <= CUs): block
// b is tile (b / 16) * 8 + b % 8 in the role (b / 8) % 2 -- 0: the primary, which hosts the
// chain, its helper and the backward end's producer; 1: its partner, which grows the forward
// end on its own gradient waves.  Blocks b and b + 8 (one XCD when blocks are dealt round-robin
// over the 8 XCDs; for speed only, the hand-off is correct on any placement) form a pair.
// PAIR: the paired launch (one-chain tiles with two-ended trajectories and partners; MIG =
// false, SPEC = true): its own instantiation, so that neither the bridges nor the partner's
// roles cost the unpaired kernels registers
template <class R, int BPT, int NNP, int PPL, int MODE, int FAM, bool MIG, bool SPEC, bool PAIR>
__global__ void __launch_bounds__(TPB, 2) nuts_kernel(const KParams* __restrict__ Pg,
                                                      const int* __restrict__ tile_map) {
  // the basis mode as a constant of the sampler's chain code (config 5 at one GPU +3 %), but
  // for the paired row-mode sampler, which reads it (config 2 +1.7 %: the compiler's schedule
  // of the producers; same-box A/B, profiles/r06_ab_rows.txt)
  constexpr int CMODE = (SPEC && PAIR && MODE == MODE_ROWS) ? -1 : MODE;
  int tix = blockIdx.x, role = 0;
  if constexpr (PAIR) {
    role = (tix >> 3) & 1;
    tix = ((tix >> 4) << 3) | (tix & 7);
    if (tix >= ((KPc*)Pg)->pair_tiles) return;   // the grid's padding to whole groups of 16
  }
  int pidx = 0, c0;
  if (tile_map) {
    const AS_CST int* tm = (const AS_CST int*)tile_map;
    pidx = __builtin_amdgcn_readfirstlane(tm[2 * tix]);
    c0 = __builtin_amdgcn_readfirstlane(tm[2 * tix + 1]);
  } else {
    c0 = tix * ((KPc*)Pg)->G;
  }
  KPc& P = *((KPc*)Pg + pidx);   // device-resident parameter block: uniform s_load reads
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // two-ended trajectories carve two more chain areas (the producers' slots 1, 2)
  const Lds<PPL> L{(AS_LDS char*)smem, P.bidi ? 3 : P.G, Lds<PPL>::chain_bytes(P.max_depth)};
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nct = min(P.G, P.chains - c0);
  __shared__ unsigned long long ring[RINGN];
  __shared__ int q_reserve, n_active, grad_cnt[GMAX];
  // post a sweep of chain slot s (lane 0 of the posting wave; its MP writes are in before):
  // sequence number from a ring-wide counter, one 64-bit store.  (Per-slot doorbells without
  // the atomic's return measured -3 to -6 %, gradient waves at priority 2-3 during sweeps
  // -16 to -19 % on config 2: profiles/r06_ab_rows.txt.)
  auto post_sweep = [&](const int s) {
    const unsigned rs = (unsigned)atomicAdd(&q_reserve, 1);
    __atomic_store_n(&ring[rs % RINGN], ((unsigned long long)rs << 32) | (unsigned)s, __ATOMIC_RELAXED);
  };
  __shared__ int bd[BD_N];   // two-ended trajectories' hand-off words (BdWord)
  __shared__ long long done_t[GMAX];   // profiling build: when the 8th wave finished chain c
  __shared__ long long start_min[GMAX], start_max[GMAX];
  // speculative leaves (P.spec, tiles of one or two chains): chain slot c's NUTS wave posts
  // a request for the bookkeeping of its leaf (deep: the leaf in HX[c]) or the prior part of
  // a speculated position; its helper wave (NUTS wave G + c) runs it and publishes the
  // request number it finished
  __shared__ int help_req[2], help_done[2], help_res[2], help_seen[2], help_gen[2], help_m[2],
      help_dead[2];
  const bool spec = SPEC;
  const bool helped = SPEC && !MIG && P.G <= 2;   // spare NUTS waves help the tile's chains
  const bool bidi = Chain<PPL, NNP, FAM, MIG, SPEC, CMODE>::kTwoEnded && helped &&
                   P.bidi != 0;   // ... and two producer waves
  __shared__ int live_chains;   // chains the tile hosts (speculation policy, Chain::live)
  // paired tiles: this pair's hand-off words and buffer; pair_on: the partner has joined
  // (partner tile: 1 = it grows the forward end, 0 = it leaves at once)
  const bool paired = PAIR && bidi;
  AS_GLB int* const xh = paired ? (AS_GLB int*)P.pair_hdr + (size_t)tix * PAIR_HDR_INTS : nullptr;
  AS_GLB double* const xb = paired ? (AS_GLB double*)P.pair_buf + (size_t)tix * P.pair_stride : nullptr;
  __shared__ int pair_on;

  load_kinv<PPL, NNP>(P, L, tid);
  if (tid == 0) {
    q_reserve = 0;
    n_active = nct;
    live_chains = nct;
    pair_on = 0;
    if (paired && role == 0 && nct > 0) __hip_atomic_fetch_or(xh + PH_STATE, PS_START, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
    if (paired && role == 1) {
      // join once the primary has begun; give up (LOCAL) if it has not within PAIR_JOIN_TICKS
      // (the blocks of a launch start within a microsecond of each other on an idle chip; the
      // primary decides only at its chain's first transition, many gradients later)
      bool join = false;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (int st = x_ldi(xh + PH_STATE); !P.pair_test_absent;) {
        if (st & PS_LOCAL) break;
        int expect = st & PS_START ? st : 0;
        const int want = st & PS_START ? st | PS_JOIN : PS_LOCAL;
        if (!(st & PS_START) && __builtin_amdgcn_s_memrealtime() - t0 < PAIR_JOIN_TICKS) {
          __builtin_amdgcn_s_sleep(2);
          st = x_ldi(xh + PH_STATE);
          continue;
        }
        if (__hip_atomic_compare_exchange_strong(xh + PH_STATE, &expect, want, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          join = (want & PS_JOIN) != 0;
          break;
        }
        st = expect;   // the primary began (or decided) meanwhile: look again
      }
      if (!join) __hip_atomic_fetch_or(xh + PH_STATE, PS_LOCAL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pair_on = join ? 1 : 0;
      n_active = join ? 1 : 0;   // the partner's bridge wave ends its gradient waves
    }
  }
  if (tid < 2) {
    // (a partner tile has no backward-end producer: its helper serves producer 1 only)
    help_req[tid] = (role == 1 && tid == 0) ? -1 : 0;
    help_done[tid] = 0;
    help_res[tid] = 0;
    help_seen[tid] = 0;
    help_gen[tid] = 0;
    help_m[tid] = 0;
    help_dead[tid] = 0;
  }
  if (tid < GMAX) {
    grad_cnt[tid] = 0;
    done_t[tid] = 0;
    start_min[tid] = 0x7FFFFFFFFFFFFFFFLL;
    start_max[tid] = 0;
  }
  if (tid < RINGN) ring[tid] = ~0ULL;
  // (a tile of one chain: the producers' areas are NUTS slots 1 and 2)
  if (tid < BD_N) bd[tid] = (tid == TW_SLOT) ? 1 : (tid == TW_SLOT + 1) ? 2 : 0;
  if (MIG && P.mig != nullptr) {   // every slot of the tile may host migrants: all NUTS waves live
    if (tid == 0) {
      const MigView M(P.mig, P.mig_tiles);
      n_active = P.G;
      __hip_atomic_store((int*)&M.load[tix], nct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((int*)&M.hdr[MIG_STARTED], 1, __ATOMIC_RELAXED,   // a count: no data
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();

  const bool stamp = kProfile && (P.stamps != nullptr) && role == 0 && lane == 0 && (wave == 0 || wave == NGW);
  const bool wstamp = kProfile && (P.stamps != nullptr) && role == 0 && lane == 0 && wave < NGW;
  long long t_wbusy = 0;
  long long t_busy = 0, n_items = 0, t_wait = 0, t_enq = 0, t_sweep = 0, t_notice = 0;
  long long t_st0 = 0, t_st1 = 0;
  long long t_begin = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
  // tile timeline (profiling build): start, first chain finished, end, on the 100 MHz clock
  __shared__ long long first_done_rt;
  __shared__ int chains_done_here;
  const long long rt_begin = kProfile ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  if (kProfile && tid == 0) {
    first_done_rt = 0;
    chains_done_here = 0;
  }
  if (kProfile) __syncthreads();
  if (wave < NGW) {  // ------------------------- gradient waves
    Bins<R, BPT, NNP, MODE> bins;
    bins.load(P, tid);
    int zero_done[GMAX] = {0, 0, 0, 0};
    // profiling build: tile occupancy -- real time and sweeps by the tile's live chains
    // (0..4) at each ring entry (wave 0; the tail of a launch is its thinned-out tiles)
    long long occ_t[GMAX + 1] = {0, 0, 0, 0, 0}, occ_n[GMAX + 1] = {0, 0, 0, 0, 0};
    long long occ_last = kProfile ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    int occ_k = GMAX;
    for (unsigned h = 0;; ++h) {
      unsigned long long e;
      bool stop = false;
      Patience w;
      for (;;) {  // wait for ring entry h
        e = lds_load64(&ring[h % RINGN]);
        if ((unsigned)(e >> 32) == h) break;
        if (lds_load(&n_active) == 0) {
          stop = true;
          break;
        }
        // hang guard: with migration a tile may idle (receivers posted) until the launch's
        // last chain ends; without, its chains may pause between sweeps (a two-ended tree's
        // chain wave, init) but never for a leaf's wait bound
        if (w.expired(MIG_WAIT_TICKS + 10 * TICKS_PER_S)) {
          stop = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (stop) break;
      const int c = (int)(e & 0xFF);
      if (kProfile && wave == 0 && P.stamps != nullptr) {
        const long long now = (long long)__builtin_amdgcn_s_memrealtime();
        occ_t[occ_k] += now - occ_last;   // the interval since the last entry, at its count
        occ_last = now;
        occ_k = min(max(lds_load(&live_chains), 0), GMAX);
        ++occ_n[occ_k];
      }
      const long long s0 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
      const long long s0w = wstamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
      if (kProfile && lane == 0) {   // sweep start spread over the 8 waves
        const unsigned long long t = (unsigned long long)__builtin_amdgcn_s_memtime();
        atomicMin((unsigned long long*)&start_min[c], t);
        atomicMax((unsigned long long*)&start_max[c], t);
      }
      if (P.prior_PD == 0)
        gradient_pass<R, BPT, NNP, MODE, true>(P, bins, L.mp(0), L.part(), zero_done, c, c + 1,
                                               tid, lane, wave);
      wave_publish();   // this wave's PART writes before its count
      if (wstamp) t_wbusy += (long long)__builtin_amdgcn_s_memtime() - s0w;
      if (lane == 0) {
        if (kProfile)   // latest finisher's time; LDS ops of a wave complete in order
          atomicMax((unsigned long long*)&done_t[c], (unsigned long long)__builtin_amdgcn_s_memtime());
        atomicAdd(&grad_cnt[c], 1);
      }
      if (stamp) {
        t_busy += (long long)__builtin_amdgcn_s_memtime() - s0;
        ++n_items;
      }
    }
    if (kProfile && role == 0 && wave == 0 && lane == 0 && P.stamps != nullptr) {
      AS_GLB long long* o = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP;
      // (the interval after the last entry: the tile's live count now, normally 0 -- a
      // tile whose chains have finished waits for migrants, or the launch's end)
      occ_t[min(max(lds_load(&live_chains), 0), GMAX)] +=
          (long long)__builtin_amdgcn_s_memrealtime() - occ_last;
      for (int k = 0; k <= GMAX; ++k) {
        o[72 + k] = occ_t[k];
        o[77 + k] = occ_n[k];
      }
    }
  } else {           // ------------------------- NUTS waves
    // the sampler is the latency-critical stage and shares each SIMD with two
    // throughput-bound gradient waves: let it win issue arbitration
    // (priority 2 / 1 / 0: -0.3 % / +-0 / -23 % on config 3)
    __builtin_amdgcn_s_setprio(3);
    const int c = wave - NGW;
    const bool mig = MIG && P.mig != nullptr;
    using Ch = Chain<PPL, NNP, FAM, MIG, SPEC, CMODE>;
    // Two-ended trajectories: producer of trajectory end s (0: backward, 1: forward) on NUTS
    // slot `slot` (its chain area holds the end's state, its subtree's levels and merge
    // uniforms, and its last subtree's record; its proposal pool is its own).  For every
    // transition g the chain starts (BD_GEN), it builds the subtrees of the doublings drawn in
    // direction s from the start outwards (Chain::sub_leaf), at most BIDI_LOOK doublings past
    // the one booked, and publishes one record per subtree once the booking has taken the
    // previous one.  `epoch`: the slot's sweeps so far (grad_cnt[slot] counts NGW per sweep).
    // Ends with BD_GEN < 0 (the tile's chain finished) or, in a migrating tile, with the launch.
    auto produce = [&](const int s, const int slot, long long epoch) {
      // helped: another wave books this end's leaves (serve: tiles of one chain -- the backward
      // end the booking helper; the forward end the partner tile's helper, or in an unpaired
      // row-mode tile the chain's wave while it waits for records), else the producer books them
      // itself (an unpaired tile with the factorised basis, whose registers have no room for the
      // chain's serving; a migrating launch's tail)
      const bool helped = !MIG && (s == 0 || PAIR || MODE == MODE_ROWS);
      int hreq = 0;   // leaves handed to the helper
      Ch pr(P, L, slot, c0, lane, nct);
      pr.bd = (volatile AS_LDS int*)bd;
      pr.pix = P.chains + (c0 / P.G) * GMAX + slot;   // its own proposal pool region
      int seen = 0;
      bool quit = false;
      // profiling build: cycles waiting for sweeps, for the lookahead / ring room, leaves,
      // and cycles inside trees
      long long pf_sw = 0, pf_may = 0, pf_n = 0, pf_tree = 0;
      // (and per leaf: finish_grad + end_update_p, staging the next leaf, the hand-over, prior_part)
      long long pf_fg = 0, pf_st = 0, pf_ho = 0, pf_pp = 0;
      auto pclk = [&]() -> long long { return kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0; };
      while (!quit) {
        int g;
        {
          Patience w;
          int polls = 0;
          const unsigned long long t_idle = MIG ? __builtin_amdgcn_s_memrealtime() : 0;
          const unsigned long long idle_max = P.tail_idle_ticks ? P.tail_idle_ticks : MIG_WAIT_TICKS;
          while ((g = lds_load(&bd[BD_GEN])) == seen || (g > 0 && (g & BD_ENDED))) {
            if (MIG) {
              // a tail producer idle this long leaves -- but only once it holds TW_BUSY, so no
              // chain claims the pair while it withdraws its role (TW_JOIN, its TW_CLAIM bit):
              // a chain never waits for records of a producer that has gone.  While
              // a chain holds TW_BUSY its tree is under way and the producer stays.
              if (__builtin_amdgcn_s_memrealtime() - t_idle > idle_max) {
                int gone = 0;
                if (lane == 0 && atomicCAS((int*)&bd[TW_BUSY], 0, 2) == 0) {
                  atomicSub((int*)&bd[TW_JOIN], 1);
                  atomicAnd((int*)&bd[TW_CLAIM], ~(1 << s));
                  __atomic_store_n(&bd[TW_BUSY], 0, __ATOMIC_RELAXED);
                  gone = 1;
                }
                if (__builtin_amdgcn_readfirstlane(__shfl(gone, 0))) {
                  quit = true;
                  break;
                }
              }
            } else if (w.expired(MIG_WAIT_TICKS)) {
              quit = true;
              break;
            }
            if (MIG && (++polls & 255) == 0 &&
                __builtin_amdgcn_readfirstlane(g_load(&MigView(P.mig, P.mig_tiles).hdr[MIG_DONE])) >=
                    P.chains) {
              quit = true;
              break;
            }
            __builtin_amdgcn_s_sleep(MIG ? 8 : 1);
          }
        }
        if (quit || g < 0) break;
        seen = g;
        wave_fence();
        // the chain being grown: its key (direction draws) and its scalars (booked depth)
        const int lcg = lds_load(&bd[TW_LC]);
        pr.key = make_key(P.seed, (uint32_t)(P.chain_offset + lcg));
        const AS_LDS ChainScalars& S0 = L.cs(lds_load(&bd[TW_CHAIN]));
        Vd<PPL> q = pr.ld(V_E0_Q), p = pr.ld(V_E0_P), gr = pr.ld(V_E0_G);
        const Vd<PPL> minv = pr.ld(V_MINV);
        const double eps = pr.Sp->eps_used;
        const uint32_t t = (uint32_t)pr.uni(pr.Sp->t);
        // bit k: doubling k grows in direction s (act_begin_subtree's draws)
        const bool mine = lane < P.max_depth &&
                          ((uniform(pr.key, t, TAG_DIR, (uint32_t)lane, 0u) > 0.5) ? 1 : 0) == s;
        const unsigned long long dmask = __builtin_amdgcn_ballot_w64(mine);
        wave_fence();
        if (lds_load(&bd[BD_GEN]) != g) continue;   // the start was rewritten while read
        const double e = s ? eps : -eps;
        // this end's next doubling after depth d (-1: none)
        auto next_depth = [&](const int d) -> int {
          const unsigned long long r = d < 0 ? dmask : dmask & ~((2ULL << d) - 1);
          return r ? (int)__builtin_ctzll(r) : -1;
        };
        // may the subtree of depth d grow now: within BIDI_LOOK doublings of the booked depth.
        // Once true it stays true for the transition (the booked depth only grows)
        auto may = [&](const int d) -> bool {
          return d <= pr.uni(*(volatile const AS_LDS int*)&S0.depth) + BIDI_LOOK;
        };
        const long long pft0 = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
        auto wait_may = [&](const int d) -> bool {   // false: the tree ended
          Patience w;
          const long long pt = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
          for (;;) {
            if (lds_load(&bd[BD_GEN]) != g) {
              if (kProfile) pf_may += (long long)__builtin_amdgcn_s_memtime() - pt;
              return false;
            }
            if (may(d)) {
              if (kProfile) pf_may += (long long)__builtin_amdgcn_s_memtime() - pt;
              return true;
            }
            // the other end may grow for long (deep trees, large N).  In effect this wait
            // ends with BD_GEN: its bound outlasts the bound on the whole tree (MIG_WAIT_TICKS
            // from the tree's start), after which BD_GEN changes
            if (w.expired(2 * MIG_WAIT_TICKS)) return false;
            __builtin_amdgcn_s_sleep(1);
          }
        };
        // record m's slot is free once the booking has taken record m - RSLOTS
        auto wait_room = [&](const int m) -> bool {   // false: the tree ended
          Patience w;
          const long long pt = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
          for (;;) {
            if (lds_load(&bd[BD_GEN]) != g) return false;
            if (lds_load(&bd[BD_CONS + s]) >= m - Ch::RSLOTS + 1) {
              if (kProfile) pf_may += (long long)__builtin_amdgcn_s_memtime() - pt;
              return true;
            }
            if (w.expired(2 * MIG_WAIT_TICKS)) return false;
            __builtin_amdgcn_s_sleep(1);
          }
        };
        // expl_leapfrog from the last leaf of this end (begin_update_p, update_q), staged for
        // the gradient waves and enqueued; the position-only prior terms overlap the sweep
        Vd<PPL> p1, q1;
        auto stage = [&](const Vd<PPL>& qa, const Vd<PPL>& pa, const Vd<PPL>& ga) {
#pragma unroll
          for (int k = 0; k < PPL; ++k) {
            p1.a[k] = fma(0.5 * e, ga.a[k], pa.a[k]);
            q1.a[k] = fma(e, minv.a[k] * p1.a[k], qa.a[k]);
          }
          pr.write_mp(q1);
          if (lane == 0) post_sweep(slot);
          ++epoch;
        };
        int d = next_depth(-1);
        if (d < 0 || !wait_may(d)) continue;
        if (!helped) pr.sub_begin(d);   // (helped: the helper begins a subtree at its leaf 0)
        int m = 0;   // subtree records published this transition (not helped)
        int j = 0;   // the leaf in its sweep: leaf j of the subtree of depth d
        stage(q, p, gr);
        pr.prior_part();
        // a leaf is in its sweep here.  Once it is in, the next one (in this subtree, or the
        // first of this end's next subtree if that may grow already) is staged first and the
        // leaf's bookkeeping runs during that sweep: the next position depends only on this
        // leaf's q, p and g (if the bookkeeping ends the subtree, that sweep is dropped)
        for (;;) {
          bool late = false;
          Patience ws;
          const long long pt = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
          while (lds_load(&grad_cnt[slot]) < (int)(NGW * epoch)) {
            if (ws.expired(LEAF_WAIT_TICKS)) {
              late = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (kProfile) {
            pf_sw += (long long)__builtin_amdgcn_s_memtime() - pt;
            ++pf_n;
          }
          if (late) {
            quit = true;
            break;
          }
          wave_fence();
          long long pc0 = pclk();
          // read with the partial sums (its latency hides in finish_grad's): a leaf the tree
          // no longer needs is dropped
          const int gen_now = lds_load(&bd[BD_GEN]);
          Vd<PPL> gn;
          double s2;
          const double lp = pr.finish_grad(gn, s2);
          Vd<PPL> pe;
#pragma unroll
          for (int k = 0; k < PPL; ++k) pe.a[k] = fma(0.5 * e, gn.a[k], p1.a[k]);   // end_update_p
          if (gen_now != g) break;   // the tree has ended: the leaf is not needed
          const Vd<PPL> qn = q1;
          const bool last = j == (1 << d) - 1;
          const int dn = last ? next_depth(d) : d;
          const bool nxt = !last || (dn >= 0 && may(dn));
          if (kProfile) {
            const long long pc1 = pclk();
            pf_fg += pc1 - pc0;
            pc0 = pc1;
          }
          if (nxt) stage(qn, pe, gn);
          if (kProfile) {
            const long long pc1 = pclk();
            pf_st += pc1 - pc0;
            pc0 = pc1;
          }
          if (helped) {
            // hand this leaf to the booking helper (two slots: once it has booked the leaf
            // before the previous one); stop when a booking cut its subtree (nothing later on
            // this end is needed)
            if (hreq > 0) {
              Patience wh;
              bool gone = false;
              while (lds_load(&help_done[s]) < hreq - 1) {
                if (lds_load(&bd[BD_GEN]) != g || wh.expired(LEAF_WAIT_TICKS)) {
                  gone = true;
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
              if (gone) break;
              const int res = lds_load(&help_res[s]);
              if ((res >> 2) == g && (res & 3) == Ch::SL_END) break;
            }
            AS_LDS double* X = L.px(s, (hreq + 1) & 1);
#pragma unroll
            for (int k = 0; k < PPL; ++k) {
              X[pr.idx(k)] = qn.a[k];
              X[Ch::VLEN + pr.idx(k)] = pe.a[k];
              X[2 * Ch::VLEN + pr.idx(k)] = gn.a[k];
            }
            if (lane == 0) {
              X[3 * Ch::VLEN] = lp;
              X[3 * Ch::VLEN + 1] = s2;
              X[3 * Ch::VLEN + 2] = (double)d;
              X[3 * Ch::VLEN + 3] = (double)j;
              X[3 * Ch::VLEN + 4] = (double)g;
            }
            wave_publish();   // the leaf lands before its request number
            ++hreq;
            if (lane == 0) __atomic_store_n(&help_req[s], hreq, __ATOMIC_RELAXED);
            if (kProfile) {
              const long long pc1 = pclk();
              pf_ho += pc1 - pc0;
              pc0 = pc1;
            }
            if (last) {
              if (dn < 0) break;   // this end has no further doubling in this tree
              if (!nxt) {
                if (!wait_may(dn)) break;
                stage(qn, pe, gn);
              }
              d = dn;
              j = 0;
            } else {
              ++j;
            }
            pr.prior_part();
            if (kProfile) pf_pp += pclk() - pc0;
            continue;
          }
          XF Tw{0.0, 0};
          int Tprop = -1;
          Vd<PPL> Tpb = pe, Trho = pe;
          double h = 0.0;
          const int r = pr.sub_leaf(qn, pe, gn, minv, lp, s2, Tw, Tprop, Tpb, Trho, h);
          if (r != Ch::SL_MID) {   // the subtree is complete (or cut): its record for the booking
            if (!wait_room(m)) break;
            const int fl = r == Ch::SL_DONE ? Ch::SR_VALID
                                            : pr.uni(pr.Sp->divergent) ? Ch::SR_DIVERGENT : 0;
            pr.sub_publish(s, m, fl, Tw, Tprop, Tpb, Trho, qn, pe, gn, lp, s2, h);
            wave_publish();   // the record lands before its count
            ++m;
            if (lane == 0) __atomic_store_n(&bd[BD_PROD + s], (g << 16) | m, __ATOMIC_RELAXED);
            if (r == Ch::SL_END || dn < 0) break;   // this end adds nothing more to the tree
            if (!nxt) {
              if (!wait_may(dn)) break;
              stage(qn, pe, gn);
            }
            d = dn;
            j = 0;
            pr.sub_begin(d);
          } else {
            ++j;
          }
          pr.prior_part();
        }
        if (kProfile) pf_tree += (long long)__builtin_amdgcn_s_memtime() - pft0;
      }
      if (helped && lane == 0) __atomic_store_n(&help_req[s], -1, __ATOMIC_RELAXED);   // its helper may leave
      if (kProfile && P.stamps != nullptr && lane == 0) {   // this end's producer (either tile)
        AS_GLB long long* o = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP + 88 + 4 * s;
        o[0] = pf_sw;
        o[1] = pf_may;
        o[2] = pf_n;
        o[3] = pf_tree;
        AS_GLB long long* o2 = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP + 100 + 4 * s;
        o2[0] = pf_fg;
        o2[1] = pf_st;
        o2[2] = pf_ho;
        o2[3] = pf_pp;
      }
    };
    // Two-ended trajectories in a tile of one chain: the booking helper (NUTS wave 1 of the tile,
    // and of a partner tile) books the leaves its producers hand over -- Chain::sub_leaf on the
    // producer's own chain area, its subtree record once the subtree ends (when the booking has
    // taken the previous one) -- while the producer completes the next gradient and stages the
    // one after.  One request of producer s: 1 served, 0 none pending, -1 the producer is gone.
    // (help_seen / help_gen / help_m: requests served, and the transition and records published
    // of producer s, kept by the helper.)
    // nb (the chain's wave serving the forward end of an unpaired tile): serve a leaf only if its
    // subtree's record would find its slot free -- that wave alone frees the slots, so it must
    // never wait for one here.  0 then: not served (the request stays pending).
    auto serve = [&](const int s, const bool nb) -> int {
      const int rq0 = lds_load(&help_req[s]);
      if (rq0 < 0) return -1;
      const int rq = lds_load(&help_seen[s]) + 1;   // requests are served in order
      if (rq > rq0) return 0;
      wave_fence();   // the leaf after its request number
      Ch hc(P, L, 1 + s, c0, lane, nct);
      hc.bd = (volatile AS_LDS int*)bd;
      hc.pix = P.chains + (c0 / P.G) * GMAX + 1 + s;
      const AS_LDS double* X = L.px(s, rq & 1);
      Vd<PPL> q, pe, gg;
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        q.a[k] = X[hc.idx(k)];
        pe.a[k] = X[Ch::VLEN + hc.idx(k)];
        gg.a[k] = X[2 * Ch::VLEN + hc.idx(k)];
      }
      const double lp = X[3 * Ch::VLEN], s2 = X[3 * Ch::VLEN + 1];
      const int d = __builtin_amdgcn_readfirstlane((int)X[3 * Ch::VLEN + 2]);
      const int j = __builtin_amdgcn_readfirstlane((int)X[3 * Ch::VLEN + 3]);
      const int gen = __builtin_amdgcn_readfirstlane((int)X[3 * Ch::VLEN + 4]);
      int r = Ch::SL_END;
      // (else a leaf of a tree that has ended, or of a subtree a booking has cut: help_dead)
      if (lds_load(&bd[BD_GEN]) == gen &&
          !(lds_load(&help_gen[s]) == gen && lds_load(&help_dead[s]) == gen)) {
        hc.key = make_key(P.seed, (uint32_t)(P.chain_offset + lds_load(&bd[TW_LC])));
        int hm = lds_load(&help_m[s]);
        if (lds_load(&help_gen[s]) != gen) hm = 0;
        if (nb && lds_load(&bd[BD_CONS + s]) < hm - Ch::RSLOTS + 1) return 0;
        if (j == 0) hc.sub_begin(d);
        XF Tw{0.0, 0};
        int Tprop = -1;
        Vd<PPL> Tpb = pe, Trho = pe;
        double h = 0.0;
        r = hc.sub_leaf(q, pe, gg, hc.ld(V_MINV), lp, s2, Tw, Tprop, Tpb, Trho, h);
        if (r != Ch::SL_MID) {   // the subtree ended: its record, once the slot is free
          Patience w;
          bool room = true;
          while (lds_load(&bd[BD_CONS + s]) < hm - Ch::RSLOTS + 1) {
            if (lds_load(&bd[BD_GEN]) != gen || w.expired(2 * MIG_WAIT_TICKS)) {
              room = false;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (room) {
            const int fl = r == Ch::SL_DONE ? Ch::SR_VALID
                                            : hc.uni(hc.Sp->divergent) ? Ch::SR_DIVERGENT : 0;
            hc.sub_publish(s, hm, fl, Tw, Tprop, Tpb, Trho, q, pe, gg, lp, s2, h);
            wave_publish();   // the record lands before its count
            ++hm;
            if (lane == 0) __atomic_store_n(&bd[BD_PROD + s], (gen << 16) | hm, __ATOMIC_RELAXED);
          } else {
            r = Ch::SL_END;
          }
        }
        if (lane == 0) {
          help_m[s] = hm;
          help_gen[s] = gen;
          if (r == Ch::SL_END) help_dead[s] = gen;
        }
      }
      wave_publish();   // the booking's LDS writes land before its result
      if (lane == 0) {
        help_seen[s] = rq;
        __atomic_store_n(&help_res[s], (gen << 2) | r, __ATOMIC_RELAXED);
        wave_publish();
        __atomic_store_n(&help_done[s], rq, __ATOMIC_RELAXED);
      }
      return 1;
    };
    // ---- paired tiles (P.pair): the bridge waves.  The forward end's producer runs unchanged
    // in the partner tile (NUTS wave 3, chain area 2); two bridge waves make the pair look like
    // one tile to it and to the primary's booking:
    //   bridge_in (primary, NUTS wave 3, where that producer would run): each transition's start
    //     (producer area 2, written by bidi_begin) and the end of each tree, and the booking's
    //     progress (records of the forward end taken, booked depth) out to the pair's words;
    //     the partner's subtree records in, into the primary's area 2, published as a local
    //     producer would (BD_PROD + 1);
    //   bridge_out (partner, NUTS wave 2): the start into the producer's area and BD_GEN; the
    //     booking's progress into BD_CONS + 1 and the depth the producer's lookahead reads;
    //     the producer's records out to the pair's record slot, then PH_COUNT.
    // A record reaches the booking only through both bridges, and the producer writes record
    // m only once the (mirrored, never larger) count of records booked is m, so one count
    // guards the record's three slots.  Counts and the booked depth carry their transition
    // (gen << 16) and only grow within it.
    constexpr int QXD = Lds<PPL>::QX_DOUBLES;   // a record: Ch::RVEC vectors, then scalars
    constexpr int RVD = Ch::RVEC * Ch::VLEN;
    auto pair_start = [&]() { return xb; };
    // the pair's record slot k (the forward end's records m, k = m % 2): vectors, scalars
    auto pair_rec = [&](const int k) { return xb + 4 * Ch::VLEN + PAIR_START_DOUBLES + k * QXD; };
    // end 1's record slot k in this tile (Chain::rvec / rsc)
    auto fwd_vec = [&](const int k) -> AS_LDS double* {
      if constexpr (Ch::RSLOTS == 1) return L.vecs(2) + V_E1_Q * Ch::VLEN;
      else return L.qx0() + (2 + k) * QXD;
    };
    auto fwd_sc = [&](const int k) -> AS_LDS double* {
      if constexpr (Ch::RSLOTS == 1) return L.vecs(2) + V_RHO * Ch::VLEN;
      else return fwd_vec(k) + RVD;
    };
    auto bridge_in = [&]() -> bool {   // false: the pair did not form (grow the end here)
      {
        Patience w;   // the chain's first transition (or its end)
        while (lds_load(&bd[BD_GEN]) == 0 && !w.expired(MIG_WAIT_TICKS)) __builtin_amdgcn_s_sleep(1);
      }
      int st = 0;
      if (lane == 0) {
        int expect = PS_START;
        st = __hip_atomic_compare_exchange_strong(xh + PH_STATE, &expect, PS_START | PS_LOCAL,
                                                  __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                 ? PS_START | PS_LOCAL
                 : expect;
      }
      st = __builtin_amdgcn_readfirstlane(__shfl(st, 0));
      if ((st & PS_LOCAL) || !(st & PS_JOIN)) return false;
      constexpr int VL = Ch::VLEN;
      AS_GLB double* const xs = pair_start();

      AS_LDS double* const av = L.vecs(2);        // producer area 2: the start, the record
      AS_LDS ChainScalars* const as = &L.cs(2);
      const volatile AS_LDS int* depth = (const volatile AS_LDS int*)&L.cs(0).depth;
      int seen = 0, copied = 0, last_cons = -1, last_depth = -1;
      Patience idle;
      for (;;) {
        const int g = lds_load(&bd[BD_GEN]);
        if (g != seen) {
          if (g < 0) {
            if (lane == 0) x_sti(xh + PH_GEN, -1);
            break;
          }
          if (!(g & BD_ENDED)) {   // a new transition: its start first
            wave_fence();   // the start after its number
#pragma unroll
            for (int s = 0; s < PPL; ++s) {
              const int k = s * WAVE + lane;
              x_st(xs + k, av[V_E0_Q * VL + k]);
              x_st(xs + VL + k, av[V_E0_P * VL + k]);
              x_st(xs + 2 * VL + k, av[V_E0_G * VL + k]);
              x_st(xs + 3 * VL + k, av[V_MINV * VL + k]);
            }
            if (lane == 0) {
              x_st(xs + 4 * VL, as->eps_used);
              x_st(xs + 4 * VL + 1, as->H0);
              x_sti(xh + PH_T, as->t);
              x_sti(xh + PH_LC, lds_load(&bd[TW_LC]));
            }
            x_drain();   // the start has reached memory before its number
          }
          if (lane == 0) {
            x_sti(xh + PH_GEN, g);   // (a tree's end: its number with BD_ENDED)
            if (!(g & BD_ENDED)) atomicAdd(P.pair_count, 1ULL);
          }
          seen = g;
          copied = 0;
          last_cons = last_depth = -1;
          idle = Patience{};
          continue;
        }
        // the booking's progress on the forward end, for the partner's lookahead and record slot
        const int cons = lds_load(&bd[BD_CONS + 1]);
        const int dep = *depth;
        if (lds_load(&bd[BD_GEN]) == seen) {
          if (lane == 0 && cons != last_cons) x_sti(xh + PH_CONS, (seen << 16) | cons);
          if (lane == 0 && dep != last_depth) x_sti(xh + PH_DEPTH, (seen << 16) | dep);
          last_cons = cons;
          last_depth = dep;
        }
        // the partner's next record of this transition
        const int pc = __builtin_amdgcn_readfirstlane(x_ldi(xh + PH_COUNT));
        if ((pc >> 16) == seen && (pc & 0xFFFF) > copied) {
          const int cnt = pc & 0xFFFF;
          for (int n = copied; n < cnt; ++n) {   // records n: the pair's slot -> end 1's slot
            const AS_GLB double* src = pair_rec(n & 1);
            AS_LDS double* dv = fwd_vec(n & 1);
            AS_LDS double* ds = fwd_sc(n & 1);
            for (int i = lane; i < QXD; i += WAVE) {
              const double v = x_ld(src + i);
              if (i < RVD) dv[i] = v;
              else ds[i - RVD] = v;
            }
          }
          wave_publish();   // the records land before their count
          copied = cnt;
          if (lane == 0) __atomic_store_n(&bd[BD_PROD + 1], (seen << 16) | copied, __ATOMIC_RELAXED);
          idle = Patience{};
          continue;
        }
        if (idle.expired(2 * MIG_WAIT_TICKS)) break;   // never, short of a fault
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) __atomic_store_n(&help_req[1], -1, __ATOMIC_RELAXED);   // no producer 1 here
      return true;
    };
    auto bridge_out = [&]() {
      constexpr int VL = Ch::VLEN;
      AS_GLB double* const xs = pair_start();

      AS_LDS double* const av = L.vecs(2);        // the producer's area
      AS_LDS ChainScalars* const as = &L.cs(2);
      volatile AS_LDS int* depth = (volatile AS_LDS int*)&L.cs(0).depth;   // the producer's S0
      if (lane == 0) {
        bd[TW_CHAIN] = 0;
        *depth = 0;
      }
      int seen = 0, copied = 0;
      Patience idle;
      for (;;) {
        const int g = __builtin_amdgcn_readfirstlane(x_ldi(xh + PH_GEN));
        const int cw = __builtin_amdgcn_readfirstlane(x_ldi(xh + PH_CONS));
        const int dw = __builtin_amdgcn_readfirstlane(x_ldi(xh + PH_DEPTH));
        if (g != seen) {
          if (g < 0) break;
          if (!(g & BD_ENDED)) {   // a new transition: the start into the producer's area
#pragma unroll
            for (int s = 0; s < PPL; ++s) {
              const int k = s * WAVE + lane;
              av[V_E0_Q * VL + k] = x_ld(xs + k);
              av[V_E0_P * VL + k] = x_ld(xs + VL + k);
              av[V_E0_G * VL + k] = x_ld(xs + 2 * VL + k);
              av[V_MINV * VL + k] = x_ld(xs + 3 * VL + k);
            }
            if (lane == 0) {
              as->eps_used = x_ld(xs + 4 * VL);
              as->H0 = x_ld(xs + 4 * VL + 1);
              as->t = x_ldi(xh + PH_T);
              bd[TW_LC] = x_ldi(xh + PH_LC);
              bd[BD_CONS + 1] = 0;
              *depth = 0;
            }
          }
          wave_publish();   // the start lands before the transition's number
          if (lane == 0) __atomic_store_n(&bd[BD_GEN], g, __ATOMIC_RELAXED);
          seen = g;
          copied = 0;
          idle = Patience{};
          continue;
        }
        if (lane == 0) {   // the booking's progress: never lowered within the transition
          if ((cw >> 16) == seen && (cw & 0xFFFF) > bd[BD_CONS + 1]) bd[BD_CONS + 1] = cw & 0xFFFF;
          if ((dw >> 16) == seen && (dw & 0xFFFF) > *depth) *depth = dw & 0xFFFF;
        }
        const int pw = lds_load(&bd[BD_PROD + 1]);
        if ((pw >> 16) == seen && (pw & 0xFFFF) > copied) {
          const int cnt = pw & 0xFFFF;
          wave_fence();   // the records after their count
          for (int n = copied; n < cnt; ++n) {   // records n: end 1's slot -> the pair's slot
            const AS_LDS double* sv = fwd_vec(n & 1);
            const AS_LDS double* ss = fwd_sc(n & 1);
            AS_GLB double* dst = pair_rec(n & 1);
            for (int i = lane; i < QXD; i += WAVE) x_st(dst + i, i < RVD ? sv[i] : ss[i - RVD]);
          }
          x_drain();   // the records have reached memory before their count
          copied = cnt;
          if (lane == 0) x_sti(xh + PH_COUNT, (seen << 16) | copied);
          idle = Patience{};
          continue;
        }
        if (idle.expired(2 * MIG_WAIT_TICKS)) break;   // never, short of a fault
        __builtin_amdgcn_s_sleep(1);
      }
      // the chain has finished: stop the producer, let it drain its sweep, end the tile
      if (lane == 0) __atomic_store_n(&bd[BD_GEN], -1, __ATOMIC_RELAXED);
      {
        Patience w;
        while (lds_load(&bd[BD_EXIT]) < 1 && !w.expired(LEAF_WAIT_TICKS)) __builtin_amdgcn_s_sleep(1);
      }
      wave_fence();
      if (lane == 0) atomicSub(&n_active, 1);
    };
    if constexpr (PAIR) {
      if (role == 1 && pair_on && c == 2) bridge_out();   // partner tile: the bridge
    }
    if constexpr (SPEC && !MIG) {
      if (bidi && c == 1 && (role == 0 || pair_on)) {
        // the booking helper of producer 0 (a primary; in a paired launch also its producer 1
        // if the pair did not form) or 1 (a partner).  An unpaired launch's producer 1 books
        // its leaves itself (a helper serving both ends would pace both).
        constexpr bool both = PAIR;
        // below the producers and the sweep's NUTS neighbours: it has slack (4.1 k of a
        // producer's 5.8 k cycles per leaf, profiling build), and the gradient wave sharing its
        // SIMD is on a sweep's critical path (config 2: priority 2 / 1 +0.5 % over 3,
        // profiles/r06_ab_prio.txt)
        __builtin_amdgcn_s_setprio(2);
        Patience w;
        long long pf_busy = 0, pf_n = 0;   // profiling build: cycles booking, leaves booked
        for (int s = role;; s = (both && role == 0) ? s ^ 1 : s) {   // (one call site of serve)
          const long long pt = kProfile ? (long long)__builtin_amdgcn_s_memtime() : 0;
          const int a = serve(s, false);
          if (a > 0) {
            if (kProfile) {
              pf_busy += (long long)__builtin_amdgcn_s_memtime() - pt;
              ++pf_n;
            }
            w = Patience{};
            continue;
          }
          const bool alt = both && role == 0;
          if (a < 0 && (!alt || lds_load(&help_req[s ^ 1]) < 0)) break;   // producers gone
          if (!alt || s == 1) {
            if (w.expired(MIG_WAIT_TICKS)) break;   // never, short of a fault
            __builtin_amdgcn_s_sleep(1);
          }
        }
        if (kProfile && P.stamps != nullptr && lane == 0) {   // this tile's booking helper
          AS_GLB long long* o = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP + 96 + 2 * role;
          o[0] = pf_busy;
          o[1] = pf_n;
        }
      }
    }
    // two-ended trajectories: producer of the backward (c = 2) / forward end (c = 3); paired
    // tiles: the forward end grows in the partner tile (its NUTS wave 3) and the primary's
    // wave 3 is the bridge.  (One call site: produce is inlined once.)
    if (bidi && c >= 2 && (role == 0 || (pair_on && c == 3))) {
      bool here = true;
      if constexpr (PAIR) {
        if (role == 0 && c == 3) here = !bridge_in();
      }
      if (here) produce(c - 2, c - 1, 0);
      wave_fence();
      if (lane == 0) atomicAdd(&bd[BD_EXIT], 1);
    }
    if (helped && !bidi && c >= P.G && c - P.G < nct) {   // the helper wave of chain slot c - G
      using Ch = Chain<PPL, NNP, FAM, MIG, SPEC, CMODE>;
      const int hs = c - P.G;
      Ch ch(P, L, hs, c0 + hs, lane, nct);
      int seen = 0;
      Patience w;
      for (;;) {
        const int r = lds_load(&help_req[hs]);
        if (r < 0) break;                       // the chain has finished
        if (r == seen) {
          // the chain releases its helper when it finishes (help_req = -1), however long
          // its gaps between speculated leaves (init, step-size searches): the hang guard
          // is in real time, not polls, as for migration receivers
          if (w.expired(MIG_WAIT_TICKS)) break;
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        w = Patience{};
        seen = r;
        wave_fence();   // the request's arguments are read after its number
        // book the handed-over leaf; publish its outcome, then the number
        const int res = ch.deep_book();
        wave_publish();
        if (lane == 0) {
          __atomic_store_n(&help_res[hs], res, __ATOMIC_RELAXED);
          wave_publish();
          __atomic_store_n(&help_done[hs], seen, __ATOMIC_RELAXED);
        }
      }
    }
    if (role == 0 && c < (mig ? P.G : nct)) {
      using Ch = Chain<PPL, NNP, FAM, MIG, SPEC, CMODE>;
      long long epoch = 0;     // this slot's hand-offs (grad_cnt[c] counts NGW per epoch)
      int lc = c < nct ? c0 + c : -1;
      int a = Ch::A_INIT_STATE;
      for (;;) {   // the slot's own chain, then (migration) chains handed over by other tiles
       if (lc >= 0) {
        Ch ch(P, L, c, lc, lane, nct);
        ch.live = (const AS_LDS int*)&live_chains;
        ch.bd = (volatile AS_LDS int*)bd;
        long long steps = 0;
        bool in_sweep = false;   // the last run() was A_PRIOR, overlapping the chain's sweep
        // ONE call site of the action machine (it is inlined once, not per caller)
        int hreq = 0;            // helper requests posted (speculative path)
        for (;;) {
          FITOCT_MARK(nuts_loop);
        const long long s0 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
        const int y = ch.run(a);
        if (Ch::kTwoEnded && y == Ch::A_BIDI_TREE) {   // the producers grow the subtrees
          const int g = lds_load(&bd[BD_GEN]);
          const bool late = false;
          // this wave books the trajectory level; in an unpaired tile it books the forward end's
          // leaves too while it waits for records
          ch.bidi_book_tree(g, [&]() -> bool {
            if constexpr (!PAIR && !MIG && MODE == MODE_ROWS) return serve(1, true) > 0;
            return false;
          });
          wave_publish();   // the producers stop growing this tree
          if (lane == 0) {
            __atomic_store_n(&bd[BD_GEN], g | BD_ENDED, __ATOMIC_RELAXED);
            __atomic_store_n(&bd[TW_BUSY], 0, __ATOMIC_RELAXED);   // (migrating tiles) another chain may claim them
          }
          wave_fence();   // the helper's bookkeeping is read after the end
          // the helper's booked leaves count toward the step bound like the chain's own
          steps += ch.uni(ch.Sp->n_leapfrog);
          if (late || ch.uni(ch.Sp->status) == ERR_TIMEOUT || steps > P.max_steps) {
            ch.Sp->status = ERR_TIMEOUT;
            a = Ch::A_FINISH;
          } else {
            a = Ch::A_END_TREE;
          }
          continue;
        }
        if (spec && y == Ch::A_SPEC_STAGED) {   // enqueue the speculated position, hand its prior part over
          if (++steps > P.max_steps) {
            ch.Sp->status = ERR_TIMEOUT;
            a = Ch::A_FINISH;
            continue;
          }
          if (lane == 0) {
            post_sweep(c);
            if (ch.deep) {
              wave_publish();   // the hand-off (HX) lands before the request number
              __atomic_store_n(&help_req[c], hreq + 1, __ATOMIC_RELAXED);
            }
          }
          if (stamp) t_enq = (long long)__builtin_amdgcn_s_memtime();
          if (ch.deep) {   // the helper books the leaf; this wave computes the next prior part
            ++hreq;
            ch.book_done = (volatile AS_LDS int*)&help_done[c];
            ch.book_res = (volatile AS_LDS int*)&help_res[c];
            ch.book_want = hreq;
            ++epoch;
            a = Ch::A_PRIOR;
            in_sweep = true;
            continue;
          }
          ++epoch;   // (no helper wave: this wave books the leaf during the sweep)
          a = Ch::A_SPEC_BOOK;
          continue;
        }
        if (spec && (y == Ch::A_SPEC_WAIT || y == Ch::A_SPEC_DISCARD)) {
          bool late = false;
          Patience w;
          const long long w0 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
          if (stamp) t_busy += w0 - s0;
          while (lds_load(&grad_cnt[c]) < (int)(NGW * epoch)) {
            if (w.expired(LEAF_WAIT_TICKS)) {
              late = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          wave_fence();   // nothing of the next action is read before the sweep and the helper are done
          if (stamp) {
            const long long t1 = (long long)__builtin_amdgcn_s_memtime();
            t_wait += t1 - w0;
            t_sweep += done_t[c] - t_enq;
            t_st0 += start_min[c] - t_enq;
            t_st1 += start_max[c] - t_enq;
            start_min[c] = 0x7FFFFFFFFFFFFFFFLL;
            start_max[c] = 0;
            t_notice += t1 - (done_t[c] > w0 ? done_t[c] : w0);
            ++n_items;
          }
          if (late) {
            ch.Sp->status = ERR_TIMEOUT;
            a = Ch::A_FINISH;
          } else {
            a = (y == Ch::A_SPEC_WAIT) ? Ch::A_GRAD : Ch::A_END_TREE;
          }
          continue;
        }
        if (in_sweep) {
          in_sweep = false;
          bool late = false;
          Patience w;
          const long long w0 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
          // A NUTS wave waits at priority 3 on a SIMD it shares with a gradient wave.  When
          // the sweep is long (8+ bins per lane, or streamed bins) and the tile hosts
          // several chains, the wait is long and the sampler is not the bottleneck: poll
          // rarely, so the waiting wave leaves the SIMD's issue to the gradient wave.
          if (P.G >= 2 && (BPT >= 8 || BPT == 0)) {
            __builtin_amdgcn_s_setprio(0);
            while (lds_load(&grad_cnt[c]) < (int)(NGW * epoch)) {
              if (w.expired(LEAF_WAIT_TICKS)) {
                late = true;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_s_setprio(3);
          } else {
            while (lds_load(&grad_cnt[c]) < (int)(NGW * epoch)) {
              if (w.expired(LEAF_WAIT_TICKS)) {
                late = true;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
          }
          if (stamp) {
            const long long t1 = (long long)__builtin_amdgcn_s_memtime();
            t_wait += t1 - w0;
            t_sweep += done_t[c] - t_enq;            // enqueue -> 8th gradient wave done
            t_st0 += start_min[c] - t_enq;           // enqueue -> first wave starts
            t_st1 += start_max[c] - t_enq;           // enqueue -> last wave starts
            start_min[c] = 0x7FFFFFFFFFFFFFFFLL;
            start_max[c] = 0;
            t_notice += t1 - (done_t[c] > w0 ? done_t[c] : w0);
          }
          if (late) {
            ch.Sp->status = ERR_TIMEOUT;
            a = Ch::A_FINISH;
          } else {
            a = Ch::A_GRAD;
          }
          continue;
        }
        if (stamp) {
          t_busy += (long long)__builtin_amdgcn_s_memtime() - s0;
          ++n_items;
        }
        const int stt = __builtin_amdgcn_readfirstlane(ch.Sp->state);
        if (stt == ST_DONE || stt == ST_MOVED) {
          if (kProfile && lane == 0 && stt == ST_DONE) {
            atomicCAS((unsigned long long*)&first_done_rt, 0ULL,
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
            atomicAdd(&chains_done_here, 1);
          }
          if (helped && lane == 0) __atomic_store_n(&help_req[c], -1, __ATOMIC_RELAXED);   // release the helper
          if (bidi) {   // release the producers; they drain their sweeps
            if (kProfile && P.stamps != nullptr && lane == 0) {   // the booking's time
              AS_GLB long long* o = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP;
              o[84] = ch.pf_busy;
              o[85] = ch.pf_wait;
              o[86] = ch.pf_n;
            }
            if (lane == 0) __atomic_store_n(&bd[BD_GEN], -1, __ATOMIC_RELAXED);
            Patience w;
            while (lds_load(&bd[BD_EXIT]) < 2 && !w.expired(LEAF_WAIT_TICKS)) __builtin_amdgcn_s_sleep(1);
          }
          if (spec && lane == 0) atomicSub(&live_chains, 1);
          break;
        }
        if (++steps > P.max_steps) {   // termination guarantee: report, never hang
          ch.Sp->status = ERR_TIMEOUT;
          a = Ch::A_FINISH;
          continue;
        }
        if constexpr (kProfile) {
          if (P.bench_sweeps > 0 && P.stamps != nullptr) {   // sweep-only measurement
            for (int r = 0; r < P.bench_sweeps; ++r) {
              if (lane == 0) post_sweep(c);
              ++epoch;
              while (lds_load(&grad_cnt[c]) < (int)(NGW * epoch)) __builtin_amdgcn_s_sleep(1);
            }
            ch.Sp->state = ST_DONE;
            break;
          }
        }
        // enqueue chain c: sequence number from a ring-wide counter, one 64-bit store
        if (lane == 0) post_sweep(c);
        if (stamp) t_enq = (long long)__builtin_amdgcn_s_memtime();
        ++epoch;
        // position-only work (prior terms, next merges' uniforms) overlaps the sweep
        a = Ch::A_PRIOR;
        in_sweep = true;
        }
        if (mig && lane == 0 && __builtin_amdgcn_readfirstlane(ch.Sp->state) == ST_DONE) {
          const MigView M(P.mig, P.mig_tiles);
          g_add(&M.load[blockIdx.x], -1);
          __hip_atomic_fetch_add((int*)&M.hdr[MIG_DONE], 1, __ATOMIC_RELAXED,   // a count: no data
                                 __HIP_MEMORY_SCOPE_AGENT);
        }
       }
        if (!mig) break;
        lc = receive_chain<PPL>(P, L, c, lane, (volatile AS_LDS int*)bd, (const AS_LDS int*)&live_chains);
        if constexpr (Ch::kTwoEnded) {
          if (lc <= -2) {   // recruited as a producer of the tile's lone chain (the tail)
            produce(-2 - lc, c, epoch);
            break;
          }
        }
        if (lc < 0) break;
        if (spec && lane == 0) atomicAdd(&live_chains, 1);
        a = Ch::A_START_TRANSITION;
      }
      wave_fence();
      if (lane == 0) atomicSub(&n_active, 1);
    }
  }
  if (wstamp) ((AS_GLB long long*)P.stamps)[(size_t)tix * NSTAMP + 56 + wave] = t_wbusy;
  if (stamp) {
    AS_GLB long long* o = (AS_GLB long long*)P.stamps + (size_t)tix * NSTAMP;
    if (wave == 0) {
      o[0] = n_items;
      o[1] = t_busy;
      o[3] = (long long)__builtin_amdgcn_s_memtime() - t_begin;
      o[64] = rt_begin;
      o[65] = (long long)__builtin_amdgcn_s_memrealtime();
      o[66] = first_done_rt;
      o[67] = chains_done_here;
    } else {
      o[2] = t_busy;
      o[40] = t_wait;
      o[42] = t_sweep;
      o[43] = t_notice;
      o[44] = t_st0;
      o[45] = t_st1;
      o[41] = n_items;
      for (int k = 0; k < 18; ++k) {
        o[4 + k] = L.cs(0).prof[0][k];
        o[22 + k] = L.cs(0).prof[1][k];
      }
      for (int k = 0; k < 8; ++k) o[48 + k] = L.cs(0).prof[0][20 + k];
      for (int k = 0; k < 4; ++k) o[68 + k] = L.cs(0).prof[0][28 + k];
    }
  }
}

template <class R, int BPT, int NNP, int PPL, int MODE, int FAM>
__global__ void __launch_bounds__(TPB, 2) logp_kernel(const KParams* __restrict__ Pg) {
  KPc& P = *(KPc*)Pg;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds<PPL> L{(AS_LDS char*)smem, P.G, Lds<PPL>::chain_bytes(P.max_depth)};
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.x * P.G;
  const int nct = min(P.G, P.chains - c0);
  __shared__ int done[GMAX];
  load_kinv<PPL, NNP>(P, L, tid);
  if (tid < GMAX) done[tid] = tid >= nct;
  __syncthreads();
  const int c = wave - NGW;
  if (wave >= NGW && c < nct) {
    Chain<PPL, NNP, FAM> ch(P, L, c, c0 + c, lane, nct);
    Vd<PPL> q;
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = s * WAVE + lane;
      q.a[s] = (k < P.D) ? ((const AS_GLB double*)P.q_in)[(size_t)(c0 + c) * P.D + k] : 0.0;
    }
    if (lane < NSLOT) ch.SUMS[lane] = 0.0;
    ch.write_mp(q);
    wave_fence();
  }
  __syncthreads();
  if (wave < NGW && P.prior_PD == 0) {
    Bins<R, BPT, NNP, MODE> bins;
    bins.load(P, tid);
    gradient_pass<R, BPT, NNP, MODE, true>(P, bins, L.mp(0), L.part(), done, 0, nct, tid, lane,
                                           wave);
  }
  __syncthreads();
  if (wave >= NGW && c < nct) {
    Chain<PPL, NNP, FAM> ch(P, L, c, c0 + c, lane, nct);
    ch.prior_part();
    wave_fence();
    Vd<PPL> g;
    double s0;
    const double lp = ch.finish_grad(g, s0);
    const size_t pt = (size_t)(c0 + c);
#pragma unroll
    for (int s = 0; s < PPL; ++s) {
      const int k = s * WAVE + lane;
      if (k < P.D) ((AS_GLB double*)P.grad_out)[pt * P.D + k] = g.a[s];
    }
    if (lane == 0) {
      ((AS_GLB double*)P.lp_out)[pt] = lp;
      if (P.s2_out) ((AS_GLB double*)P.s2_out)[pt] = s0;
    }
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch over the template grid.  This file is compiled once per
// prior family (-DFITOCT_FAMILY=0/1/2, in parallel); the family is a template
// parameter of the sampler so that no family branch survives in its code.
// ---------------------------------------------------------------------------
#ifndef FITOCT_FAMILY
#error "compile with -DFITOCT_FAMILY=0|1|2"
#endif
#define FITOCT_CAT2(a, b) a##b
#define FITOCT_CAT(a, b) FITOCT_CAT2(a, b)

#if FITOCT_FAMILY == 0
int lds_bytes(int ppl, int G, int max_depth) {
  return ppl == 1 ? Lds<1>::bytes(G, max_depth) : Lds<2>::bytes(G, max_depth);
}
// doubles in a chain's migration image: its LDS region up to the tree levels
int mig_img_words(int ppl) {
  return ppl == 1 ? Lds<1>::chain_bytes(0) / 8 : Lds<2>::chain_bytes(0) / 8;
}
#endif

template <class R, int BPT, int NNP, int PPL, int MODE>
static hipError_t launch_t(bool logp, const KParams& P, const KParams* dP, int tiles,
                           hipStream_t st, const int* tile_map) {
  constexpr int F = FITOCT_FAMILY;
  // two-ended trajectories: 3 chain areas (the chain's and its two producers')
  const int lds = (!logp && P.bidi) ? Lds<PPL>::bytes(3, P.max_depth) : Lds<PPL>::bytes(P.G, P.max_depth);
  if (logp) {
    auto k = logp_kernel<R, BPT, NNP, PPL, MODE, F>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(tiles), dim3(TPB), lds, st, dP);
  } else {
    // three samplers: with migration, with speculative leaves (one chain per tile), plain
    // four samplers: with / without migration, with / without speculative leaves
    auto k = P.mig != nullptr
                 ? (P.spec ? nuts_kernel<R, BPT, NNP, PPL, MODE, F, true, true, false>
                           : nuts_kernel<R, BPT, NNP, PPL, MODE, F, true, false, false>)
             : P.spec ? (P.pair ? nuts_kernel<R, BPT, NNP, PPL, MODE, F, false, true, true>
                                : nuts_kernel<R, BPT, NNP, PPL, MODE, F, false, true, false>)
                      : nuts_kernel<R, BPT, NNP, PPL, MODE, F, false, false, false>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(tiles), dim3(TPB), lds, st, dP, tile_map);
  }
  return hipGetLastError();
}

template <class R, int NNP, int PPL, int MODE>
static hipError_t launch_m(bool logp, int bpt, const KParams& P, const KParams* dP, int tiles,
                           hipStream_t st, const int* tm) {
  switch (bpt) {
    case 0: return launch_t<R, 0, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
    case 1: return launch_t<R, 1, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
    case 2: return launch_t<R, 2, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
    case 4: return launch_t<R, 4, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
    case 8:
      if constexpr (MODE == MODE_POLY) return launch_t<R, 8, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
      return hipErrorInvalidValue;
    case 16:   // compact geo layout, f64 only (N in (2048, 4096] on an arithmetic grid)
      if constexpr (MODE == MODE_POLY && sizeof(R) == 8)
        return launch_t<R, 16, NNP, PPL, MODE>(logp, P, dP, tiles, st, tm);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int NNP, int PPL>
static hipError_t launch_n(bool logp, bool mixed, int bpt, const KParams& P, const KParams* dP,
                           int tiles, hipStream_t st, const int* tm) {
  if (!mixed) {
    if (P.mode == MODE_POLY)
      return launch_m<double, NNP, PPL, MODE_POLY>(logp, bpt, P, dP, tiles, st, tm);
    if constexpr (NNP == 15 && PPL == 1) {   // N <= 512: the rows in registers
      if (bpt == 1) return launch_t<double, 1, NNP, PPL, MODE_ROWS>(logp, P, dP, tiles, st, tm);
      if (bpt == 2) return launch_t<double, 2, NNP, PPL, MODE_ROWS>(logp, P, dP, tiles, st, tm);
    }
    if (bpt != 0) return hipErrorInvalidValue;
    return launch_t<double, 0, NNP, PPL, MODE_ROWS>(logp, P, dP, tiles, st, tm);
  }
  return launch_m<float, NNP, PPL, MODE_ROWS>(logp, bpt, P, dP, tiles, st, tm);
}

// P: host copy (shapes); dP: the same block already copied to device memory
hipError_t FITOCT_CAT(launch_family_, FITOCT_FAMILY)(bool logp, bool mixed, int bpt, int nnp,
                                                     const KParams& P, const KParams* dP,
                                                     int tiles, hipStream_t st,
                                                     const int* tile_map) {
  if (nnp == 15) return launch_n<15, 1>(logp, mixed, bpt, P, dP, tiles, st, tile_map);
  return launch_n<24, 2>(logp, mixed, bpt, P, dP, tiles, st, tile_map);
}

}  // namespace fitoct
