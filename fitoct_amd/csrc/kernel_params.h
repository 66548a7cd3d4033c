// Launch parameters shared by the host planner (fitoct_api.cpp) and the device
// sampler (nuts_device.hip).  Plain data, passed by value as a kernel argument.
#pragma once
#include <stdint.h>

namespace fitoct {

constexpr int WAVE = 64;          // CDNA wavefront
// A tile is 8 waves = 2 per SIMD (waves w and w+4 share SIMD w mod 4): one
// gradient wave and one NUTS wave on every SIMD, 256 VGPRs each.  The sweep is
// VALU-issue bound; one gradient wave per SIMD (rather than two) halves the
// per-sweep cross-lane reduction work and the partial sums the NUTS wave adds.
constexpr int NW = 8;             // waves per tile (workgroup)
constexpr int TPB = NW * WAVE;    // 512 threads per tile
constexpr int NGW = 4;            // gradient waves (waves 0..3): the likelihood sweep
constexpr int GT = NGW * WAVE;    // 256 gradient lanes; bins are strided over them
constexpr int GMAX = NW - NGW;    // NUTS waves (4..7), one chain each: max chains per tile
constexpr int MAXDEPTH = 16;      // hard cap on max_treedepth
constexpr int NSLOT = 32;         // reduced sums per chain (4 + NNP <= 32)
constexpr int MPW = 32;           // model-parameter words per chain (theta[3], pad, yGP[NNP])
constexpr int POOL_VECS = 2;      // vectors per proposal-pool slot in HBM (q, grad)
constexpr int KMAX = 24;          // max GP control points (K^-1 tile in LDS)
constexpr int NSTAMP = 108;        // diagnostic stamps per tile (FITOCT_STAMPS)
constexpr int PAIR_HDR_INTS = 64; // paired tiles: hand-off words per pair (nuts_device.hip PairHdr)
constexpr int PAIR_START_DOUBLES = 8;   // ... and per pair in pair_buf: the start's 4 vectors, then
                                        // these scalars, then the ring
// the kernel's static LDS (rings, hand-off words, counters: 352 B measured, the
// -Rpass-analysis "LDS Size" of every sampler instantiation), reserved in every LDS plan
constexpr int STATIC_LDS_RESERVE = 1024;
// paired tiles: blocks launched for `tiles` tiles (groups of 8 primaries + 8 partners)
inline int pair_grid(int tiles) { return 16 * ((tiles + 7) / 8); }

// how a tile evaluates the GP modulation dL = B yGP and its adjoint B^T h.
// With BPT > 0 a lane's bins stay in VGPRs for the whole run, with BPT == 0 the
// bins are streamed from global memory (L2-resident) on every pass.
enum BasisMode : int {
  MODE_POLY = 0,    // factorised SE basis: per-bin (t, a), Horner + moments (f64 path)
  MODE_ROWS = 1,    // explicit basis rows B[i, 0..NNP) (user basis, fp32 path)
};

enum ChainState : int { ST_INIT = 0, ST_STEPSIZE = 1, ST_TREE = 2, ST_DONE = 3, ST_MOVED = 4 };

// Chain migration between tiles (work balance at the end of a run).  Layout of
// KParams::mig (int32, zeroed before every launch):
enum MigCtrl : int {
  MIG_WAITING = 0,   // NUTS slots posted as free (receivers)
  MIG_DONE = 1,      // chains finished (ST_DONE) over the whole launch
  MIG_STARTED = 2,   // tiles that have begun: receivers wait only once all have
  MIG_MOVES = 3,     // chains handed over (reported in fitoct_result::migrations)
  MIG_HDR = 4,       // then: load[tiles] | free_mask[tiles] | mailbox[tiles * GMAX]
};

struct KParams {
  // ---- data (device pointers, padded to n_pad bins) ----
  const void* cx;      // R[n_pad]  c * x_i
  const void* y;       // R[n_pad]
  const void* isu;     // R[n_pad]  1/uy_i (0 on padding)
  const void* B;       // BREG/STREAM: R[n_pad][NNP] basis rows; POLY: R[n_pad][2] (t, a)
  const double* Kinv;  // POLY: [Nn][Nn] (K(xGP,xGP) + nugget I)^-1
  const double* bvec;  // POLY: [Nn] b_l
  int N, n_pad, Nn, D, family, prior_PD, mode;
  // POLY on a uniform depth grid: bin tid + b*GT has t = t_tid * R^b, so a lane's
  // moments sum_b w_b t_b^l = t_tid^l * sum_b w_b (R^l)^b (Horner in R^l).
  int geo;                  // 1: geo_R valid (host-verified arithmetic x grid)
  double geo_R[24];         // R^l, l < 24 (moments: l < NNP; BPT 16 also t_b = t_tid R^b)
  // BPT == 16 (N in (2048, 4096] on an arithmetic grid): a lane keeps only y, 1/uy
  // and a of its 16 bins; c*x_b = cx_tid + geo_dcx[b] and t_b = min(t_tid R^b, geo_tmax)
  // (the clamp keeps padding bins, whose a is 0, finite)
  double geo_dcx[16];
  double geo_tmax;
  double theta0[3];
  double S0inv[9];
  double lambda_rate_eff;   // rate of the exponential prior on lambda (normal family)
  double lambda_scale;      // lasso lambda_s
  double nu;                // horseshoe nu
  double sigma_scale;
  double sigma_scale_inv;   // 1 / sigma_scale
  // ---- sampler ----
  int chains;               // chains in this launch
  int chain_offset;         // global id of chain 0
  int G;                    // chains per tile
  int warmup, samples, max_depth, save_warmup, adapt;
  uint64_t seed;
  double adapt_delta, gamma, kappa, t0, stepsize0, init_radius;
  int init_buffer, term_buffer, base_window;
  long long max_steps;      // per-tile step bound (termination guarantee)
  // warm restart (fitoct_plan_set_init; nullptr: defaults): per-chain initial step size,
  // diagonal inverse metric and unconstrained position, indexed by the launch's chain
  const double* init_eps;   // [chains]
  const double* init_minv;  // [chains][D]
  const double* init_q;     // [chains][D]
  // ---- outputs ----
  double* draws;            // [chains][iters_saved][ncols]
  int ncols, iters_saved;
  double* stack;            // proposal pool [chains][max_depth + 1][POOL_VECS][vlen]
  double* fin_eps;          // [chains]
  double* fin_minv;         // [chains][D]
  double* fin_q;            // [chains][D]
  int* chain_status;        // [chains]
  long long* leapfrogs;     // [chains]
  long long* stamps;        // optional [tiles][4]: half-steps, gradient busy, NUTS busy, total cycles
  int bench_sweeps;         // profiling build only (FITOCT_BENCH_SWEEPS): after the first
                            // position, each chain re-enqueues it this many times and stops
                            // (the sweep alone, no sampler work between sweeps)
  // ---- chain migration (nullptr / 0: off) ----
  int* mig;                 // MigCtrl header | load | free_mask | mailbox (see MigCtrl)
  double* mig_img;          // [tiles * GMAX][mig_img_words] chain images in flight
  int mig_tiles, mig_img_words;
  int spec;                 // 1: the speculative-leaf sampler (nuts_device.hip leaf_spec)
  int spec_live;            // ... a chain speculates while its tile hosts <= spec_live live
                            // chains (tiles of one chain: always, with a helper wave)
  // ---- run-time progress / cancellation (host-pinned; nullptr: off) ----
  int* progress;            // [chains] transitions completed (written at each boundary)
  const int* cancel;        // != 0: every chain stops at its next checked boundary
  // ---- logp mode ----
  const double* q_in;       // [points][D]
  double* lp_out;           // [points]
  double* grad_out;         // [points][D]
  double* s2_out;           // [points]
  // appended (ABI 5), so the offsets of every field above are those of round 3
  double theta_rate;        // mono-exp, theta_prior = 1: theta_k ~ exponential(theta_rate)
  // ---- two-ended trajectories (tiles of one chain; 0: off) ----
  // two producer waves build the subtrees of the trajectory's backward and forward ends from
  // the transition's start at once, each in its own chain area; the chain's wave books the
  // trajectory level from one record per subtree (nuts_device.hip, "two-ended trajectories")
  int bidi;                 // 1: on (the tile's LDS then carves 3 chain areas)
  // ---- two-ended trajectories in a migrating launch's tail (0: off) ----
  // once at most tail_left chains of the launch are unfinished, a chain alone in its tile
  // recruits two of the tile's idle receivers as producers (their own chain areas)
  int tail_bidi;
  int tail_left;
  // a tail producer idle this long (s_memrealtime ticks, 100 MHz) withdraws its role; 0:
  // MIG_WAIT_TICKS (test hook FITOCT_TEST_TAIL_IDLE_US)
  unsigned long long tail_idle_ticks;
  unsigned long long* bidi_count;   // two-ended transitions of the launch (fitoct_result)
  // ---- paired tiles (one-chain tiles with two-ended trajectories, 2 x tiles <= CUs; 0: off) ----
  // the forward end of each tile's trajectories grows in a partner tile with its own gradient
  // waves (nuts_device.hip "paired tiles"); the grid is 16 * ceil(pair_tiles / 8) blocks
  int pair;
  int pair_tiles;           // tiles of the launch (the tile map's entries)
  int pair_stride;          // doubles per pair in pair_buf: start (4 vectors + 8) | 2 records (5 + 16)
  int pair_test_absent;     // test hook (FITOCT_TEST_PAIR_ABSENT): partners leave at once
  int* pair_hdr;            // [pair_tiles][PAIR_HDR_INTS] hand-off words, zeroed per launch
  double* pair_buf;         // [pair_tiles][pair_stride]
  unsigned long long* pair_count;   // transitions grown by a pair (fitoct_result)
};

}  // namespace fitoct
