/*
 * fitoct.h -- C ABI of libfitoct.so, the MI355X-native NUTS sampler for FitOCT's
 * modulated-exponential (ExpGP) posterior.
 *
 * This is the drop-in boundary of SURVEY.md §8b.  In the reference, the hot path
 * is reached from R through FitOCTLib::fitExpGP (external package; called at
 * FitOCT.R:110-124, priPost.R:2-16, ShinyInterface/server.R:408-426), which hands
 * a Stan data list to rstan::sampling (chains fanned out over R worker processes,
 * FitOCT.R:13).  libfitoct replaces rstan::sampling + the Stan C++ model/NUTS with:
 *
 *   fitoct_expgp_sample()   <- FitOCTLib::fitExpGP(method='sample') -> rstan::sampling
 *                              (FitOCT.R:110-124 / priPost.R:2-16 / server.R:408-426)
 *   fitoct_logp_grad()      <- Stan model log_prob + stan-math gradient
 *                              (the ExpGP model whose parameters are named at plotExpGP.R:9,41)
 *   fitoct_build_basis()    <- the GP design of server.R:623-650 (xGP grid, SE kernel)
 *   fitoct_split_rhat_ess() <- rstan::summary(...)$summary[, c('n_eff','Rhat')]
 *                              (server.R:88-104,189-213)
 *   fitoct_plan_*()         <- same as fitoct_expgp_sample, split so that inputs can stay
 *                              resident in HBM across calls and draws can land in a
 *                              caller-owned device buffer (multi-GPU gather / benchmarking)
 *
 * Conventions: plain C types only; every host buffer is owned by the caller; the
 * library never keeps a caller pointer after returning; device memory it allocates
 * is released on return or by fitoct_plan_destroy().  Functions return
 * FITOCT_OK (0) or a negative fitoct_status; fitoct_last_error() then describes
 * the failure (thread-local string).  No C++ exception crosses this boundary.
 */
#ifndef FITOCT_H
#define FITOCT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FITOCT_ABI_VERSION 8
/* largest accepted N (depth bins): bounds every host and device allocation derived from it */
#define FITOCT_MAX_BINS (1 << 22)
/* largest device list of one call (fitoct_config.devices) */
#define FITOCT_MAX_DEVICES 16

typedef enum fitoct_status {
  FITOCT_OK = 0,
  FITOCT_E_ARG = -1,       /* invalid argument / unsupported shape */
  FITOCT_E_HIP = -2,       /* HIP runtime error */
  FITOCT_E_NODEVICE = -3,  /* no HIP device visible */
  FITOCT_E_INIT = -4,      /* no finite initial point after 100 attempts */
  FITOCT_E_NUMERIC = -5,   /* step size search diverged (eps > 1e7 or eps == 0) */
  FITOCT_E_TIMEOUT = -6,   /* device step bound reached before all chains finished */
  FITOCT_E_INTERNAL = -7,
  FITOCT_E_CANCELLED = -8  /* fitoct_plan_cancel: chains stopped at a transition boundary */
} fitoct_status;

/* yGP hyper-prior families */
enum { FITOCT_PRIOR_NORMAL = 0, FITOCT_PRIOR_LASSO = 1, FITOCT_PRIOR_HORSESHOE = 2 };
/* prior_type value selecting the mono-exponential model of FitOCTLib::fitMonoExp
 * (FitOCT.R:95, server.R:341): y = theta1 + theta2 exp(-c x / theta3), no GP term,
 * flat prior on theta > 0, sigma fixed at 1 (uy is the noise sd; ⚑ SURVEY §8f row 2).
 * D = 3; Nn, rho, B, Sigma0 and the hyper-parameters are ignored; theta0 is only
 * the initialisation centre. */
enum { FITOCT_MODEL_MONOEXP = 3 };
/* GP control grid (server.R:627-631) */
enum { FITOCT_GRID_INTERNAL = 0, FITOCT_GRID_EXTREMAL = 1 };
/* arithmetic of the per-bin likelihood sweep; reductions and sampler state are f64 always */
enum { FITOCT_PREC_F64 = 0, FITOCT_PREC_MIXED = 1 };

/* Inputs of FitOCTLib::fitExpGP (same meaning, FitOCT.R:110-124) plus the ⚑ model switches. */
typedef struct fitoct_problem {
  int32_t N;             /* depth bins */
  const double* x;       /* [N] depth (um), strictly increasing not required, max > min */
  const double* y;       /* [N] intensity / amplitude */
  const double* uy;      /* [N] data uncertainty (> 0) */
  int32_t data_type;     /* c in exp(-c*x/theta3): 1 amplitude, 2 intensity (FitOCT.R:39) */
  int32_t Nn;            /* GP control points, 2..24 (ui.R:200-207 allows 5..20) */
  int32_t grid_type;     /* FITOCT_GRID_* */
  double rho;            /* GP length scale on normalised depth; <= 0 -> 1/Nn (FitOCT.R:119) */
  const double* B;       /* optional [N*Nn] row-major basis; NULL -> fitoct_build_basis */
  double theta0[3];      /* prior mean of theta (estimateExpPrior, FitOCT.R:103-107) */
  double Sigma0[9];      /* prior covariance of theta, row-major */
  int32_t prior_type;    /* FITOCT_PRIOR_* */
  double lambda_rate;    /* normal family: lambda ~ Exponential (see lambda_conv) (FitOCT.R:47) */
  double lambda_scale;   /* lasso family: lambda_s of lassoPrior.stan:4 */
  double nu;             /* horseshoe family: nu of horseShoePrior.stan:13 (1 = horseshoe) */
  int32_t prior_PD;      /* 1: likelihood off (prior predictive, priPost.R:14) */
  int32_t kernel_conv;   /* ⚑ 0: exp(-d^2/(2 rho^2)) (Stan), 1: exp(-(d/rho)^2) (RMgauss) */
  int32_t lambda_conv;   /* ⚑ 0: rate = 1/lambda_rate, 1: rate = lambda_rate */
  double sigma_scale;    /* ⚑ sigma ~ half-normal(0, sigma_scale) */
  double nugget;         /* diagonal jitter of K(xGP,xGP) (1e-9) */
  /* theta prior of the mono-exponential model (ABI 5).  0: the model's own (flat on
   * theta > 0).  1: theta_k ~ exponential(1 / lambda_scale) i.i.d. -- Tests/testGamma.R's
   * model `lambda ~ exponential(1./lambda_scale)` (lambda_scale = 10) on each of the three
   * coordinates, a proper prior, so prior_PD = 1 samples it alone: the reference's own
   * known answer for the sampler (mean = sd = lambda_scale; tests/test_gpu_kat.py).
   * Only with prior_type = FITOCT_MODEL_MONOEXP. */
  int32_t theta_prior;
} fitoct_problem;

/* rstan::sampling controls (testGamma.R:42-47) + sharding / device selection. */
typedef struct fitoct_config {
  int32_t chains;        /* chains run by THIS call */
  int32_t chain_offset;  /* global id of the first chain: RNG stream = (seed, chain id) */
  int32_t warmup;        /* nb_warmup */
  int32_t samples;       /* nb_iter - nb_warmup */
  uint64_t seed;
  double adapt_delta;    /* 0.8 */
  int32_t max_treedepth; /* 10 (1..16) */
  int32_t adapt_engaged; /* 1 */
  double stepsize;       /* initial step size (1) */
  double gamma, kappa, t0;                     /* dual averaging: 0.05, 0.75, 10 */
  int32_t init_buffer, term_buffer, window;    /* 75, 50, 25 */
  double init_radius;    /* jitter around the default init (0 -> deterministic) */
  int32_t save_warmup;   /* 1: warmup draws are stored too (traceplot(inc_warmup=TRUE)) */
  int32_t precision;     /* FITOCT_PREC_* */
  int32_t device;        /* HIP device ordinal (used when n_devices == 0) */
  /* Device list (SURVEY.md §8b "device list"; R fitExpGP(n_gpus = k) passes 0..k-1).  This
   * replaces rstan's chain parallelism over host cores, options(mc.cores =
   * parallel::detectCores()) at FitOCT.R:13 / ShinyInterface/server.R:19.  With
   * n_devices >= 1 the call's chains are split into contiguous blocks of global chain ids,
   * block r = [chain_offset + off_r, chain_offset + off_r + count_r) with count_r =
   * chains / n + (r < chains % n) and off_r = r * (chains / n) + min(r, chains % n), run
   * on devices[r] by one host thread per device (a batch splits its problems the same
   * way).  Random streams are keyed by global chain id, so the draws are bit-identical
   * to a one-device run whatever the list.  Only the first min(n_devices, chains) entries
   * (problems, for a batch) are used; an ordinal may repeat (several plans on one GPU). */
  int32_t n_devices;     /* 0: `device` alone; 1..FITOCT_MAX_DEVICES */
  int32_t devices[FITOCT_MAX_DEVICES];
} fitoct_config;

/* Outputs; every pointer is caller-allocated (NULL = not wanted). */
typedef struct fitoct_result {
  double* draws;            /* [chains][iters_saved][n_cols], see fitoct_column_name */
  int64_t draws_capacity;   /* elements available at draws */
  double* stepsize;         /* [chains] adapted step size */
  double* inv_metric;       /* [chains][D] adapted diagonal inverse metric */
  double* last_q;           /* [chains][D] final unconstrained position (NaN, as stepsize
                               and inv_metric, for a chain whose status is FITOCT_E_TIMEOUT) */
  int32_t* chain_status;    /* [chains] 0 or a fitoct_status per chain */
  int32_t n_cols;           /* out */
  int32_t iters_saved;      /* out */
  int32_t dim;              /* out: D, unconstrained dimension */
  int32_t migrations;       /* out: chains handed between tiles (work balance; no effect on draws) */
  int64_t total_leapfrogs;  /* out: sum of n_leapfrog__ over every transition of every chain */
  double kernel_ms;         /* out: device time of the sampler kernel (HIP events) */
  double wall_ms;           /* out: host wall time of the call */
  int64_t two_ended_transitions; /* out (ABI 6): transitions whose trajectory grew both ends at
                               once (tiles of one chain; chains alone in a migrating launch's
                               tail); the draws do not depend on it */
  int64_t paired_transitions; /* out (ABI 7): of those, transitions whose forward end grew in a
                               partner tile (fitoct_plan_info::paired); no effect on draws */
} fitoct_result;

/* Static description of a planned run. */
typedef struct fitoct_plan_info {
  int32_t dim;             /* D */
  int32_t n_cols;          /* D + 8 */
  int32_t iters_saved;
  int32_t chains;
  int32_t tiles;           /* workgroups launched */
  int32_t chains_per_tile; /* G */
  int32_t bins_per_thread; /* 0 = streamed from global memory */
  int32_t threads_per_tile;
  int32_t lds_bytes;
  int32_t n_pad;           /* padded bin count */
  int64_t draws_bytes;     /* size of the draws buffer */
  int32_t sampler;         /* sampler variant launched: FITOCT_SAMPLER_* */
  int32_t n_devices;       /* devices the plan's chains (a batch's problems) run on */
  /* ABI 6: two-ended trajectories (tiles of one chain grow the trajectory's backward and
   * forward ends on two spare waves at once; same draws bit for bit).  two_ended = 1 when
   * the plan's one-chain tiles run them, 2 (ABI 7) when a migrating plan's chains do so once
   * alone in their tile (the launch's tail: two idle receivers of the tile become the
   * producers), 0 when off.  ABI 7: each end's producer builds its subtrees whole and hands
   * the booking one record per subtree: ring_records = 1 (records in flight per end) when on,
   * ring_records_in_levels = 0 (kept for layout); both 0 when off. */
  int32_t two_ended;
  int32_t ring_records;
  int32_t ring_records_in_levels;
  /* ABI 7: paired tiles.  1 when a plan of one-chain two-ended tiles that fit twice on the
   * chip (2 x tiles <= CUs, e.g. 128 chains on 256 CUs) launches a partner tile per tile that
   * grows the forward end on its own gradient waves (workgroups = pair_grid(tiles), see
   * `workgroups`); same draws bit for bit.  A partner that gets no CU at launch leaves its
   * tile to grow both ends itself (fitoct_result::paired_transitions counts the paired ones). */
  int32_t paired;
  int32_t workgroups;      /* workgroups launched (tiles, or 16 * ceil(tiles / 8) when paired) */
  /* ABI 8: how the sweep forms the GP modulation.  0: the factorised basis (per-bin
   * polynomial, K^-1 products in the sampler's leaf); 1: the basis rows B[i, :] (resident in
   * the gradient waves' registers for N <= 512 -- bins_per_thread 1 or 2 -- or streamed for
   * a caller's basis).  The struct's size is unchanged (the slot was padding). */
  int32_t basis_mode;
} fitoct_plan_info;

/* fitoct_plan_info::sampler.  PLAIN: no speculation, no migration;
 * MIGRATE: chains move between tiles at transition boundaries (work balance);
 * SPECULATIVE: speculative leaves -- a chain's next leapfrog position is swept while the
 * current leaf's tree bookkeeping runs: always in a tile of one chain (a spare wave
 * helps), and in migrating tiles of several chains once they have thinned out to <= 3
 * live chains (the launch's tail);
 * MIGRATE_SPEC: both (the headline shape).  FITOCT_NO_SPEC=1 / FITOCT_NO_MIGRATE=1 turn
 * either off.  The draws are the same bit for bit whichever variant runs. */
#define FITOCT_SAMPLER_PLAIN 0
#define FITOCT_SAMPLER_MIGRATE 1
#define FITOCT_SAMPLER_SPECULATIVE 2
#define FITOCT_SAMPLER_MIGRATE_SPEC 3

typedef struct fitoct_plan fitoct_plan;

/* ---- library ---------------------------------------------------------- */
int32_t fitoct_abi_version(void);
const char* fitoct_last_error(void);
int32_t fitoct_device_count(void);
/* sizeof of the ABI structs, so bindings can assert their layout */
int32_t fitoct_struct_sizes(int32_t* problem, int32_t* config, int32_t* result, int32_t* info);
void fitoct_default_config(fitoct_config* cfg);
void fitoct_default_problem(fitoct_problem* prob);

/* ---- model layout (host only) -------------------------------------------- */
int32_t fitoct_dim(int32_t prior_type, int32_t Nn);
int32_t fitoct_n_cols(int32_t prior_type, int32_t Nn);
/* Stan-CSV style name of draw column i (lp__, accept_stat__, ..., theta.1, ...) */
int32_t fitoct_column_name(int32_t prior_type, int32_t Nn, int32_t i, char* buf, int32_t buflen);

/* FitOCTLib::fitMonoExp's starting point for theta from the data alone (x[N], y[N]):
 * theta1 = median of the deepest max(3, N/10) bins, then a least-squares line through
 * log(y - theta1) where y - theta1 > 5% of its maximum gives theta2 (intercept) and
 * theta3 = dataType / -slope.  Only the optimiser's / sampler's start (⚑ FitOCTLib's
 * own initialisation is not visible). */
int32_t fitoct_mono_initial_theta(int32_t N, const double* x, const double* y, int32_t data_type,
                                  double* theta_out /*[3]*/);

/* ---- GP basis (host only, fp64 Cholesky) --------------------------------- */
int32_t fitoct_build_basis(const fitoct_problem* prob, double* B_out /*[N*Nn]*/,
                           double* xGP_out /*[Nn] or NULL*/);

/* ---- hot path ------------------------------------------------------------ */
/* log density and gradient at n_points unconstrained positions q[n_points][D]
 * (host buffers); lp_out[n_points], grad_out[n_points][D], sumr2_out[n_points]
 * (sum(((y-m)/uy)^2), NULL allowed). */
int32_t fitoct_logp_grad(const fitoct_problem* prob, int32_t n_points, const double* q,
                         double* lp_out, double* grad_out, double* sumr2_out,
                         int32_t precision, int32_t device);

/* one-shot: plan + run + download + destroy */
int32_t fitoct_expgp_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res);

int32_t fitoct_plan_create(const fitoct_problem* prob, const fitoct_config* cfg,
                           fitoct_plan** out);
int32_t fitoct_plan_get_info(const fitoct_plan* plan, fitoct_plan_info* info);
/* Run the sampler on `stream` (hipStream_t; NULL = default stream).  If d_draws is
 * non-NULL the draws go to that caller-owned DEVICE buffer (>= info.draws_bytes),
 * otherwise to a plan-internal one.  Returns after the kernel completes.
 * Multi-device plans (cfg.n_devices > 1): `stream` must be NULL.  Each device's shard
 * runs on a private non-blocking stream of the library (shards never order against
 * each other); d_draws may live on any device: the shards on that device write their
 * blocks in place and every other block is copied into it peer-to-peer over xGMI once
 * its device has finished (the one gather of SURVEY.md §8e, inside one process; peer
 * access between the buffer's device and each shard's device is enabled on first use).
 * Ordering rule: the in-place shards start after all work the caller queued on the
 * buffer device's NULL stream before this call (an event recorded there), so a fill or
 * copy into d_draws issued on that stream cannot land after the draws.
 * The poll / cancel / wait / download / set_init calls below act on every device; a
 * failure on one device cancels the others and the call returns that one status.
 * set_init checks every block before any device takes its part. */
int32_t fitoct_plan_run(fitoct_plan* plan, void* d_draws, void* stream);
/* The same run in two halves, for long fits driven from an interactive host.  It
 * replaces the progress that rstan writes to stan.log and the Shiny server reads
 * (server.R:457-484).  The R shim runs the poll loop on the R main thread, between
 * R_CheckUserInterrupt checks (threading).
 *   fitoct_plan_launch  enqueue the sampler on `stream` and return at once;
 *   fitoct_plan_poll    transitions completed so far over all chains (each chain
 *                       publishes its count at every transition boundary), the total
 *                       chains * (warmup + samples), and whether the kernel has drained;
 *   fitoct_plan_cancel  ask every chain to stop at its next 8th transition boundary
 *                       (it then reports FITOCT_E_CANCELLED; the kernel drains);
 *   fitoct_plan_wait    block until the launch has drained (then download as usual).
 * fitoct_plan_run = launch + wait.  Batch plans have no progress/cancel channel. */
int32_t fitoct_plan_launch(fitoct_plan* plan, void* d_draws, void* stream);
int32_t fitoct_plan_poll(fitoct_plan* plan, int64_t* iterations_done, int64_t* iterations_total,
                         int32_t* finished);
int32_t fitoct_plan_cancel(fitoct_plan* plan);
int32_t fitoct_plan_wait(fitoct_plan* plan);
/* Warm restart (SURVEY.md §5 "Checkpoint / resume"; rstan::sampling's `init`, `control =
 * list(stepsize)` and CmdStan's `inv_metric`): per-chain starting values for the plan's
 * next runs, host buffers copied at once (NULL = keep that default):
 *   q_init     [chains][D] unconstrained positions, e.g. a previous run's last_q;
 *   stepsize   [chains] initial step sizes (> 0), e.g. its stepsize;
 *   inv_metric [chains][D] diagonal inverse metrics (> 0), e.g. its inv_metric.
 * Defaults: the jittered start around theta0 (init_radius), cfg.stepsize, a unit metric.
 * With adapt_engaged = 0 the chains sample with that step size and metric unchanged; with
 * adaptation they are where Stan's adaptation starts (step-size search, windows).  A chain
 * whose q_init has a non-finite lp / gradient fails with FITOCT_E_INIT (no retry: Stan
 * rejects a user init likewise).  A NULL argument clears that input.  Not while a launch
 * is in flight (FITOCT_E_ARG). */
int32_t fitoct_plan_set_init(fitoct_plan* plan, const double* q_init, const double* stepsize,
                             const double* inv_metric);
/* Copy the last run's outputs to host buffers of `res`. */
int32_t fitoct_plan_download(fitoct_plan* plan, fitoct_result* res);
void fitoct_plan_destroy(fitoct_plan* plan);

/* ---- batch mode ---------------------------------------------------------- *
 * Replaces FitOCT.R's per-file loop (FitOCT.R:70-124: one FitOCTLib::fitExpGP ->
 * rstan::sampling call per Courbe.csv) with ONE persistent launch sampling every
 * file's chains: `n_problems` problems sharing prior_type and Nn, each with
 * cfg->chains chains (a tile never mixes files).  Chain c of problem p is keyed
 * as global chain cfg->chain_offset + p*cfg->chains + c, so problem p's draws
 * equal a single plan of it with chain_offset = cfg->chain_offset + p*chains.
 * Draws land in [n_problems][chains][iters_saved][n_cols] (caller device buffer
 * of info.draws_bytes, or internal).  Caller buffers are not retained.
 * With a device list (cfg.n_devices > 1) the files are split into contiguous blocks,
 * one sub-batch per device (stream must be NULL; the ordering rule of fitoct_plan_run
 * applies to d_draws).  When one device's run fails (a HIP error: the call returns that
 * status) the other devices' chains stop at their next checked transition boundary
 * instead of running on.  A failed chain of one file (e.g. FITOCT_E_INIT) is only that
 * file's status at download, with or without a device list: files are independent fits. */
typedef struct fitoct_batch fitoct_batch;
int32_t fitoct_batch_create(const fitoct_problem* probs, int32_t n_problems,
                            const fitoct_config* cfg, fitoct_batch** out);
int32_t fitoct_batch_get_info(const fitoct_batch* batch, fitoct_plan_info* info);
int32_t fitoct_batch_run(fitoct_batch* batch, void* d_draws, void* stream);
/* outputs of problem `problem` (draws of that problem only), as fitoct_plan_download */
int32_t fitoct_batch_download(fitoct_batch* batch, int32_t problem, fitoct_result* res);
void fitoct_batch_destroy(fitoct_batch* batch);

/* ---- batched density evaluator ------------------------------------------- *
 * The model of a problem staged once in HBM, evaluated at up to `capacity`
 * points per call by the same kernel as fitoct_logp_grad (which is a one-shot
 * evaluator).  Replaces rstan's log_prob / grad_log_prob methods of a stanfit
 * (used by optimHess inside rstan::optimizing).  `jacobian` = 0 drops the
 * log-Jacobian of the positivity transforms (Stan optimizing); `normalised` = 1
 * adds the constants dropped by `~` statements (Stan log_prob<propto=false>). */
typedef struct fitoct_evaluator fitoct_evaluator;
int32_t fitoct_evaluator_create(const fitoct_problem* prob, int32_t capacity, int32_t precision,
                                int32_t device, fitoct_evaluator** out);
int32_t fitoct_evaluator_run(fitoct_evaluator* ev, int32_t n_points, const double* q,
                             int32_t jacobian, int32_t normalised, double* lp_out,
                             double* grad_out /* [n][D] or NULL */, double* sumr2_out);
void fitoct_evaluator_destroy(fitoct_evaluator* ev);
/* unconstrained q[n][D] -> constrained parameters in draw-column order (theta,
 * yGP/z, lambda, sigma, ...: columns 7..7+D-1 of fitoct_column_name) */
int32_t fitoct_constrain(int32_t prior_type, int32_t Nn, int32_t n_points, const double* q,
                         double* out);

/* ---- rstan::optimizing (FitOCT.R:42 method='optim'; server.R:156-172) ------ *
 * L-BFGS on the log density without Jacobian (Stan's defaults below), then the
 * Hessian on the unconstrained scale by central differences of the gradient
 * with step `hessian_step` (rstan's optimHess, ndeps = 1e-3), all 2D
 * displaced points evaluated in one batched launch. */
typedef struct fitoct_optim_config {
  int32_t iter;          /* 2000 */
  int32_t history;       /* 5 */
  double init_alpha;     /* 1e-3: first line-search step */
  double tol_obj;        /* 1e-12 */
  double tol_rel_obj;    /* 1e4  (x machine eps) */
  double tol_grad;       /* 1e-8 */
  double tol_rel_grad;   /* 1e7  (x machine eps) */
  double tol_param;      /* 1e-8 */
  int32_t hessian;       /* 1: fill res->hessian */
  int32_t jacobian;      /* 0 (Stan optimizing) */
  double hessian_step;   /* 1e-3 */
  int32_t precision;
  int32_t device;
} fitoct_optim_config;

/* Stan's BFGS termination codes */
enum { FITOCT_TERM_SUCCESS = 0, FITOCT_TERM_ABSX = 10, FITOCT_TERM_ABSF = 20,
       FITOCT_TERM_RELF = 21, FITOCT_TERM_ABSGRAD = 30, FITOCT_TERM_RELGRAD = 31,
       FITOCT_TERM_MAXIT = 40, FITOCT_TERM_LSFAIL = -1 };

typedef struct fitoct_optim_result {
  double* par;           /* [D] out: unconstrained optimum (caller-owned) */
  double* hessian;       /* [D][D] out (NULL = not wanted): Hessian of lp, unconstrained */
  double value;          /* lp at the optimum (propto=false, jacobian per config) */
  double sumr2;          /* sum(((y-m)/uy)^2) at the optimum (br = sumr2 / N) */
  int32_t iterations;
  int32_t n_evals;       /* density evaluations (points) */
  int32_t termination;   /* FITOCT_TERM_* */
  int32_t return_code;   /* 0 = terminated normally (rstan return_code), 70 = error */
} fitoct_optim_result;

void fitoct_default_optim_config(fitoct_optim_config* cfg);
/* init_q: [D] unconstrained start (NULL -> theta = theta0, everything else 0) */
int32_t fitoct_optimize(const fitoct_problem* prob, const fitoct_optim_config* cfg,
                        const double* init_q, fitoct_optim_result* res);

/* ---- rstan::vb, mean-field ADVI (FitOCT.R:42 method='vb') -------------------- *
 * Stan's algorithm (Kucukelbir et al. 2017): eta adaptation over
 * {100, 10, 1, 0.1, 0.01}, adaGrad-style steps, relative-ELBO convergence on a
 * rolling window.  Random numbers are Philox-addressed by (seed, eta index,
 * iteration), so the five adaptation runs are evaluated side by side in one
 * batch and give the same result as Stan's sequential loop would. */
typedef struct fitoct_vb_config {
  int32_t iter;            /* 10000 */
  int32_t grad_samples;    /* 1 */
  int32_t elbo_samples;    /* 100 */
  int32_t eval_elbo;       /* 100 */
  double eta;              /* step size when adapt_engaged = 0 */
  int32_t adapt_engaged;   /* 1 */
  int32_t adapt_iter;      /* 50 */
  double tol_rel_obj;      /* 0.01 */
  int32_t output_samples;  /* 1000 */
  int32_t pad_;
  uint64_t seed;
  int32_t precision;
  int32_t device;
} fitoct_vb_config;

typedef struct fitoct_vb_result {
  double* mu;              /* [D] out: mean of the approximation (unconstrained) */
  double* omega;           /* [D] out: log standard deviations */
  double* draws;           /* [output_samples][D] out: unconstrained draws, or NULL */
  double* log_p;           /* [output_samples] log density (propto=false, jacobian), or NULL */
  double* log_g;           /* [output_samples] -0.5 |eta|^2 of each draw, or NULL */
  double* sumr2;           /* [output_samples] or NULL */
  double eta;              /* adapted / used step size */
  double elbo;             /* last ELBO estimate */
  int32_t iterations;
  int32_t converged;       /* 1 mean or median relative ELBO change < tol_rel_obj */
  int32_t n_evals;
  int32_t pad_;
} fitoct_vb_result;

void fitoct_default_vb_config(fitoct_vb_config* cfg);
int32_t fitoct_vb(const fitoct_problem* prob, const fitoct_vb_config* cfg, const double* init_q,
                  fitoct_vb_result* res);

/* ---- Stan output (host only) ------------------------------------------------ *
 * Replaces the stanfit that rstan::sampling / rstan::vb return inside
 * FitOCTLib::fitExpGP.  Its consumers ask for pars = c('theta','yGP','lambda','sigma',
 * 'br','lp__') for every prior family (plotExpGP.R:9,41-43; server.R:88-237), so the
 * output layout is the kernel's draw columns plus the model's transformed parameters,
 * in Stan's order (parameters, transformed parameters, generated quantities):
 *   normal    : theta[3] yGP[Nn] lambda sigma br
 *   lasso     : theta[3] yGP[Nn] sigma lambda br        (⚑ lambda = lambda_scale, a constant:
 *                                                        lassoPrior.stan:4 has it as data)
 *   horseshoe : theta[3] z[Nn] r1_global r2_global r1_local[Nn] r2_local[Nn] sigma
 *               tau lambda[Nn] yGP[Nn] br              (horseShoePrior.stan:25-33)
 *   monoexp   : theta[3] br
 * br is dropped when prior_PD = 1 (plotExpGP.R:42-43).  Only prior_type, Nn, prior_PD
 * and lambda_scale of `prob` are read by the layout functions. */
/* number and names of the output parameter columns (after any leading columns) */
int32_t fitoct_output_n_params(const fitoct_problem* prob);
int32_t fitoct_output_param_name(const fitoct_problem* prob, int32_t i, char* buf, int32_t buflen);
/* raw rows [n_rows][n_lead + D + 1] (n_lead leading columns copied as they are -- 7 sampler
 * columns for kernel draws, 0 for a bare parameter row --, then the D constrained
 * parameters and br) -> out [n_rows][n_lead + fitoct_output_n_params] */
int32_t fitoct_output_rows(const fitoct_problem* prob, int32_t n_lead, int64_t n_rows,
                           const double* raw, double* out);
/* One chain of a sampler run as a CmdStan CSV file (rstan::read_stan_csv builds the
 * stanfit from it: print, extract, as.matrix, summary()$summary with Rhat / n_eff,
 * traceplot(inc_warmup = TRUE), pairs).  raw: that chain's kernel draws
 * [iters_saved][fitoct_n_cols] (warmup rows first when cfg->save_warmup); the file has
 * the CmdStan argument header, the output columns above, the adaptation block
 * (step size, diagonal inverse metric) between warmup and sampling rows, and the
 * elapsed-time trailer.  `chain` indexes cfg's chains (id = chain_offset + chain + 1). */
int32_t fitoct_write_stan_csv(const char* path, const fitoct_problem* prob,
                              const fitoct_config* cfg, int32_t chain, const double* raw,
                              double stepsize, const double* inv_metric /*[D] or NULL*/,
                              double warmup_s, double sampling_s);
/* A mean-field ADVI result as CmdStan's variational CSV (first row: the constrained mean
 * of the approximation; then one row per unconstrained draw q[n][D] with lp__ = 0,
 * log_p__, log_g__).  mean_sumr2 / sumr2 give br (NaN when unknown / NULL). */
int32_t fitoct_write_vb_csv(const char* path, const fitoct_problem* prob,
                            const fitoct_vb_config* cfg, const double* mu, double mean_sumr2,
                            int32_t n, const double* q, const double* log_p, const double* log_g,
                            const double* sumr2, double eta);
/* Generated quantities of n parameter rows (plotExpGP.R:46-57 spaghetti draws,
 * fit$par$m / fit$par$resid of plotMonoExp.R:15-16): dL = B yGP,
 * m = theta1 + theta2 exp(-c x / (theta3 (1 + dL))), resid = (y - m) / uy, br = mean(resid^2).
 * theta[n][3], ygp[n][Nn] (ignored for FITOCT_MODEL_MONOEXP); outputs [n][N] (br [n]),
 * each NULL if not wanted.  The basis is prob->B or built as fitoct_build_basis does. */
int32_t fitoct_expgp_curves(const fitoct_problem* prob, int32_t n, const double* theta,
                            const double* ygp, double* dL, double* m, double* resid, double* br);

/* rstan's progress line for a run that has completed `done` of `total` transitions
 * (fitoct_plan_poll) with `warmup` + `samples` iterations per chain:
 *     "Chain k: Iteration: i / n [ p%]  (Warmup|Sampling)"
 * The Shiny server tails these lines from stan.log and decodes the overall fraction as
 * ((k - 1) * 100 + p) / 4, i.e. it assumes 4 chains run one after another
 * (server.R:457-472).  All chains of a fitoct run advance together, so the line encodes
 * the run's overall fraction f = done / total in that convention: 4 f = (k - 1) + p / 100,
 * and i = round(p / 100 * n) is the matching per-chain iteration.  Returns
 * floor(100 f) (callers print when it changes) or a negative fitoct_status. */
int32_t fitoct_progress_line(int64_t done, int64_t total, int32_t warmup, int32_t samples,
                             char* buf, int32_t buflen);

/* ---- diagnostics (host only) ---------------------------------------------- */
/* x[chains][n] of one scalar: rstan legacy split-R-hat and n_eff (autocorrelation,
 * Geyer initial monotone sequence), as shown by rstan::summary (server.R:88-104). */
int32_t fitoct_split_rhat_ess(const double* x, int32_t chains, int32_t n,
                              double* rhat, double* ess);
/* rank-normalised split-R-hat (Vehtari et al. 2021), max of bulk and folded. */
int32_t fitoct_rank_rhat(const double* x, int32_t chains, int32_t n, double* rhat);

#ifdef __cplusplus
}
#endif
#endif /* FITOCT_H */
