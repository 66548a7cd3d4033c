/* fitoct_drive: the R-independent half of FitOCTLib's .Call shim (fitoct_R.c).
 *
 * Runs one fitExpGP / fitMonoExp fit through the C ABI of include/fitoct.h on the
 * calling thread.  For method = 'sample': create -> launch -> poll loop -> wait ->
 * download -> destroy; between polls it asks the host whether the user interrupted
 * (R: R_CheckUserInterrupt under R_ToplevelExec, so no longjmp crosses this code)
 * and reports progress.  On an interrupt it cancels the launch, waits for the kernel
 * to drain and returns FITOCT_E_CANCELLED.  Every library resource is released
 * before it returns, whatever the outcome (errors, threading,
 * ownership).
 *
 * Kept free of R headers so that it is compiled and tested in this repository
 * (tests/test_rshim_driver.py) where R is absent: everything the R wrapper
 * (rshim/R/fitExpGP.R) receives is produced here.
 */
#ifndef FITOCT_DRIVE_H
#define FITOCT_DRIVE_H
#include "fitoct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t (*fitoct_interrupt_fn)(void* ctx);                          /* nonzero: stop */
typedef void (*fitoct_progress_fn)(void* ctx, int64_t done, int64_t total);
typedef void (*fitoct_line_fn)(void* ctx, const char* line);                /* one text line */

/* poll_ms: host sleep between polls (<= 0 -> 50 ms).  progress / interrupted may be NULL.
 * progress is called when the completed-transition count changed, and once at the end
 * with done == total on success.  Returns FITOCT_OK or a negative fitoct_status. */
int32_t fitoct_drive_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res, int32_t poll_ms, fitoct_progress_fn progress,
                            fitoct_interrupt_fn interrupted, void* ctx);

/* fitExpGP(method = 'sample') as the R wrapper runs it.
 *  - progress: rstan-format lines "Chain k: Iteration: i / n [ p%]  (Warmup|Sampling)"
 *    (fitoct_progress_line) go to `line` whenever the overall percentage changes, whatever
 *    open_progress is: the Shiny server sinks stdout to stan.log and parses them
 *    (server.R:391-393,457-484; FitOCT.R:123 and server.R:425 pass open_progress = FALSE);
 *  - output: one Stan CSV per chain at paths[0 .. cfg->chains-1] (fitoct_write_stan_csv),
 *    which the wrapper hands to rstan::read_stan_csv.  Elapsed warmup / sampling times of
 *    a chain split the kernel time by that chain's n_leapfrog__ in each phase.
 * line may be NULL.  Host buffers are allocated and freed here. */
int32_t fitoct_drive_sample_csv(const fitoct_problem* prob, const fitoct_config* cfg,
                                const char* const* paths, int32_t poll_ms, fitoct_line_fn line,
                                fitoct_interrupt_fn interrupted, void* ctx);

/* fitExpGP(method = 'sample') for many chains (config 4: 8192), where one Stan CSV file per
 * chain (fitoct_drive_sample_csv: ~1500 text rows each, parsed by rstan::read_stan_csv)
 * does not scale.  Same run, progress and interrupts as fitoct_drive_sample_csv; the
 * outputs stay binary and land in caller buffers that R allocates as its own vectors:
 *  - draws [chains][n_out][rows], n_out = 7 + fitoct_output_n_params(prob): per chain,
 *    every output column (the 7 sampler columns lp__ .. energy__, then the parameters,
 *    transformed parameters and br of the output layout) as one contiguous run of
 *    `rows` = iters_saved values.  This is R's column-major array(dim = c(rows, n_out,
 *    chains)): the wrapper hands it, unchanged, to the stanfit constructor
 *    (rshim/R/fitExpGP.R:fitoct_stanfit);
 *  - stepsize [chains], inv_metric [chains][D] (Stan's adaptation info);
 *  - elapsed [chains][2]: warmup / sampling seconds (the kernel time split by each
 *    chain's n_leapfrog__ in each phase, as in the CSV trailer).
 * draws_capacity is the number of doubles at `draws`.  Host buffers are caller-owned. */
int32_t fitoct_drive_sample_bulk(const fitoct_problem* prob, const fitoct_config* cfg,
                                 double* draws, int64_t draws_capacity, double* stepsize,
                                 double* inv_metric, double* elapsed, int32_t poll_ms,
                                 fitoct_line_fn line, fitoct_interrupt_fn interrupted, void* ctx);
/* The layout step alone (host only): raw kernel draws [chains][rows][fitoct_n_cols] ->
 * out [chains][n_out][rows] as above. */
int32_t fitoct_drive_bulk_layout(const fitoct_problem* prob, int32_t chains, int64_t rows,
                                 const double* raw, double* out);

/* method = 'optim' (rstan::optimizing(hessian = TRUE) inside FitOCTLib::fitExpGP /
 * fitMonoExp; read as fit$par$theta, fit$par$br, fit$par$m, fit$par$resid, fit$hessian at
 * plotExpGP.R:13-18, plotMonoExp.R:15-16, server.R:107-172).
 *  par_out     [fitoct_output_n_params]: the optimum in the output layout (names from
 *              fitoct_output_param_name; br from the residuals at the optimum);
 *  hessian_out [D][D] or NULL: Hessian of lp on the unconstrained scale, rows / columns
 *              named like the draw columns 7..7+D-1 (fitoct_column_name);
 *  dL/m/resid  [N] or NULL: generated quantities at the optimum (fitoct_expgp_curves);
 *  value, return_code: rstan's `value` and `return_code`. */
int32_t fitoct_drive_optimize(const fitoct_problem* prob, const fitoct_optim_config* cfg,
                              const double* init_q, double* par_out, double* hessian_out,
                              double* dL, double* m, double* resid, double* value,
                              int32_t* return_code);

/* method = 'vb' (rstan::vb): mean-field ADVI, written as CmdStan's variational CSV at
 * `path` (fitoct_write_vb_csv; br of the mean row from the residuals at the mean). */
int32_t fitoct_drive_vb_csv(const fitoct_problem* prob, const fitoct_vb_config* cfg,
                            const double* init_q, const char* path);

#ifdef __cplusplus
}
#endif
#endif
