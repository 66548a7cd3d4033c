/* fitoct_drive: the R-independent half of FitOCTLib's .Call shim (fitoct_R.c).
 *
 * Runs one fitExpGP(method='sample') fit through the plan API of include/fitoct.h on
 * the calling thread: create -> launch -> poll loop -> wait -> download -> destroy.
 * Between polls it asks the host whether the user interrupted (R: R_CheckUserInterrupt
 * under R_ToplevelExec, so no longjmp crosses this code) and reports progress (R:
 * Rprintf lines that replace the stan.log progress the Shiny server reads,
 * server.R:457-484).  On an interrupt it cancels the launch, waits for the kernel to
 * drain and returns FITOCT_E_CANCELLED.  Every library resource is released before it
 * returns, whatever the outcome (errors, threading, ownership).
 *
 * Kept free of R headers so that it is compiled and tested in this repository
 * (tests/test_rshim_driver.py) where R is absent.
 */
#ifndef FITOCT_DRIVE_H
#define FITOCT_DRIVE_H
#include "fitoct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t (*fitoct_interrupt_fn)(void* ctx);                          /* nonzero: stop */
typedef void (*fitoct_progress_fn)(void* ctx, int64_t done, int64_t total);

/* poll_ms: host sleep between polls (<= 0 -> 50 ms).  progress / interrupted may be NULL.
 * progress is called when the completed-transition count changed, and once at the end
 * with done == total on success.  Returns FITOCT_OK or a negative fitoct_status. */
int32_t fitoct_drive_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res, int32_t poll_ms, fitoct_progress_fn progress,
                            fitoct_interrupt_fn interrupted, void* ctx);

#ifdef __cplusplus
}
#endif
#endif
