/* See fitoct_drive.h.  Plain C99 over the C ABI of include/fitoct.h. */
#define _POSIX_C_SOURCE 199309L
#include "fitoct_drive.h"

#include <time.h>

static void sleep_ms(int32_t ms) {
  struct timespec ts;
  ts.tv_sec = ms / 1000;
  ts.tv_nsec = (long)(ms % 1000) * 1000000L;
  nanosleep(&ts, NULL);
}

int32_t fitoct_drive_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                            fitoct_result* res, int32_t poll_ms, fitoct_progress_fn progress,
                            fitoct_interrupt_fn interrupted, void* ctx) {
  fitoct_plan* plan = NULL;
  int32_t rc = fitoct_plan_create(prob, cfg, &plan);
  if (rc != FITOCT_OK) return rc;            /* nothing allocated */
  rc = fitoct_plan_launch(plan, NULL, NULL);
  int cancelled = 0;
  if (rc == FITOCT_OK) {
    int64_t done = 0, total = 0, last = -1;
    int32_t fin = 0;
    if (poll_ms <= 0) poll_ms = 50;
    for (;;) {
      rc = fitoct_plan_poll(plan, &done, &total, &fin);
      if (rc != FITOCT_OK || fin) break;
      if (!cancelled && interrupted && interrupted(ctx)) {
        rc = fitoct_plan_cancel(plan);       /* chains stop at their next 8th transition */
        if (rc != FITOCT_OK) break;
        cancelled = 1;
      }
      if (progress && !cancelled && done != last) {
        progress(ctx, done, total);
        last = done;
      }
      sleep_ms(poll_ms);
    }
    /* always drain the launch before the plan's buffers go away */
    const int32_t rw = fitoct_plan_wait(plan);
    if (rc == FITOCT_OK) rc = rw;
    if (rc == FITOCT_OK) rc = fitoct_plan_download(plan, res);
    if (rc == FITOCT_OK && progress) progress(ctx, total, total);
  }
  fitoct_plan_destroy(plan);
  if (cancelled && (rc == FITOCT_OK || rc == FITOCT_E_CANCELLED)) rc = FITOCT_E_CANCELLED;
  return rc;
}
