// Multi-device plans and batches: the device list of fitoct_config (include/fitoct.h,
// SURVEY.md §8b "device list", R fitExpGP(n_gpus = k)).
//
// The reference parallelises rstan's chains over host cores with
// options(mc.cores = parallel::detectCores()) (FitOCT.R:13, ShinyInterface/server.R:19,
// Tests/testGamma.R:13).  Here the chains of one call are split into contiguous blocks
// of global chain ids, one block per device, and every device runs its block through the
// single-device plan path in a host thread of its own (plan creation: basis, staging and
// allocation; the wait, the xGMI copy into the caller's buffer, the download).  Chains
// are independent and their random streams are keyed by global chain id, so there is no
// exchange between devices and the draws equal a one-device run bit for bit.  The one
// data movement between devices is the gather of every block into the caller's device
// buffer (hipMemcpyPeer over xGMI), the in-process counterpart of the RCCL gather of the
// torch.distributed path (fitoct_amd/distributed.py).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"
#include "plan_internal.h"

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(FITOCT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

namespace fitoct {

void block_range(int total, int n, int r, int& off, int& cnt) {
  const int base = total / n, rem = total % n;
  cnt = base + (r < rem ? 1 : 0);
  off = r * base + std::min(r, rem);
}

int resolve_devices(const fitoct_config* cfg, int units, std::vector<int>& devs) {
  devs.clear();
  if (cfg->n_devices == 0) {
    devs.push_back(cfg->device);
    return FITOCT_OK;
  }
  if (cfg->n_devices < 0 || cfg->n_devices > FITOCT_MAX_DEVICES)
    return fail(FITOCT_E_ARG, "n_devices must be in [0, FITOCT_MAX_DEVICES = " +
                                  std::to_string(FITOCT_MAX_DEVICES) + "]");
  for (int r = 0; r < cfg->n_devices; ++r)
    if (cfg->devices[r] < 0)
      return fail(FITOCT_E_ARG, "devices[" + std::to_string(r) + "] is negative");
  const int used = std::max(1, std::min(cfg->n_devices, units));
  devs.assign(cfg->devices, cfg->devices + used);
  return FITOCT_OK;
}

namespace {

// The calling thread's HIP device is restored when a multi-device call returns (the
// shards switch it; a caller such as PyTorch keeps its own notion of the current device).
struct DeviceRestore {
  int dev = -1;
  DeviceRestore() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceRestore() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

// f(r) for r in [0, n) on one host thread per device (r = 0 on the calling thread).
// Returns FITOCT_OK, or the status of the lowest-numbered failure that is not a
// cancellation (a device reports FITOCT_E_CANCELLED when another device's failure
// stopped it), with that failure's message moved to the calling thread
// (fitoct_last_error is thread-local).
template <class F>
int on_devices(int n, F&& f) {
  std::vector<int> rc(n, FITOCT_OK);
  std::vector<std::string> msg(n);
  auto body = [&](int r) {
    rc[r] = guarded("device worker", [&]() -> int32_t { return f(r); });
    if (rc[r] != FITOCT_OK) msg[r] = g_last_error;
  };
  std::vector<std::thread> th;
  th.reserve(n);
  int started = 1;
  try {
    for (int r = 1; r < n; ++r, ++started) th.emplace_back(body, r);
  } catch (...) {   // no thread for device `started` onwards: report it, run nothing there
    for (int r = started; r < n; ++r) {
      rc[r] = FITOCT_E_INTERNAL;
      msg[r] = "could not start a host thread for device " + std::to_string(r);
    }
  }
  body(0);
  for (auto& t : th) t.join();
  int first = -1;
  for (int r = 0; r < n && first < 0; ++r)
    if (rc[r] != FITOCT_OK && rc[r] != FITOCT_E_CANCELLED) first = r;
  for (int r = 0; r < n && first < 0; ++r)
    if (rc[r] != FITOCT_OK) first = r;
  return first < 0 ? FITOCT_OK : fail(rc[first], msg[first]);
}

// the device a caller's d_draws buffer lives on (FITOCT_E_ARG if it is not device memory)
int buffer_device(const void* p, int& dev) {
  hipPointerAttribute_t a{};
  HIP_TRY(hipPointerGetAttributes(&a, p));
  if (a.type != hipMemoryTypeDevice)
    return fail(FITOCT_E_ARG, "d_draws must be a device buffer (hipMalloc)");
  dev = a.device;
  return FITOCT_OK;
}

// FITOCT_GATHER_COPY=1 (tests): blocks on the buffer's own device are also written to a
// device-internal buffer and copied, so one GPU exercises the copy path of the gather
bool in_place(const void* d_draws, int dev, int gdev) {
  static const bool force_copy = getenv("FITOCT_GATHER_COPY") != nullptr;
  return d_draws && dev == gdev && !force_copy;
}

// a non-blocking stream on `dev` for one shard: the shards of a group never order
// against each other, nor against the synchronous status reads / peer copies issued
// for another shard, through the device's default stream
int own_stream(int dev, hipStream_t& st) {
  HIP_TRY(hipSetDevice(dev));
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  return FITOCT_OK;
}

// Peer access between the gather buffer's device and a shard's device, enabled once per
// pair and direction for the process (hipMemcpyPeer then moves the block over xGMI; without
// it the runtime stages the copy through host memory).  A pair the hardware cannot map, or
// whose enabling fails, is remembered too and left to the staged copy: peer access is a
// speed-up of the gather, never a reason to fail the call.
int enable_peer(int gdev, int sdev) {
  if (gdev < 0 || gdev == sdev) return FITOCT_OK;
  static std::mutex mu;
  static std::set<std::pair<int, int>> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({gdev, sdev})) return FITOCT_OK;
  int can_g = 0, can_s = 0;
  HIP_TRY(hipDeviceCanAccessPeer(&can_g, gdev, sdev));
  HIP_TRY(hipDeviceCanAccessPeer(&can_s, sdev, gdev));
  const std::pair<int, int> dirs[2] = {{gdev, sdev}, {sdev, gdev}};
  const int can[2] = {can_g, can_s};
  for (int i = 0; i < 2; ++i) {
    if (!can[i]) continue;
    HIP_TRY(hipSetDevice(dirs[i].first));
    if (hipDeviceEnablePeerAccess(dirs[i].second, 0) != hipSuccess)
      (void)hipGetLastError();   // already enabled elsewhere, or unavailable: staged copy
  }
  done.insert({gdev, sdev});
  return FITOCT_OK;
}

// The ordering rule of fitoct_plan_run for a caller buffer (include/fitoct.h): an event
// recorded on the buffer device's NULL stream, which every in-place shard's private stream
// waits on before its first write into the buffer.
struct NullStreamFence {
  hipEvent_t ev = nullptr;
  int dev = -1;
  ~NullStreamFence() {
    if (ev) {
      (void)hipSetDevice(dev);
      (void)hipEventDestroy(ev);
    }
  }
  int record(int gdev) {
    dev = gdev;
    HIP_TRY(hipSetDevice(gdev));
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ev, nullptr));
    return FITOCT_OK;
  }
  int order(hipStream_t st) const {
    if (ev) HIP_TRY(hipStreamWaitEvent(st, ev, 0));
    return FITOCT_OK;
  }
};

size_t chain_bytes(const fitoct_plan* sh) {
  return sizeof(double) * (size_t)sh->kp.iters_saved * sh->kp.ncols;
}

}  // namespace

// ---- plans ------------------------------------------------------------------------
int group_plan_create(const fitoct_problem* prob, const fitoct_config* cfg,
                      const std::vector<int>& devs, fitoct_plan** out) {
  const int n = (int)devs.size(), C = cfg->chains;
  std::unique_ptr<fitoct_plan, void (*)(fitoct_plan*)> guard(new fitoct_plan(),
                                                             fitoct_plan_destroy);
  fitoct_plan* pl = guard.get();
  pl->shards.assign(n, nullptr);
  pl->shard_off.assign(n, 0);
  DeviceRestore keep;
  const int rc = on_devices(n, [&](int r) -> int {
    int off, cnt;
    block_range(C, n, r, off, cnt);
    fitoct_config c = *cfg;
    c.chains = cnt;
    c.chain_offset = cfg->chain_offset + off;
    c.device = devs[r];
    c.n_devices = 0;
    pl->shard_off[r] = off;
    const int e = fitoct_plan_create(prob, &c, &pl->shards[r]);
    return e ? fail(e, "device " + std::to_string(devs[r]) + ": " + g_last_error) : FITOCT_OK;
  });
  if (rc) return rc;
  const fitoct_plan* s0 = pl->shards[0];
  pl->cfg = *cfg;
  pl->prob = s0->prob;   // caller pointers already dropped
  pl->kp = s0->kp;
  pl->kp.chains = C;
  pl->kp.chain_offset = cfg->chain_offset;
  for (const fitoct_plan* sh : pl->shards) {
    pl->draws_bytes += sh->draws_bytes;
    pl->tiles += sh->tiles;
  }
  *out = guard.release();
  return FITOCT_OK;
}

int group_plan_info(const fitoct_plan* pl, fitoct_plan_info* info) {
  const int rc = fitoct_plan_get_info(pl->shards[0], info);
  if (rc) return rc;
  info->chains = pl->kp.chains;
  info->tiles = pl->tiles;
  info->draws_bytes = (int64_t)pl->draws_bytes;
  info->n_devices = (int32_t)pl->shards.size();
  return FITOCT_OK;
}

int group_plan_set_init(fitoct_plan* pl, const double* q, const double* eps, const double* minv) {
  const int D = pl->kp.D;
  for (const fitoct_plan* sh : pl->shards)
    if (sh->launched) return fail(FITOCT_E_ARG, "plan is running: call fitoct_plan_wait first");
  // every block is checked before any shard takes its part: a rejected value leaves the
  // whole plan as it was (no half warm-started plan)
  const int ck = check_init(pl->kp.chains, D, q, eps, minv);
  if (ck) return ck;
  DeviceRestore keep;
  for (size_t r = 0; r < pl->shards.size(); ++r) {
    const size_t o = (size_t)pl->shard_off[r];
    const int rc = fitoct_plan_set_init(pl->shards[r], q ? q + o * D : nullptr,
                                        eps ? eps + o : nullptr, minv ? minv + o * D : nullptr);
    if (rc) return rc;
  }
  return FITOCT_OK;
}

int group_plan_launch(fitoct_plan* pl, void* d_draws, void* stream) {
  if (stream)
    return fail(FITOCT_E_ARG, "a multi-device plan runs each device on a private stream of "
                              "the library: pass stream = NULL");
  for (const fitoct_plan* sh : pl->shards)
    if (sh->launched) return fail(FITOCT_E_ARG, "plan is running: call fitoct_plan_wait first");
  int gdev = -1;
  if (d_draws) {
    const int rc = buffer_device(d_draws, gdev);
    if (rc) return rc;
  }
  DeviceRestore keep;
  NullStreamFence fence;
  if (d_draws) {
    bool any_direct = false;
    for (const fitoct_plan* sh : pl->shards) {
      any_direct = any_direct || in_place(d_draws, sh->cfg.device, gdev);
      const int e = enable_peer(gdev, sh->cfg.device);
      if (e) return e;
    }
    if (any_direct) {
      const int e = fence.record(gdev);
      if (e) return e;
    }
  }
  for (size_t r = 0; r < pl->shards.size(); ++r) {
    fitoct_plan* sh = pl->shards[r];
    // a shard on the buffer's device writes its block in place (after the caller's NULL
    // stream work, the fence); the others are copied over xGMI once they finish
    // (group_plan_wait)
    const bool direct = in_place(d_draws, sh->cfg.device, gdev);
    void* dst = direct ? (char*)d_draws + chain_bytes(sh) * (size_t)pl->shard_off[r] : nullptr;
    int rc = FITOCT_OK;
    if (!sh->own_stream) rc = own_stream(sh->cfg.device, sh->own_stream);
    if (!rc && direct) rc = fence.order(sh->own_stream);
    if (!rc) rc = fitoct_plan_launch(sh, dst, sh->own_stream);
    if (rc) {   // stop what was launched before reporting
      const std::string msg = g_last_error;
      for (size_t k = 0; k < r; ++k) {
        (void)fitoct_plan_cancel(pl->shards[k]);
        (void)fitoct_plan_wait(pl->shards[k]);
      }
      return fail(rc, msg);
    }
  }
  pl->gather_dst = d_draws;
  pl->gather_dev = gdev;
  pl->launched = true;
  pl->ran = false;
  return FITOCT_OK;
}

int group_plan_poll(fitoct_plan* pl, int64_t* done, int64_t* total, int32_t* finished) {
  int64_t d = 0, t = 0;
  int32_t f = 1;
  DeviceRestore keep;
  for (fitoct_plan* sh : pl->shards) {
    int64_t ds = 0, ts = 0;
    int32_t fs = 0;
    const int rc = fitoct_plan_poll(sh, &ds, &ts, &fs);
    if (rc) return rc;
    d += ds;
    t += ts;
    f = f && fs;
  }
  if (done) *done = d;
  if (total) *total = t;
  if (finished) *finished = f;
  return FITOCT_OK;
}

int group_plan_cancel(fitoct_plan* pl) {
  for (fitoct_plan* sh : pl->shards) {
    const int rc = fitoct_plan_cancel(sh);
    if (rc) return rc;
  }
  return FITOCT_OK;
}

int group_plan_wait(fitoct_plan* pl) {
  if (!pl->launched) return pl->ran ? FITOCT_OK : fail(FITOCT_E_ARG, "plan has not been launched");
  pl->launched = false;
  const int n = (int)pl->shards.size();
  auto cancel_others = [&](int r) {
    for (int k = 0; k < n; ++k)
      if (k != r) (void)fitoct_plan_cancel(pl->shards[k]);
  };
  DeviceRestore keep;
  // every error return of a device's part (its wait, the status read, the peer copy of its
  // block) cancels the other devices: "a failure on one device cancels the others"
  auto part = [&](int r) -> int {
    fitoct_plan* sh = pl->shards[r];
    const int e = fitoct_plan_wait(sh);
    if (e) return e;
    // a failed chain (non-finite init, step-size search) fails the whole call: the other
    // devices' chains stop at their next transition boundary instead of running on
    std::vector<int> st(sh->kp.chains);
    HIP_TRY(hipMemcpy(st.data(), sh->kp.chain_status, sizeof(int) * st.size(),
                      hipMemcpyDeviceToHost));
    for (int s : st)
      if (s != 0 && s != FITOCT_E_CANCELLED) {
        cancel_others(r);
        break;
      }
    if (pl->gather_dst && sh->last_draws != (double*)((char*)pl->gather_dst +
                                                      chain_bytes(sh) * (size_t)pl->shard_off[r]))
      HIP_TRY(hipMemcpyPeer((char*)pl->gather_dst + chain_bytes(sh) * (size_t)pl->shard_off[r],
                            pl->gather_dev, sh->last_draws, sh->cfg.device, sh->draws_bytes));
    return FITOCT_OK;
  };
  const int rc = on_devices(n, [&](int r) -> int {
    const int e = part(r);
    if (e) cancel_others(r);
    return e;
  });
  pl->kernel_ms = 0.0;
  for (const fitoct_plan* sh : pl->shards) pl->kernel_ms = std::max(pl->kernel_ms, sh->kernel_ms);
  pl->ran = (rc == FITOCT_OK);
  return rc;
}

int group_plan_download(fitoct_plan* pl, fitoct_result* res) {
  if (!pl->ran) return fail(FITOCT_E_ARG, "plan has not run");
  const KParams& k = pl->kp;
  const int n = (int)pl->shards.size(), D = k.D;
  const int64_t per_chain = (int64_t)k.iters_saved * k.ncols;
  if (res->draws && res->draws_capacity < (int64_t)k.chains * per_chain)
    return fail(FITOCT_E_ARG, "draws buffer too small");
  std::vector<fitoct_result> sub(n);
  DeviceRestore keep;
  const int rc = on_devices(n, [&](int r) -> int {
    const size_t o = (size_t)pl->shard_off[r];
    fitoct_plan* sh = pl->shards[r];
    fitoct_result& s = sub[r];
    s = fitoct_result{};
    s.draws = res->draws ? res->draws + o * per_chain : nullptr;
    s.draws_capacity = (int64_t)sh->kp.chains * per_chain;
    s.stepsize = res->stepsize ? res->stepsize + o : nullptr;
    s.inv_metric = res->inv_metric ? res->inv_metric + o * D : nullptr;
    s.last_q = res->last_q ? res->last_q + o * D : nullptr;
    s.chain_status = res->chain_status ? res->chain_status + o : nullptr;
    return fitoct_plan_download(sh, &s);
  });
  res->n_cols = k.ncols;
  res->iters_saved = k.iters_saved;
  res->dim = D;
  res->kernel_ms = pl->kernel_ms;
  res->migrations = 0;
  res->total_leapfrogs = 0;
  res->two_ended_transitions = 0;
  res->paired_transitions = 0;
  for (const fitoct_result& s : sub) {
    res->migrations += s.migrations;
    res->total_leapfrogs += s.total_leapfrogs;
    res->two_ended_transitions += s.two_ended_transitions;
    res->paired_transitions += s.paired_transitions;
  }
  return rc;
}

int group_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                 const std::vector<int>& devs, fitoct_result* res) {
  fitoct_plan* pl = nullptr;
  int rc = group_plan_create(prob, cfg, devs, &pl);
  if (rc) return rc;
  rc = fitoct_plan_launch(pl, nullptr, nullptr);
  if (!rc) rc = fitoct_plan_wait(pl);
  if (!rc && res) rc = fitoct_plan_download(pl, res);
  const std::string msg = g_last_error;
  fitoct_plan_destroy(pl);
  return rc ? fail(rc, msg) : FITOCT_OK;
}

// ---- batches ----------------------------------------------------------------------
int group_batch_create(const fitoct_problem* probs, int n_problems, const fitoct_config* cfg,
                       const std::vector<int>& devs, fitoct_batch** out) {
  const int n = (int)devs.size(), C = cfg->chains;
  std::unique_ptr<fitoct_batch, void (*)(fitoct_batch*)> guard(new fitoct_batch(),
                                                               fitoct_batch_destroy);
  fitoct_batch* b = guard.get();
  b->cfg = *cfg;
  b->n_problems = n_problems;
  b->subs.assign(n, nullptr);
  b->sub_off.assign(n, 0);
  DeviceRestore keep;
  const int rc = on_devices(n, [&](int r) -> int {
    int off, cnt;
    block_range(n_problems, n, r, off, cnt);
    fitoct_config c = *cfg;
    c.chain_offset = cfg->chain_offset + off * C;   // problem p keeps global chains p*C + c
    c.device = devs[r];
    c.n_devices = 0;
    b->sub_off[r] = off;
    const int e = fitoct_batch_create(probs + off, cnt, &c, &b->subs[r]);
    return e ? fail(e, "device " + std::to_string(devs[r]) + ": " + g_last_error) : FITOCT_OK;
  });
  if (rc) return rc;
  b->per_bytes = b->subs[0]->per_bytes;
  for (const fitoct_batch* sb : b->subs) b->tiles += sb->tiles;
  *out = guard.release();
  return FITOCT_OK;
}

int group_batch_info(const fitoct_batch* b, fitoct_plan_info* info) {
  const int rc = fitoct_batch_get_info(b->subs[0], info);
  if (rc) return rc;
  info->chains = b->cfg.chains * b->n_problems;
  info->tiles = b->tiles;
  info->draws_bytes = (int64_t)(b->per_bytes * (size_t)b->n_problems);
  info->n_devices = (int32_t)b->subs.size();
  return FITOCT_OK;
}

int group_batch_run(fitoct_batch* b, void* d_draws, void* stream) {
  if (stream)
    return fail(FITOCT_E_ARG, "a multi-device batch runs each device on a private stream of "
                              "the library: pass stream = NULL");
  int gdev = -1;
  if (d_draws) {
    const int rc = buffer_device(d_draws, gdev);
    if (rc) return rc;
  }
  const int n = (int)b->subs.size();
  DeviceRestore keep;
  NullStreamFence fence;
  if (d_draws) {
    bool any_direct = false;
    for (const fitoct_batch* sb : b->subs) {
      any_direct = any_direct || in_place(d_draws, sb->cfg.device, gdev);
      const int e = enable_peer(gdev, sb->cfg.device);
      if (e) return e;
    }
    if (any_direct) {
      const int e = fence.record(gdev);
      if (e) return e;
    }
  }
  // every flag is cleared before any device starts, so a cancellation raised by an early
  // failure is never undone by a later device's start
  for (fitoct_batch* sb : b->subs) __atomic_store_n(sb->h_cancel, 0, __ATOMIC_SEQ_CST);
  auto cancel_others = [&](int r) {
    for (int k = 0; k < n; ++k)
      if (k != r) __atomic_store_n(b->subs[k]->h_cancel, 1, __ATOMIC_SEQ_CST);
  };
  // (every error return of a device's part cancels the other devices, the peer copy's too)
  auto part = [&](int r) -> int {
    fitoct_batch* sb = b->subs[r];
    char* slice = d_draws ? (char*)d_draws + b->per_bytes * (size_t)b->sub_off[r] : nullptr;
    const bool direct = in_place(d_draws, sb->cfg.device, gdev);
    if (!sb->own_stream) {
      const int e = own_stream(sb->cfg.device, sb->own_stream);
      if (e) return e;
    }
    if (direct) {
      const int e = fence.order(sb->own_stream);
      if (e) return e;
    }
    // FITOCT_TEST_FAIL_ENTRY=r (tests only): device entry r fails before its launch, so
    // one GPU can exercise the cancellation of the other entries (read on every call)
    const char* inject = getenv("FITOCT_TEST_FAIL_ENTRY");
    const int e = (inject && atoi(inject) == r)
                      ? fail(FITOCT_E_INTERNAL, "injected failure (FITOCT_TEST_FAIL_ENTRY)")
                      : batch_run_single(sb, direct ? slice : nullptr, sb->own_stream);
    if (e) return e;   // the call fails: the other devices' chains stop at their next checked boundary
    // A failed chain of one file (non-finite init, step-size search) is that file's status
    // at download, as in a one-device batch: files are independent fits (FitOCT.R:70-124)
    // and the other files, on this device or another, run on.
    if (d_draws && !direct)
      HIP_TRY(hipMemcpyPeer(slice, gdev, sb->d_draws, sb->cfg.device,
                            b->per_bytes * sb->plans.size()));
    return FITOCT_OK;
  };
  const int rc = on_devices(n, [&](int r) -> int {
    const int e = part(r);
    if (e) cancel_others(r);
    return e;
  });
  b->kernel_ms = 0.0;
  for (const fitoct_batch* sb : b->subs) b->kernel_ms = std::max(b->kernel_ms, sb->kernel_ms);
  b->ran = (rc == FITOCT_OK);
  return rc;
}

int group_batch_download(fitoct_batch* b, int problem, fitoct_result* res) {
  if (!b->ran) return fail(FITOCT_E_ARG, "batch has not run");
  for (size_t r = b->subs.size(); r-- > 0;)
    if (problem >= b->sub_off[r]) {
      DeviceRestore keep;
      return fitoct_batch_download(b->subs[r], problem - b->sub_off[r], res);
    }
  return fail(FITOCT_E_INTERNAL, "problem not found in any sub-batch");
}

}  // namespace fitoct
