// Plan and batch objects behind the opaque handles of include/fitoct.h, shared by the
// single-device entry points (fitoct_api.cpp) and the multi-device layer
// (multi_device.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "fitoct.h"
#include "host_internal.h"
#include "kernel_params.h"

struct fitoct_plan {
  fitoct_problem prob{};
  fitoct_config cfg{};
  fitoct::KParams kp{};
  int tiles = 0, bpt = 0, nnp = 15, ppl = 1, lds = 0, ncu = 0;
  bool mixed = false;
  int* d_mig = nullptr;       // chain-migration control block (see MigCtrl)
  double* d_mig_img = nullptr;
  size_t mig_bytes = 0;
  size_t draws_bytes = 0;
  void* d_data = nullptr;     // cx | y | isu | B  (type R)
  double* d_draws = nullptr;  // internal draws buffer (lazily allocated)
  double* d_stack = nullptr;
  double* d_fin = nullptr;    // eps[C] | minv[C*D] | q[C*D]
  double* d_init = nullptr;   // warm restart (fitoct_plan_set_init): eps[C] | minv[C*D] | q[C*D]
  int* d_status = nullptr;
  long long* d_leap = nullptr;
  fitoct::KParams* d_kp = nullptr;    // device copy of the launch parameters
  double* last_draws = nullptr;
  double kernel_ms = 0.0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool ran = false;
  bool launched = false;      // fitoct_plan_launch issued, fitoct_plan_wait not yet
  int* h_prog = nullptr;      // host-pinned [chains]: transitions done (kernel-written)
  int* h_cancel = nullptr;    // host-pinned flag polled by the kernel
  long long* d_stamps = nullptr;   // diagnostic stamps of the launch in flight
  int* d_pair_hdr = nullptr;       // paired tiles (KParams::pair): hand-off words
  double* d_pair_buf = nullptr;    // ... starts and rings
  // blocks of the launch: the tiles, or with paired tiles a primary and a partner each
  int grid() const { return kp.pair ? fitoct::pair_grid(tiles) : tiles; }

  // ---- multi-device plan (cfg.n_devices > 1; multi_device.cpp) ----
  // One single-device plan per device; shard r runs this plan's chains
  // [shard_off[r], shard_off[r] + shards[r]->kp.chains).  A multi-device plan holds no
  // device memory of its own: every entry point forwards to its shards.
  std::vector<fitoct_plan*> shards;
  std::vector<int> shard_off;
  void* gather_dst = nullptr;  // caller's d_draws of the launch in flight (or NULL)
  int gather_dev = -1;         // device holding gather_dst
  // a shard's own non-blocking stream: shards never wait on one another (nor on the
  // synchronous status reads and peer copies of other shards) through a default stream
  hipStream_t own_stream = nullptr;
};

struct fitoct_batch {
  std::vector<fitoct_plan*> plans;
  fitoct_config cfg{};
  int tiles = 0;
  size_t per_bytes = 0;       // draws bytes of one problem
  fitoct::KParams* d_kp = nullptr;    // [n_problems]
  int* d_map = nullptr;       // [tiles][2]
  double* d_draws = nullptr;  // internal [n_problems][chains][iters][cols] (lazy)
  double kernel_ms = 0.0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool ran = false;
  // host-pinned flag polled by every problem's chains (KParams::cancel): set by the
  // multi-device layer when another device's chain failed; cleared by each run
  int* h_cancel = nullptr;
  int* d_cancel = nullptr;    // its device alias
  int* d_pair_hdr = nullptr;  // paired tiles (every problem's KParams::pair_*)
  double* d_pair_buf = nullptr;
  int pair_stride = 0;

  // ---- multi-device batch: problems [sub_off[r], sub_off[r] + subs[r]->plans.size())
  // on sub-batch r, one device each (multi_device.cpp) ----
  std::vector<fitoct_batch*> subs;
  std::vector<int> sub_off;
  int n_problems = 0;
  hipStream_t own_stream = nullptr;   // a sub-batch's own non-blocking stream
};

namespace fitoct {

// the device list of a call: ordinals of the first min(n_devices, units) entries of
// cfg->devices (or {cfg->device} when n_devices == 0); FITOCT_E_ARG on a bad list
int resolve_devices(const fitoct_config* cfg, int units, std::vector<int>& devs);
// contiguous block partition of `total` units over `n` parts (part r: [off, off + cnt))
void block_range(int total, int n, int r, int& off, int& cnt);

// multi-device forms of the plan / batch entry points (multi_device.cpp)
int group_plan_create(const fitoct_problem* prob, const fitoct_config* cfg,
                      const std::vector<int>& devs, fitoct_plan** out);
int group_plan_info(const fitoct_plan* pl, fitoct_plan_info* info);
int group_plan_set_init(fitoct_plan* pl, const double* q, const double* eps, const double* minv);
int group_plan_launch(fitoct_plan* pl, void* d_draws, void* stream);
int group_plan_poll(fitoct_plan* pl, int64_t* done, int64_t* total, int32_t* finished);
int group_plan_cancel(fitoct_plan* pl);
int group_plan_wait(fitoct_plan* pl);
int group_plan_download(fitoct_plan* pl, fitoct_result* res);
int group_sample(const fitoct_problem* prob, const fitoct_config* cfg,
                 const std::vector<int>& devs, fitoct_result* res);

int group_batch_create(const fitoct_problem* probs, int n_problems, const fitoct_config* cfg,
                       const std::vector<int>& devs, fitoct_batch** out);
int group_batch_info(const fitoct_batch* b, fitoct_plan_info* info);
int group_batch_run(fitoct_batch* b, void* d_draws, void* stream);
// a single-device batch's run (fitoct_batch_run without clearing the cancel flag)
int batch_run_single(fitoct_batch* b, void* d_draws, void* stream);
// warm-restart inputs of C chains checked on the host (fitoct_plan_set_init's rules)
int check_init(int C, int D, const double* q, const double* eps, const double* minv);
int group_batch_download(fitoct_batch* b, int problem, fitoct_result* res);

}  // namespace fitoct
