// Internal declarations shared by the host translation units of libfitoct.
#pragma once
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "fitoct.h"

namespace fitoct {

extern thread_local std::string g_last_error;
int fail(int code, const std::string& msg);

int build_basis(const fitoct_problem* p, std::vector<double>& B, std::vector<double>& xg);
int model_dim(int prior, int Nn);
std::string column_name(int prior, int Nn, int i);
int split_rhat_ess(const double* x, int chains, int n, double* rhat, double* ess);
int rank_rhat(const double* x, int chains, int n, double* out);
bool log_transformed(int prior, int Nn, int j);
void constrain(int prior, int Nn, const double* q, double* out);
double lp_constant(const fitoct_problem* p);
// A run's per-chain outcome (fitoct_plan_download): every chain whose status is
// FITOCT_E_TIMEOUT gets NaN warm-restart outputs (stepsize, inverse metric, last q; any of
// them may be NULL); returns the chain whose status the call reports -- the first chain's
// own failure, before any FITOCT_E_CANCELLED it caused -- or -1 when every chain is 0.
int chain_outcome(int C, int D, const int* status, double* stepsize, double* inv_metric,
                  double* last_q);

// Every extern "C" entry that can allocate runs its body through guarded(): no C++
// exception crosses the ABI (include/fitoct.h); a failure becomes a status + message.
template <class F>
int guarded(const char* fn, F&& body) noexcept {
  try {
    return body();
  } catch (const std::bad_alloc&) {
    return fail(FITOCT_E_INTERNAL, std::string(fn) + ": out of host memory");
  } catch (const std::exception& e) {
    return fail(FITOCT_E_INTERNAL, std::string(fn) + ": " + e.what());
  } catch (...) {
    return fail(FITOCT_E_INTERNAL, std::string(fn) + ": unknown exception");
  }
}

}  // namespace fitoct
