// Error plumbing, version, small utility kernels.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

static thread_local char g_xa_err[512] = "";

void xa_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_xa_err, sizeof(g_xa_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* xa_last_error(void) { return g_xa_err; }
extern "C" int xa_abi_version(void) { return XA_ABI_VERSION; }

extern "C" int xa_mlp_param_count(int obs_dim, int n_actions) {
  const int H = XA_MLP_HIDDEN;
  return obs_dim * H + H + H * H + H + H * n_actions + n_actions + H + 1;
}

__global__ void counter_bump_kernel(uint64_t* c) { c[0] += 1; }

extern "C" int xa_counter_bump(uint64_t* counter, void* stream) {
  XA_CHECK_ARG(counter != nullptr, "xa_counter_bump: null counter");
  hipLaunchKernelGGL(counter_bump_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  XA_CHECK_LAUNCH("xa_counter_bump");
  return 0;
}
