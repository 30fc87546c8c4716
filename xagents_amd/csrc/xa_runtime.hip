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

// the SHA-256 prefix of the sources this library was built from (xagents_amd/_build.py
// passes it; the marker lets the loader find it in the file without loading it)
#ifndef XA_BUILD_HASH
#define XA_BUILD_HASH "unknown"
#endif
static const char kXaBuildHash[] = "XA_BUILD_HASH:" XA_BUILD_HASH;
extern "C" const char* xa_build_hash(void) { return kXaBuildHash + 14; }

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
