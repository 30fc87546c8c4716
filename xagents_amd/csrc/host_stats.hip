// Episode statistics to pinned host memory in one small launch.
//
// After every on-policy train step the host folds the rollout's done flags and running
// episode returns into total_rewards / games (the reference's step_envs bookkeeping,
// xagents/base.py:388-426). At small env counts the three D2H DMA copies that carried them
// (done [N][T+1], returns [N][T], the persistent update's status word) cost ~4.6 us of
// stream time each, mostly fixed DMA setup; one 256-thread kernel storing the same words
// straight into the mapped pinned host buffers costs one short launch. Stores are plain
// vector stores; the launch's end-of-kernel release makes them visible to the host event.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

#include <algorithm>

namespace {

__global__ __launch_bounds__(256) void host_copy_kernel(XaHostCopyArgs a) {
  for (int s = 0; s < a.n_segments; ++s) {
    const uint32_t* __restrict__ src = static_cast<const uint32_t*>(a.src[s]);
    uint32_t* __restrict__ dst = static_cast<uint32_t*>(a.dst[s]);
    const int64_t words = a.bytes[s] / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < words;
         i += (int64_t)gridDim.x * blockDim.x)
      dst[i] = src[i];
  }
}

}  // namespace

extern "C" int xa_host_device_pointer(void* host, void** dev) {
  XA_CHECK_ARG(host != nullptr && dev != nullptr, "xa_host_device_pointer: null pointer");
  const hipError_t e = hipHostGetDevicePointer(dev, host, 0);
  XA_CHECK_ARG(e == hipSuccess, "xa_host_device_pointer: %s (not pinned host memory?)",
               hipGetErrorString(e));
  return 0;
}

extern "C" int xa_copy_to_host(const XaHostCopyArgs* a, void* stream) {
  XA_CHECK_ARG(a != nullptr, "xa_copy_to_host: null args");
  XA_CHECK_ARG(a->n_segments >= 1 && a->n_segments <= XA_HOST_COPY_MAX,
               "xa_copy_to_host: n_segments must be in [1, %d]", XA_HOST_COPY_MAX);
  int64_t total = 0;
  for (int s = 0; s < a->n_segments; ++s) {
    XA_CHECK_ARG(a->src[s] && a->dst[s], "xa_copy_to_host: null segment %d", s);
    XA_CHECK_ARG(a->bytes[s] >= 0 && a->bytes[s] % 4 == 0,
                 "xa_copy_to_host: segment %d bytes must be a non-negative multiple of 4", s);
    XA_CHECK_ARG(((uintptr_t)a->src[s] | (uintptr_t)a->dst[s]) % 4 == 0,
                 "xa_copy_to_host: segment %d not 4-byte aligned", s);
    total += a->bytes[s];
  }
  const int64_t words = total / 4;
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>((words + 4095) / 4096, 1), 64);
  hipLaunchKernelGGL(host_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *a);
  XA_CHECK_LAUNCH("xa_copy_to_host");
  return 0;
}
