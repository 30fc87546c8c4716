// One-shot peer all-reduce for the small per-minibatch exchanges of the data-parallel
// update (one all_reduce(SUM) of the flat gradient per optimizer step,
// ppo/agent.py:136-137 applied to the union of the ranks' minibatches, plus the
// advantage sums of ppo/agent.py:180-183).
//
// Why not RCCL for these: the MLP gradient is 18.7 KB and the advantage sums 2 KB, so
// a ring over xGMI is pure latency (2(W-1) dependent hops). Here every rank PUSHES its
// values straight into every peer's IPC-mapped, uncached HBM block as 8-byte
// (value word, epoch) pairs -- one system-coherent 64-bit store per word and peer over
// the point-to-point xGMI links -- and then polls its OWN block until all W pairs of a
// word carry the current epoch. An aligned 8-byte store lands whole, so a matching
// epoch proves the value next to it is the current one: no separate flag, no fence,
// one link latency per exchange (the "LL" idea of NCCL's low-latency protocol, sized
// here for gradients of a few KB). Each rank then sums the W values in rank order
// 0..W-1, so every rank gets identical bits.
//
// Block layout (one per rank and channel, hipDeviceMallocUncached, IPC-exported):
//   [0, 256)   unused header
//   then pairs[2][W][slot_words] of u64 = (word | epoch << 32); epoch e uses parity e & 1
// Per-rank state (ordinary device memory, only this rank touches it):
//   state[0] = sticky error (0 healthy, 1 + p = timed out waiting for rank p)
//   state[1 + c] = epoch counter of word chunk c (kChunkWords words per workgroup)
// Parity reuse is safe: rank q rewrites chunk c at parity (e & 1) only at epoch e + 2,
// which needs this rank's epoch-(e + 1) pairs for chunk c, which this rank pushes only
// after its epoch-e kernel (and its reads of chunk c) finished on its stream.
//
// With has_tail, the last workgroup to finish applies clip + Keras Adam to the summed
// gradient (xa_adam.hpp, same arithmetic as xa_clip_adam), so a data-parallel optimizer
// step costs no launch beyond the exchange itself.
//
// Every wait is bounded (s_memrealtime, 100 MHz): on timeout the kernel records the
// sticky error and returns the local values; later calls see the error and skip the
// exchange, so a broken peer path can never hang the GPU. The host reads the error and
// falls back to RCCL (xagents_amd/comm.py).
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/xagents_hip.h"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

constexpr int kHdr = 256;
constexpr int kThreads = 256;
constexpr int kWordsPerThread = 4;  // 16 B of payload per thread
constexpr int kChunkWords = kThreads * kWordsPerThread;

XA_DEV void st_pair(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
XA_DEV uint64_t ld_pair(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
XA_DEV T word_value(const uint32_t* w);
template <>
XA_DEV float word_value<float>(const uint32_t* w) {
  return __uint_as_float(w[0]);
}
template <>
XA_DEV double word_value<double>(const uint32_t* w) {
  return __hiloint2double((int)w[1], (int)w[0]);
}

// W > 0: compile-time world (all loads of a poll issued together); W == 0: runtime world
template <typename T, int W>
__global__ __launch_bounds__(kThreads) void peer_allreduce_kernel(XaPeerAllReduceArgs a) {
  constexpr int kEW = sizeof(T) / 4;                  // words per element
  constexpr int kMaxW = W > 0 ? W : XA_PEER_MAX;
  const int world = W > 0 ? W : a.world;
  const int chunk = blockIdx.x;
  uint32_t* state = a.state;
  const uint32_t ep = state[1 + chunk] + 1u;
  const bool skip = state[0] != 0u;
  const long n_words = a.count * kEW;
  const long w0 = (long)chunk * kChunkWords + (long)threadIdx.x * kWordsPerThread;
  const long slot_words = (long)(a.slot_bytes / 4);
  const uint32_t* src = (const uint32_t*)a.src;
  uint32_t* dst = (uint32_t*)a.dst;

  uint32_t mine[kWordsPerThread];
#pragma unroll
  for (int k = 0; k < kWordsPerThread; ++k) mine[k] = w0 + k < n_words ? src[w0 + k] : 0u;
  const size_t par_off = (size_t)(ep & 1u) * world * slot_words;

  uint32_t got[kMaxW][kWordsPerThread];
  bool ok = !skip;
  if (ok && w0 < n_words) {
    // push: one 8-byte (word, epoch) store per word and peer, own block included
    for (int p = 0; p < world; ++p) {
      uint64_t* dstp = (uint64_t*)((uint8_t*)a.blocks[p] + kHdr) + par_off +
                       (size_t)a.rank * slot_words + w0;
#pragma unroll
      for (int k = 0; k < kWordsPerThread; ++k)
        if (w0 + k < n_words) st_pair(dstp + k, (uint64_t)mine[k] | ((uint64_t)ep << 32));
    }
    // poll the own block until every rank's pairs of these words carry epoch ep
    const uint64_t* base = (const uint64_t*)((const uint8_t*)a.blocks[a.rank] + kHdr) + par_off + w0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      bool ready = true;
      int late = 0;
#pragma unroll
      for (int p = 0; p < kMaxW; ++p) {
        if (W == 0 && p >= world) break;
#pragma unroll
        for (int k = 0; k < kWordsPerThread; ++k) {
          const uint64_t v = w0 + k < n_words ? ld_pair(base + (size_t)p * slot_words + k)
                                              : ((uint64_t)ep << 32);
          got[p][k] = (uint32_t)v;
          if ((uint32_t)(v >> 32) != ep) {
            ready = false;
            late = p;
          }
        }
      }
      if (ready) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        __hip_atomic_store(&state[0], 1u + (uint32_t)late, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // rank-ordered sum (identical bits on every rank); local values after a failure
  if (w0 < n_words) {
    if (ok) {
#pragma unroll
      for (int k = 0; k < kWordsPerThread; k += kEW) {
        T acc = word_value<T>(&got[0][k]);
        for (int p = 1; p < world; ++p) acc += word_value<T>(&got[p][k]);
        uint32_t out[kEW];
        memcpy(out, &acc, sizeof(T));
#pragma unroll
        for (int e = 0; e < kEW; ++e)
          if (w0 + k + e < n_words) dst[w0 + k + e] = out[e];
      }
    } else {
#pragma unroll
      for (int k = 0; k < kWordsPerThread; ++k)
        if (w0 + k < n_words) dst[w0 + k] = mine[k];
    }
  }
  __syncthreads();  // every thread has read state[1 + chunk]
  if (threadIdx.x == 0) state[1 + chunk] = ep;
  // optimizer tail on the summed gradient (f32 only; checked on the host)
  if constexpr (sizeof(T) == 4) {
    if (a.has_tail && last_block_arrived(a.tail.arrivals))
      adam_tail_apply(a.tail, (const float*)a.dst, (int)a.count);
  }
}

template <typename T>
void launch_peer(const XaPeerAllReduceArgs& a, int chunks, hipStream_t s) {
  switch (a.world) {
#define XA_PEER_CASE(w)                                                                  \
  case w:                                                                                \
    hipLaunchKernelGGL((peer_allreduce_kernel<T, w>), dim3(chunks), dim3(kThreads), 0, s, a); \
    return;
    XA_PEER_CASE(1) XA_PEER_CASE(2) XA_PEER_CASE(3) XA_PEER_CASE(4)
    XA_PEER_CASE(5) XA_PEER_CASE(6) XA_PEER_CASE(7) XA_PEER_CASE(8)
#undef XA_PEER_CASE
    default:
      hipLaunchKernelGGL((peer_allreduce_kernel<T, 0>), dim3(chunks), dim3(kThreads), 0, s, a);
  }
}

}  // namespace

extern "C" size_t xa_peer_block_bytes(size_t slot_bytes, int world) {
  const size_t words = (slot_bytes + kChunkWords * 4 - 1) / (kChunkWords * 4) * kChunkWords;
  return (size_t)kHdr + 2 * (size_t)world * words * 8;
}

extern "C" int xa_peer_state_words(size_t slot_bytes) {
  return 1 + (int)((slot_bytes + kChunkWords * 4 - 1) / (kChunkWords * 4));
}

extern "C" int xa_peer_block_alloc(size_t bytes, void** block) {
  XA_CHECK_ARG(block != nullptr && bytes >= (size_t)kHdr, "xa_peer_block_alloc: bad arguments");
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    xa_set_error("xa_peer_block_alloc: hipExtMallocWithFlags(uncached, %zu): %s", bytes,
                 hipGetErrorString(e));
    return -4;
  }
  e = hipMemset(p, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(p);
    xa_set_error("xa_peer_block_alloc: hipMemset: %s", hipGetErrorString(e));
    return -4;
  }
  *block = p;
  return 0;
}

extern "C" int xa_peer_block_free(void* block) {
  if (block == nullptr) return 0;
  hipError_t e = hipFree(block);
  if (e != hipSuccess) {
    xa_set_error("xa_peer_block_free: %s", hipGetErrorString(e));
    return -4;
  }
  return 0;
}

extern "C" int xa_peer_ipc_handle(void* block, void* handle_out) {
  XA_CHECK_ARG(block && handle_out, "xa_peer_ipc_handle: null pointer");
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, block);
  if (e != hipSuccess) {
    xa_set_error("xa_peer_ipc_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    return -4;
  }
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

extern "C" int xa_peer_ipc_open(const void* handle, void** block) {
  XA_CHECK_ARG(handle && block, "xa_peer_ipc_open: null pointer");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    xa_set_error("xa_peer_ipc_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    return -4;
  }
  *block = p;
  return 0;
}

extern "C" int xa_peer_ipc_close(void* block) {
  if (block == nullptr) return 0;
  hipError_t e = hipIpcCloseMemHandle(block);
  if (e != hipSuccess) {
    xa_set_error("xa_peer_ipc_close: %s", hipGetErrorString(e));
    return -4;
  }
  return 0;
}

extern "C" int xa_peer_allreduce(const XaPeerAllReduceArgs* a, void* stream) {
  XA_CHECK_ARG(a && a->src && a->dst && a->state, "xa_peer_allreduce: null pointer");
  XA_CHECK_ARG(a->world >= 1 && a->world <= XA_PEER_MAX && a->rank >= 0 && a->rank < a->world,
               "xa_peer_allreduce: bad rank %d / world %d", a->rank, a->world);
  XA_CHECK_ARG(a->dtype == XA_DTYPE_F32 || a->dtype == XA_DTYPE_F64,
               "xa_peer_allreduce: dtype must be f32 or f64");
  const size_t esz = a->dtype == XA_DTYPE_F64 ? 8 : 4;
  XA_CHECK_ARG(a->slot_bytes % (kChunkWords * 4) == 0,
               "xa_peer_allreduce: slot_bytes must be a multiple of %d", kChunkWords * 4);
  XA_CHECK_ARG(a->count >= 0 && (size_t)a->count * esz <= a->slot_bytes,
               "xa_peer_allreduce: %lld elements do not fit a %zu-byte slot",
               (long long)a->count, a->slot_bytes);
  for (int p = 0; p < a->world; ++p)
    XA_CHECK_ARG(a->blocks[p] != nullptr && ((uintptr_t)a->blocks[p] & 255) == 0,
                 "xa_peer_allreduce: block of rank %d missing or not 256-byte aligned", p);
  XA_CHECK_ARG(((uintptr_t)a->src & 7) == 0 && ((uintptr_t)a->dst & 7) == 0,
               "xa_peer_allreduce: src/dst must be 8-byte aligned");
  if (a->has_tail)
    XA_CHECK_ARG(a->dtype == XA_DTYPE_F32 && a->count <= XA_ADAM_TAIL_MAX_PARAMS &&
                     a->tail.theta && a->tail.m && a->tail.v && a->tail.adam_step &&
                     a->tail.arrivals,
                 "xa_peer_allreduce: an optimizer tail needs f32, <= %d elements, theta, m, v, "
                 "adam_step and arrivals", XA_ADAM_TAIL_MAX_PARAMS);
  if (a->count == 0) return 0;
  const long words = a->count * (long)(esz / 4);
  const int chunks = (int)((words + kChunkWords - 1) / kChunkWords);
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == XA_DTYPE_F64) launch_peer<double>(*a, chunks, s);
  else launch_peer<float>(*a, chunks, s);
  XA_CHECK_LAUNCH("xa_peer_allreduce");
  return 0;
}
