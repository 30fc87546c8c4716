// Persistent PPO update kernel (the C-ABI entry points: ppo_update.hip): every optimizer step
// of one train step -- E epochs x M
// minibatches of shuffle, per-minibatch advantage normalisation, forward, clipped loss,
// backward, tf.clip_by_global_norm and Keras Adam -- in ONE launch.
// Replaces PPO.get_mini_batches + run_ppo_epochs + update_gradients
// (xagents/ppo/agent.py:96-191); same arithmetic as the per-minibatch chain
// (xa_ppo_minibatches -> E*M x [xa_ac_grad -> xa_grad_reduce] -> xa_clip_adam), minus
// its 2 E*M + 2 launches and its partial-row round trips through separate kernels.
//
// G resident workgroups (one per CU, G = min(32-sample tiles per minibatch, resident
// capacity)); workgroup b owns tiles b, b + G, ... of every minibatch.
//   phase 0   advantage sums of every (minibatch, workgroup) -> hop -> per-minibatch
//             mean / population std in LDS (ppo/agent.py:180-183)
//   per minibatch k:
//     A  forward + loss + backward of the block's tiles (ppo_tile.hpp) -> the block's
//        gradient row [P] -> hop
//     B  block b reduces parameters [b PB, (b+1) PB) over the G rows in a fixed order
//        (f64) -> g slice -> hop
//     C  every block: global norm from its own copy of g (fixed order, identical in every
//        block), clip + Keras Adam with t = t0 + k + 1 on its register-resident slice
//        of theta / m / v (ppo_tile.hpp PSlice), refresh the LDS weight tiles
//   block 0 stores theta / m / v and the Adam step count at the end.
// Data parallel (dp_world = W > 1, the DP template variant): phase 0's per-minibatch
// advantage totals and, in every step, each block's phase-B slice are pushed to every
// rank's IPC-mapped exchange block and summed in rank order from the own block (system-
// scope 8-byte {word, tag} pairs, the xa_peer_allreduce protocol) -- so every rank applies
// the optimizer step of the union of the ranks' minibatches with one cross-GPU hop per step
// and no launch or collective outside the kernel.
// Hand-offs follow the write-through protocol (cdna_hip_programming.md Guideline 16,
// MI355X_MICROARCH.md visibility table row 1): handed-off words are stored write-through
// (sc1) and loaded with sc1 loads. Every hop is data-as-flag: the handed-off values carry a
// tag (granules, or the tag's parity in each value's lowest mantissa bit: tagged pairs,
// below) and consumers poll the data itself.
// Nothing is reset between launches (no memset node in front of the kernel): the launch
// generation `gen` in the workspace numbers the launches, granule tags are unique per
// (launch, step), and the abort word holds the number of the launch that aborted. Spins are
// bounded (wall clock); a timeout raises the abort word and `status` (after which the
// workspace must be re-zeroed), and every block leaves.
#pragma once
#include <math.h>
#include <stdlib.h>

#include "../../include/xagents_hip.h"
#include "ppo_tile.hpp"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

using namespace xa_ac;
using namespace xa_pt;

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int kMaxSteps = 128;              // E * M optimizer steps per launch (xagents: 16)
constexpr int kCtlBytes = 256;              // control words at the workspace start
// 10 s of the 100 MHz wall clock per hop: data parallel, a hop also absorbs the other ranks'
// host-side skew (one process per GPU)
constexpr uint64_t kSpinTicks = 1000000000;
constexpr int kXcds = 8;            // MI355X: 8 XCDs, each with its own L2
// control words: the phase-0 arrival counter ((gen + 1) G after launch gen) and the abort
// word (the number gen + 1 of a launch that timed out), never reset; the XCD election of
// the XCD-local mode (below) in two parity slots -- launch gen uses slot gen & 1, which
// launch gen - 1 (of either mode) zeroed at its end
enum { kCntStats = 0, kAbort = 1, kWin = 2 /* [2] */, kElect = 4 /* [2][kXcds] */ };
#ifndef XA_TWO_LEVEL_MIN_G  // (diagnostic A/B builds override it)
#define XA_TWO_LEVEL_MIN_G 64
#endif
constexpr int kTwoLevelMinG = XA_TWO_LEVEL_MIN_G;  // >= 8 blocks per XCD: reduce inside each XCD's L2 first


// ---- write-through hand-off primitives (global address space, agent scope) ----
XA_DEV void st_wt(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
XA_DEV void st_wt(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
XA_DEV float ld_wt(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XA_DEV double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int kRsrcWord3 = 0x00020000;  // raw buffer, gfx9-family resource word 3
constexpr int kAuxSc1 = 16;             // buffer instruction aux bits: write-through (sc1)

XA_DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, kRsrcWord3);
}
XA_DEV void st_wt4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(f32x4v{v.x, v.y, v.z, v.w}, r, byte_off, 0, kAuxSc1);
}
XA_DEV float4 ld_wt4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAuxSc1);
  return make_float4(v[0], v[1], v[2], v[3]);
}
// two f64 in one 16-B write-through access
XA_DEV void st_wt_d2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, double a, double b) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4v, make_double2(a, b)), r,
                                         byte_off, 0, kAuxSc1);
}
XA_DEV double2 ld_wt_d2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAuxSc1));
}
// {v0, tag} {v1, tag} as one 16-byte store, write-through (cross-XCD readers) or plain
// (readers on this XCD: the line stays in the shared L2)
XA_DEV void st_gran2(__amdgpu_buffer_rsrc_t r, uint32_t off, float v0, float v1, unsigned tag,
                     bool wt) {
  const f32x4v v = {v0, __uint_as_float(tag), v1, __uint_as_float(tag)};
  if (wt) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSc1);
  else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
XA_DEV void st_gran_f64(__amdgpu_buffer_rsrc_t r, uint32_t off, double d, unsigned tag,
                        bool wt = true) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  st_gran2(r, off, __uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32)), tag, wt);
}
XA_DEV bool gran_ok(const f32x4v& v, unsigned tag) {
  return __float_as_uint(v[1]) == tag && __float_as_uint(v[3]) == tag;
}
XA_DEV double gran_f64(const f32x4v& v) {
  return __longlong_as_double((long long)(((unsigned long long)__float_as_uint(v[2]) << 32) |
                                          __float_as_uint(v[0])));
}

// The blocks' gradient rows (the bulk of the in-launch exchange) as TAGGED PAIRS: 8 bytes
// per two values, the step's tag parity in each value's lowest mantissa bit (the value moves
// by at most one ulp, 6e-8 relative; the update is checked against float64 with a
// tolerance). Parity suffices: a row word is rewritten every step, tags are consecutive
// integers (gen K + k + 1) across launches, a kernel boundary writes the previous launch's
// words back, and a reader that has seen step k - 1's value at an address never sees an
// older one there (per-address coherence of one L2 / the fabric). Every 4-byte word carries
// its own tag, so no store width has to be untorn. Half the bytes of the {value, tag}
// granule pairs (XA_ROW_PAIRS=0: those, the round-5 format).
#ifndef XA_ROW_PAIRS
#define XA_ROW_PAIRS 1
#endif
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
#if XA_ROW_PAIRS
typedef f32x2v RowG;
constexpr uint32_t kRowPB = 8;  // bytes per pair column of a row
XA_DEV float row_tagged(float v, unsigned tag) {
  return __uint_as_float((__float_as_uint(v) & ~1u) | (tag & 1u));
}
XA_DEV void st_row(__amdgpu_buffer_rsrc_t r, uint32_t off, float v0, float v1, unsigned tag,
                   bool wt) {
  const u32x2v u = {__float_as_uint(row_tagged(v0, tag)), __float_as_uint(row_tagged(v1, tag))};
  if (wt) __builtin_amdgcn_raw_buffer_store_b64(u, r, off, 0, kAuxSc1);
  else __builtin_amdgcn_raw_buffer_store_b64(u, r, off, 0, 0);
}
XA_DEV RowG ld_row(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x2v, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSc1));
}
// one tagged word of a row (byte offset off): every word carries its own tag parity, so a
// pair's two words may come from two stores
XA_DEV void st_row1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v, unsigned tag, bool wt) {
  const unsigned u = __float_as_uint(row_tagged(v, tag));
  if (wt) __builtin_amdgcn_raw_buffer_store_b32(u, r, off, 0, kAuxSc1);
  else __builtin_amdgcn_raw_buffer_store_b32(u, r, off, 0, 0);
}
XA_DEV bool row_ok(const RowG& v, unsigned tag) {
  return ((__float_as_uint(v[0]) ^ tag) & 1u) == 0u && ((__float_as_uint(v[1]) ^ tag) & 1u) == 0u;
}
XA_DEV float row_v0(const RowG& v) { return v[0]; }
XA_DEV float row_v1(const RowG& v) { return v[1]; }
#else
typedef f32x4v RowG;
constexpr uint32_t kRowPB = 16;
XA_DEV void st_row(__amdgpu_buffer_rsrc_t r, uint32_t off, float v0, float v1, unsigned tag,
                   bool wt) {
  st_gran2(r, off, v0, v1, tag, wt);
}
XA_DEV RowG ld_row(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1);
}
XA_DEV bool row_ok(const RowG& v, unsigned tag) { return gran_ok(v, tag); }
XA_DEV float row_v0(const RowG& v) { return v[0]; }
XA_DEV float row_v1(const RowG& v) { return v[2]; }
#endif
#if !XA_ROW_PAIRS
#error "the reduced gradient and the XCD partials travel as tagged pairs (XA_ROW_PAIRS)"
#endif

// Two f64 in one 16-B access, each carrying the step's tag parity in its lowest mantissa
// bit (moves a value by at most one f64 ulp): the per-XCD partial sums of the two-level
// reduce, half the bytes of two {lo, tag} {hi, tag} granule pairs. Each f64 is one
// naturally aligned 8-B half (untorn), so each carries its own tag.
XA_DEV double d_tagged(double d, unsigned tag) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return __longlong_as_double((long long)((u & ~1ull) | (unsigned long long)(tag & 1u)));
}
XA_DEV void st_d2_tagged(__amdgpu_buffer_rsrc_t r, uint32_t off, double a, double b, unsigned tag) {
  st_wt_d2(r, off, d_tagged(a, tag), d_tagged(b, tag));
}
XA_DEV bool d2_ok(const double2& v, unsigned tag) {
  return ((((unsigned)__double_as_longlong(v.x)) ^ tag) & 1u) == 0u &&
         ((((unsigned)__double_as_longlong(v.y)) ^ tag) & 1u) == 0u;
}

// Poll n (<= N) granule pairs (write-through loads) until every tag equals `tag`. Bounded
// by the wall clock and the abort word; false on timeout / abort (the caller leaves).
// One poll round is ONE L2 round trip: the abort word and the wall clock are read only
// every 16th round (the abort word then travels in the same batch of loads as the
// granules, not behind them; read every round from every wave it would pile the whole
// grid's polls onto one L2 channel), so a granule that lands just after a round was
// issued is seen one round trip later.
// (measurement knob) s_sleep units (64 cycles) between poll rounds
// every block forms the global gradient norm from its own copy of the reduced g (phase C:
// each parameter sits on exactly one thread, f64 squares summed in a fixed thread / wave
// order, identical in every block) -- no published sum-of-squares partials, phase C polls
// only g (16-env update 145 -> 141 us, C2 267 -> 257 us event-timed vs the round-5 form,
// profiles/r06d_variants_ab.txt)
#ifndef XA_POLL_SLEEP
#define XA_POLL_SLEEP 1
#endif
template <int N>
XA_DEV bool poll_gran(__amdgpu_buffer_rsrc_t r, const uint32_t (&off)[N], int n, unsigned tag,
                      f32x4v (&v)[N], unsigned* ctl, unsigned epoch, int* status) {
  uint64_t t0 = 0;
  for (unsigned it = 0;; ++it) {
    const bool slow = (it & 15u) == 15u;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < n) v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, off[u], 0, kAuxSc1);
    const unsigned ab = slow ? __hip_atomic_load((gu32*)(ctl + kAbort), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0u;
    bool ok = true;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < n) ok = ok && gran_ok(v[u], tag);
    if (ok) return true;
    if (!slow) {
#ifndef XA_POLL_NOSLEEP
      __builtin_amdgcn_s_sleep(XA_POLL_SLEEP);
#endif
      continue;
    }
    if (ab == epoch) return false;
    {
      const uint64_t now = wall_clock64();
      if (t0 == 0) t0 = now;
      else if (now - t0 > kSpinTicks) {
        __hip_atomic_store((gu32*)(ctl + kAbort), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (status) __hip_atomic_store((gu32*)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
}

// poll_gran over row granules (tagged pairs or granule pairs, above)
template <int N>
XA_DEV bool poll_row(__amdgpu_buffer_rsrc_t r, const uint32_t (&off)[N], int n, unsigned tag,
                     RowG (&v)[N], unsigned* ctl, unsigned epoch, int* status) {
  uint64_t t0 = 0;
  for (unsigned it = 0;; ++it) {
    const bool slow = (it & 15u) == 15u;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < n) v[u] = ld_row(r, off[u]);
    const unsigned ab = slow ? __hip_atomic_load((gu32*)(ctl + kAbort), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0u;
    bool ok = true;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < n) ok = ok && row_ok(v[u], tag);
    if (ok) return true;
    if (!slow) {
#ifndef XA_POLL_NOSLEEP
      __builtin_amdgcn_s_sleep(XA_POLL_SLEEP);
#endif
      continue;
    }
    if (ab == epoch) return false;
    {
      const uint64_t now = wall_clock64();
      if (t0 == 0) t0 = now;
      else if (now - t0 > kSpinTicks) {
        __hip_atomic_store((gu32*)(ctl + kAbort), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (status) __hip_atomic_store((gu32*)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
}

// poll_gran over tagged f64 pairs (d_tagged, above); entry u is polled when bit u of `valid`
// is set
template <int N>
XA_DEV bool poll_d2(__amdgpu_buffer_rsrc_t r, const uint32_t (&off)[N], uint32_t valid,
                    unsigned tag, double2 (&v)[N], unsigned* ctl, unsigned epoch, int* status) {
  uint64_t t0 = 0;
  for (unsigned it = 0;; ++it) {
    const bool slow = (it & 15u) == 15u;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if ((valid >> u) & 1u) v[u] = ld_wt_d2(r, off[u]);
    const unsigned ab = slow ? __hip_atomic_load((gu32*)(ctl + kAbort), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0u;
    bool ok = true;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if ((valid >> u) & 1u) ok = ok && d2_ok(v[u], tag);
    if (ok) return true;
    if (!slow) {
#ifndef XA_POLL_NOSLEEP
      __builtin_amdgcn_s_sleep(XA_POLL_SLEEP);
#endif
      continue;
    }
    if (ab == epoch) return false;
    {
      const uint64_t now = wall_clock64();
      if (t0 == 0) t0 = now;
      else if (now - t0 > kSpinTicks) {
        __hip_atomic_store((gu32*)(ctl + kAbort), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (status) __hip_atomic_store((gu32*)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
}

// this workgroup's XCD (MI355X_MICROARCH.md: read placement from HW_REG_XCC_ID)
XA_DEV int xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return (int)(x & (kXcds - 1));
}

// Per-block phase trace (diagnostic -DXA_TRACE builds only, tools/trace_ppo_update.py):
// thread 0 of every logical block records the low 32 bits of the 100 MHz real-time clock
// at 16 points of every optimizer step into LDS (a global store there would hold up the
// next barrier until it is acknowledged) and copies them out at the end of the launch;
// slot kTraceSteps - 1 holds the launch start / phase-0 hop and the shader clock pairs.
#ifdef XA_TRACE
constexpr int kTraceSteps = 32, kTracePts = 16;
__device__ unsigned xa_ppo_trace[256 * kTraceSteps * kTracePts];
#define XA_TRACE_PT(blk, k, i)                                                        \
  do {                                                                                \
    if (threadIdx.x == 0 && (k) < kTraceSteps) {                                      \
      unsigned long long t_;                                                          \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
      U.trace[(k) * kTracePts + (i)] = (unsigned)t_;                                  \
    }                                                                                 \
  } while (0)
// the shader clock beside the real-time clock (the clock rate the launch ran at)
#define XA_TRACE_CLK(blk, i)                                                          \
  do {                                                                                \
    if (threadIdx.x == 0) {                                                           \
      unsigned long long t_, c_;                                                      \
      asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"        \
                   : "=s"(t_), "=s"(c_)::"memory");                                   \
      U.trace[(kTraceSteps - 1) * kTracePts + 8 + 2 * (i)] = (unsigned)t_;            \
      U.trace[(kTraceSteps - 1) * kTracePts + 9 + 2 * (i)] = (unsigned)c_;            \
    }                                                                                 \
  } while (0)
#define XA_TRACE_FLUSH(blk)                                                           \
  do {                                                                                \
    __syncthreads();                                                                  \
    for (int i_ = threadIdx.x; i_ < kTraceSteps * kTracePts; i_ += 256)              \
      xa_ppo_trace[(size_t)(blk) * kTraceSteps * kTracePts + i_] = U.trace[i_];      \
  } while (0)
#else
#define XA_TRACE_PT(blk, k, i) \
  do {                         \
  } while (0)
#define XA_TRACE_CLK(blk, i) \
  do {                       \
  } while (0)
#define XA_TRACE_FLUSH(blk) \
  do {                      \
  } while (0)
#endif

// Workspace (device memory, zeroed once by the caller at allocation; nothing in it is
// reset between launches):
//   ctl      control words (abort word, XCD election; word 0 unused since round 6)
//   persist  the launch generation gen (the granule tags of every launch differ)
//   rows_g   [G, PP/2] tagged pairs (8 B): the blocks' gradient rows
//   g_g      [PP/2] tagged pairs: the reduced gradient (sized for the round-5 form, which
//            also held per-block norm partials)
//   adv      [K, G, 2] f64 advantage sums (phase-0 hop)
//   cen_g    [G] granule pairs: the XCD each block runs on (two-level census)
//   xpart_g  [kXcds, PP/2] tagged f64 pairs (16 B): per-XCD partial sums of the rows
//            (two-level)
// A granule is 8 bytes {32-bit value, 32-bit tag}; two of them travel in one 16-byte
// access (MI355X_MICROARCH.md: 16-B write-through halves observed untorn), and the tag
// is the step's epoch, so the data is its own flag: consumers poll the data. A tagged
// pair / tagged f64 pair carries only the tag's parity, in each value's lowest mantissa
// bit (XA_ROW_PAIRS, below).
struct Ws {
  unsigned* ctl;
  unsigned* persist;
  void* rows_g;
  void* g_g;
  double* adv;
  void* cen_g;
  void* xpart_g;
  size_t total;
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

__host__ __device__ inline int padded(int P) { return (P + 3) & ~3; }

__host__ __device__ inline Ws carve(void* base, int G, int P, int K) {
  Ws w;
  char* c = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = c + off;
    off = align_up(off + bytes, 256);
    return q;
  };
  const size_t PP = padded(P);
  w.ctl = (unsigned*)take(kCtlBytes);
  w.persist = (unsigned*)take(256);
  w.rows_g = take((size_t)G * PP * 8);
  w.g_g = take(PP * 8 + (size_t)G * 64);
  w.adv = (double*)take((size_t)K * G * 2 * sizeof(double));
  w.cen_g = take((size_t)G * 16);
  w.xpart_g = take((size_t)kXcds * PP * 16);
  w.total = off;
  return w;
}

__host__ __device__ inline size_t ws_bytes(int G, int P, int K) {
  return carve(nullptr, G, P, K).total;
}

// Data-parallel exchange block (one per rank, uncached, IPC-mapped into every rank,
// zeroed once): (32-bit word, 32-bit tag) pairs written with system-scope 8-byte stores
// by the pushing rank and polled by the owner (the xa_peer_allreduce protocol, comm.hip)
//   adv [G][W][K] x 4 pairs: block b's copy of rank r's minibatch-k advantage sums (2 f64)
//   gsl [2 parity][G][W][CB] x 2 pairs: rank r's reduced slice b (pair column c) at step
//       parity k & 1 (a rank runs at most one step ahead of any other: step k + 1 needs
//       every rank's step-(k + 1) slice, pushed only after that rank consumed step k)
struct DpLayout {
  size_t adv, gsl, total;
};
__host__ __device__ inline DpLayout dp_layout(int G, int W, int K, int CB) {
  DpLayout d;
  d.adv = 0;
  d.gsl = align_up((size_t)G * W * K * 32, 256);
  d.total = d.gsl + (size_t)2 * G * W * CB * 16;
  return d;
}
XA_DEV void dp_st(void* base, size_t off, uint32_t word, unsigned tag) {
  __hip_atomic_store((unsigned long long*)((char*)base + off),
                     (unsigned long long)word | ((unsigned long long)tag << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
XA_DEV unsigned long long dp_ld(const void* base, size_t off) {
  return __hip_atomic_load((unsigned long long*)((char*)base + off), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
// Poll n (<= N) pairs of the own block until every tag equals `tag` (bounded by the wall
// clock and the abort word, like poll_gran); the words land in w.
template <int N>
XA_DEV bool dp_poll(const void* base, const size_t (&off)[N], int n, unsigned tag,
                    uint32_t (&w)[N], unsigned* ctl, unsigned epoch, int* status) {
  uint64_t t0 = 0;
  for (unsigned it = 0;; ++it) {  // abort word and clock every 16th round, as poll_gran
    const bool slow = (it & 15u) == 15u;
    bool ok = true;
#pragma unroll
    for (int u = 0; u < N; ++u)
      if (u < n) {
        const unsigned long long v = dp_ld(base, off[u]);
        w[u] = (uint32_t)v;
        ok = ok && (unsigned)(v >> 32) == tag;
      }
    const unsigned ab = slow ? __hip_atomic_load((gu32*)(ctl + kAbort), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0u;
    if (ok) return true;
    if (slow) {
      if (ab == epoch) return false;
      const uint64_t now = wall_clock64();
      if (t0 == 0) t0 = now;
      else if (now - t0 > kSpinTicks) {
        __hip_atomic_store((gu32*)(ctl + kAbort), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (status) __hip_atomic_store((gu32*)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(XA_POLL_SLEEP);
  }
}

struct ShufKeys {
  uint32_t k[4];
  uint32_t half_bits;
};

// same keys / permutation as xa_ppo_minibatches (ac_update.hip)
XA_DEV ShufKeys shuf_keys(const XaShuffle& sh, uint64_t ctr, int epoch, int batch) {
  ShufKeys s;
  const xa_u4 r = xa_philox((uint32_t)epoch, 0x5u, (uint32_t)ctr, (uint32_t)(ctr >> 32),
                            (uint32_t)sh.seed, (uint32_t)(sh.seed >> 32));
  s.k[0] = r.x;
  s.k[1] = r.y;
  s.k[2] = r.z;
  s.k[3] = r.w;
  const uint32_t bits = batch <= 1 ? 1u : 32u - __clz((uint32_t)(batch - 1));
  s.half_bits = (bits + 1u) / 2u;
  if (s.half_bits == 0) s.half_bits = 1;
  return s;
}

XA_DEV int shuf_index(const XaShuffle& sh, const ShufKeys& keys, int epoch, int batch, int g) {
  if (sh.perm) return sh.perm[(size_t)epoch * batch + g];
  return (int)xa_permute((uint32_t)g, (uint32_t)batch, keys.half_bits, keys.k[0], keys.k[1],
                         keys.k[2], keys.k[3]);
}

// Per-sample inputs of every tile a block processes in the launch, gathered in phase 0
// when they fit: {obs[OBS], action (-1 = padding), return, old value, old log-prob}.
constexpr int kPreBytes = 16384;
template <int OBS>
constexpr int pre_max() { return kPreBytes / ((OBS + 4) * 4); }

constexpr int kBF = 11;  // granules per thread of a one-round flat gather
template <int OBS, int A, int TS>
struct UpdLds {
  PtLds<OBS, A, TS> t;
  alignas(16) float row[(offs(OBS, A).P + 3) & ~3];  // the gradient row's non-W2 part, staged
  alignas(16) float pre[pre_max<OBS>() * (OBS + 4)]; // preloaded tile inputs
  alignas(16) float stage[TS * (OBS + 4)];           // one tile's inputs (when not preloaded)
  // flat-gather scratch of phase B: its own array at TS = 16; at TS = 32 the tile's
  // activation buffers sH1 .. sdA2 (dead between the row write and the next step's tile)
  alignas(16) float scr_own[TS == 32 ? 4 : 2 * 256 * kBF];
  XA_DEV float* scr() {
    static_assert(TS != 32 || (H + 2 * TS) * LDW + H * PtLds<OBS, A, TS>::LDT >= 2 * 256 * kBF,
                  "gather scratch");
    return TS == 32 ? t.sH1 : scr_own;
  }
  // Adam moments of the thread's parameter slice (16 W2 values, then the rest: NS slots),
  // four slots per 16-byte word, thread-major (lane-consecutive, no bank conflicts):
  // mv4[0][q / 4][t] holds m of slots q .. q + 3, mv4[1] the same for v
  static constexpr int NS = 16 + Dims<OBS, A>::RPT, NQ4 = (NS + 3) / 4;
  float4 mv4[2][NQ4][256];
  float alpha[kMaxSteps];    // per optimizer step: the Adam step size
  // per optimizer step: advantage mean, population std, 1 / (std + eps), loss scale
  float stat[kMaxSteps][4];
  double red[256 * 4];
  double wsum[4];
  int flag;
  int xn[kXcds];      // blocks per XCD (census)
  int wx[4][kXcds];   // census: blocks per (wave of block ids, XCD)
  int xmem[256];      // this XCD's blocks, ascending block id (two-level)
  int xrank;          // this block's position among them
#ifdef XA_TRACE
  unsigned trace[kTraceSteps * kTracePts];
#endif
};

// XCD-local mode: the launch has kXcds x G workgroups; the G that run on the XCD whose
// G-th workgroup arrives first do the update (logical block ids = their arrival ranks),
// every other workgroup leaves at once. A winner always exists once every XCD's first G
// arrivals are resident (the host launches this mode only when kXcds G fit), and every
// hand-off of the launch then stays inside one L2: plain stores (the lines stay in the
// shared L2) and L1-bypassing sc1 loads, no write-through round trip to the fabric.
// Placement decides speed, never correctness: a workgroup learns its XCD from
// HW_REG_XCC_ID and only workgroups of the elected XCD exchange data.
// Two halves, so that phase 0's gather runs while the election completes (speculatively:
// nothing is stored before the winner is known). elect_rank: the workgroup's arrival rank
// on its XCD (its logical block id if the XCD wins; >= G: leave); the G-th arrival claims the
// winner word. Contains a __syncthreads().
XA_DEV int elect_rank(unsigned* ctl, int G, unsigned par, int xcc, int& lds) {
  if (threadIdx.x == 0) {
    const unsigned r = __hip_atomic_fetch_add((gu32*)(ctl + kElect + par * kXcds + xcc), 1u,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int id = r < (unsigned)G ? (int)r : -1;
    if (r == (unsigned)G - 1u) {
      // the G-th arrival: claim the winner word (no wait for the result here: elect_won
      // reads it later); the claim's own result then decides without a poll
      unsigned expect = 0u;
      const bool mine = __hip_atomic_compare_exchange_strong(
          (gu32*)(ctl + kWin + par), &expect, (unsigned)xcc + 1u, __ATOMIC_RELAXED,
          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      id = mine ? id : -2 - id;  // (-2 - r: rank r of a losing XCD, decided already)
    }
    lds = id;
  }
  __syncthreads();
  const int v = lds;
  return v <= -2 ? -2 - v : v;
}
// elect_won (thread 0 only): did this XCD win? The G-th arrival knows from its claim; the
// others poll the winner word (bounded: a timeout raises the abort word and `status`)
XA_DEV bool elect_won(unsigned* ctl, unsigned par, int xcc, int claim, unsigned epoch,
                      int* status) {
  if (claim != 0) return claim > 0;
  gu32* win_w = (gu32*)(ctl + kWin + par);
  const uint64_t t0 = wall_clock64();
  unsigned win;
  while ((win = __hip_atomic_load(win_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u) {
    if (wall_clock64() - t0 > kSpinTicks) {
      __hip_atomic_store((gu32*)(ctl + kAbort), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (status) __hip_atomic_store((gu32*)status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(XA_POLL_SLEEP);
  }
  return win == (unsigned)xcc + 1u;
}

// TS = samples per tile (32; 16 when the minibatch has at most 16 tiles of 32: twice the
// blocks, half the element-wise work per block and step); PRE = every tile input of the
// launch fits the block's LDS records (gathered once in phase 0); loc = XCD-local mode
// BF = the phase-B reduce forms compiled in: 0 every form (chosen per block at run time);
// 1 the column form only (the host checked col_b_everywhere); 2 the two-level reduce only
// (spread grids of >= kTwoLevelMinG blocks with 32-sample tiles). Compiling the unused forms
// out lowers the register allocation of the whole kernel body (16-env update 167 -> 161 us,
// profiles/r03ah_variants.txt)
// BF = 3: the column form AND the headline shape compiled in (16 envs x 128 steps, 4 epochs
// x 4 minibatches of 512 per rank, 32 blocks of 16-sample tiles: every loop bound, tile
// count and exchange offset a constant, fewer live uniform values -- xa_ppo_update picks it
// when the launch is exactly that shape)
// BF = 4: the same for BASELINE configs[1] (256 envs x 128 steps, minibatches of 8192, 256
// spread blocks of 32-sample tiles, the two-level reduce)
template <int BF>
struct FixShape {  // (B, MB, K, n_mb, G) of a fixed-shape instantiation (per rank)
  static constexpr int B = BF == 3 ? 2048 : 32768, MB = BF == 3 ? 512 : 8192, K = 16, NMB = 4;
  static constexpr int G = BF == 3 ? 32 : 256;
};
template <int OBS, int A, int TS, bool DP, bool PRE, int BF = 0>
__global__ __launch_bounds__(256) void ppo_update_kernel(XaPpoUpdateArgs p, Ws ws, int K_,
                                                          int n_mb_, int loc_) {
  constexpr bool FIX = BF == 3 || BF == 4;
  typedef FixShape<BF> FS;
  const int K = FIX ? FS::K : K_, n_mb = FIX ? FS::NMB : n_mb_, loc = loc_;
  constexpr int RPT = Dims<OBS, A>::RPT;
  __shared__ __attribute__((aligned(16))) UpdLds<OBS, A, TS> U;
  PtLds<OBS, A, TS>& L = U.t;
  const Offs o = offs(OBS, A);
  const int P = o.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  XA_STAMP_DECL
#ifdef XA_TRACE
  unsigned long long t_entry_;  // (diagnostic) kernel entry, before the election
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_entry_)::"memory");
#endif

  // the launch generation (written write-through by block 0 at the end of the previous
  // launch; block 0 of this launch writes the next one only after it polled every block's
  // phase-0 sums, which each block stores after reading this word)
  const unsigned gen =
      __hip_atomic_load((gu32*)ws.persist, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned epoch = gen + 1u;
  const unsigned par = gen & 1u;
  const int xcc = xcc_id();
  const int G = FIX ? FS::G : loc ? p.n_blocks : (int)gridDim.x;
  // XCD-local mode: the arrival rank (the block id if this XCD wins); the G-th arrival's
  // claim result rides in U.flag's sign until elect_won (claim: +1 won, -1 lost, 0 poll)
  int claim = 0;
  int b = (int)blockIdx.x;
  if (loc) {
    b = elect_rank(ws.ctl, G, par, xcc, U.flag);
    if (b < 0) return;
    if (b == G - 1 && tid == 0) claim = U.flag >= 0 ? 1 : -1;
  }
#ifdef XA_TRACE
  if (tid == 0) U.trace[(kTraceSteps - 1) * kTracePts + 5] = (unsigned)t_entry_;
#endif
  // the train step's episode statistics into host slot gen % XA_PPO_STATS_SLOTS (posted
  // stores to mapped host memory that drain while the update runs): the thread's first
  // kSW words loaded now and stored after the phase-0 gather (a store waits for its load:
  // issued here it held the block for an HBM round trip before any other work)
  constexpr int kSW = 2;
  const unsigned* const st_src = static_cast<const unsigned*>(p.stats_src);
  unsigned* const st_dst =
      p.stats_words > 0 ? static_cast<unsigned*>(p.stats_dst[gen % XA_PPO_STATS_SLOTS]) : nullptr;
  unsigned st_w[kSW];
#pragma unroll
  for (int u = 0; u < kSW; ++u) {
    const int i = b * 256 + tid + u * G * 256;
    st_w[u] = i < p.stats_words ? st_src[i] : 0u;
  }
  XA_STAMP_BLOCK(b == 0)
  XA_STAMP(30);
  XA_TRACE_PT(b, kTraceSteps - 1, 6);  // launch start (after the election)
  XA_TRACE_CLK(b, 0);
  const int B = FIX ? FS::B : p.batch, MB = FIX ? FS::MB : p.mb_size;
  const uint64_t ctr = p.shuffle.rng_counter ? *p.shuffle.rng_counter : 0ull;
  // parameters: theta / m / v slices in registers for the whole launch (m / v parked in LDS
  // after phase 0); their loads issued first, in flight under phase 0
  constexpr int RPT_ = Dims<OBS, A>::RPT;
  PSlice<OBS, A, TS> ps;
  ps.init(tid);
  float wv[16], rv[RPT_], mw[16], mr[RPT_], vw[16], vr[RPT_];
  ps.load(p.theta, wv, rv);
  ps.load(p.adam_m, mw, mr);
  ps.load(p.adam_v, vw, vr);
  // hand-off stores: write-through across XCDs, plain inside the elected XCD's L2
  const bool kWt = !loc;

  // ---- census: which XCD this block runs on (a granule, read after the phase-0 hop) ----
  // 16-sample tiles run only on small grids (<= 32 blocks): one level, known at compile time
  const bool two_level = BF == 2 || BF == 4 || (BF == 0 && !loc && TS == S && G >= kTwoLevelMinG);
  const __amdgpu_buffer_rsrc_t cen_r = rsrc(ws.cen_g, (uint32_t)(G * 16));
  if (two_level && tid == 0) st_gran2(cen_r, (uint32_t)(16 * b), __uint_as_float((unsigned)xcc),
                                      __uint_as_float((unsigned)xcc), epoch, true);

  // ---- phase 0: advantage sums of this block's samples of every minibatch; their
  // inputs into LDS when all of them fit; the Adam step size of every step ----
  const int n_tiles_max = (min(MB, B) + TS - 1) / TS;
  const int TPB = (n_tiles_max + G - 1) / G;  // tiles per block per step (at most)
  constexpr bool pre = PRE;  // the host checked K * TPB * TS <= pre_max
  const int t0 = *p.adam_step;
  for (int k = tid; k < K; k += 256)
    U.alpha[k] = adam_alpha(p.adam.lr, p.adam.beta1, p.adam.beta2, t0 + k + 1);
  // with the inputs preloaded: all 256 threads gather the (step, sample) items and park each
  // advantage in LDS (U.red, free until phase B), then a wave per step sums them in the
  // lane-strided order of the loop below (bit-identical sums, all lanes busy in the gather)
  float* const advs = reinterpret_cast<float*>(U.red);
  // the blocks' per-minibatch advantage sums: tagged f64 pairs {s1, s2} (tag: the launch
  // epoch's parity), polled by every block -- the data is its own flag, no counter hop
  const __amdgpu_buffer_rsrc_t adv_r = rsrc(ws.adv, (uint32_t)((size_t)K * G * 16));
  const int per_k = TPB * TS;
  if (pre) {
    for (int i = tid; i < K * per_k; i += 256) {
      const int k = i / per_k, j = i - k * per_k;
      const int e = k / n_mb, m = k - e * n_mb;
      const int start = m * MB, cnt = min(MB, B - start);
      const int n_tiles = (cnt + TS - 1) / TS;
      const int mine = n_tiles > b ? (n_tiles - b + G - 1) / G : 0;
      const int q = (b + (j / TS) * G) * TS + (j % TS);
      float* slot = &U.pre[(size_t)i * (OBS + 4)];
      if (!(j < mine * TS && q < cnt)) {
        // padding: zero inputs (they meet zero gradients, never NaNs)
#pragma unroll
        for (int kk = 0; kk < OBS + 4; ++kk) slot[kk] = 0.0f;
        slot[OBS] = -1.0f;
        advs[i] = 0.0f;
        continue;
      }
      const ShufKeys keys = shuf_keys(p.shuffle, ctr, e, B);
      const int idx = shuf_index(p.shuffle, keys, e, B, start + q);
      const float ret = p.returns[idx], oldv = p.old_values[idx];
      advs[i] = ret - oldv;
#pragma unroll
      for (int kk = 0; kk < OBS; ++kk) slot[kk] = p.obs[(size_t)idx * OBS + kk];
      slot[OBS] = (float)p.actions[idx];
      slot[OBS + 1] = ret;
      slot[OBS + 2] = oldv;
      slot[OBS + 3] = p.old_logp[idx];
    }
    __syncthreads();
  }
  if (loc) {
    // stores follow: leave unless this XCD won the election
    if (tid == 0) U.flag = elect_won(ws.ctl, par, xcc, claim, epoch, p.status) ? 1 : 0;
    __syncthreads();
    if (U.flag == 0) return;
  }
  XA_TRACE_PT(b, kTraceSteps - 1, 0);  // phase-0 gather done
  // preloaded inputs of <= 32 samples per step: each minibatch's sums on a 16- or 32-lane row
  // group, 4 or 2 minibatches per wave at once -- the xa_wave_sum_f64 tree of one minibatch
  // with the other lanes zero (intra-row stages, then row_bcast15 for 32 lanes), so the
  // same f64 sums (the lanes outside the group only ever added zeros there)
  const bool grp0 = pre && per_k <= 32;
  if (grp0) {
    const int RL = per_k <= 16 ? 16 : 32, KPW = 64 / RL;
    const int g = lane / RL, j = lane - g * RL;
    for (int k0 = w; k0 < K; k0 += 4 * KPW) {
      const int k = k0 + 4 * g;
      double s1 = 0.0, s2 = 0.0;
      if (k < K && j < per_k) {
        const double a = (double)advs[k * per_k + j];
        s1 += a;
        s2 += a * a;
      }
      s1 = s1 + xa_dpp_f64<0xB1>(s1);
      s2 = s2 + xa_dpp_f64<0xB1>(s2);
      s1 = s1 + xa_dpp_f64<0x4E>(s1);
      s2 = s2 + xa_dpp_f64<0x4E>(s2);
      s1 = s1 + xa_dpp_f64<0x141>(s1);
      s2 = s2 + xa_dpp_f64<0x141>(s2);
      s1 = s1 + xa_dpp_f64<0x140>(s1);
      s2 = s2 + xa_dpp_f64<0x140>(s2);
      if (RL == 32) {
        s1 = s1 + xa_dpp_f64<0x142, 0xA>(s1);
        s2 = s2 + xa_dpp_f64<0x142, 0xA>(s2);
      }
      if (k < K && j == RL - 1) st_d2_tagged(adv_r, (uint32_t)((k * G + b) * 16), s1, s2, epoch);
    }
  }
#ifndef XA_ABL_P0
  for (int k = w; k < K && !grp0; k += 4) {
#else
  for (int k = w; k < 0; k += 4) {
#endif
    if (pre) {
      double s1 = 0.0, s2 = 0.0;
      for (int j = lane; j < per_k; j += 64) {
        const double a = (double)advs[k * per_k + j];
        s1 += a;
        s2 += a * a;
      }
      s1 = xa_wave_sum_f64(s1);
      s2 = xa_wave_sum_f64(s2);
      if (lane == 0) st_d2_tagged(adv_r, (uint32_t)((k * G + b) * 16), s1, s2, epoch);
      continue;
    }
    const int e = k / n_mb, m = k - e * n_mb;
    const int start = m * MB, cnt = min(MB, B - start);
    const int n_tiles = (cnt + TS - 1) / TS;
    const ShufKeys keys = shuf_keys(p.shuffle, ctr, e, B);
    const int mine = n_tiles > b ? (n_tiles - b + G - 1) / G : 0;  // tiles of this block
    double s1 = 0.0, s2 = 0.0;
    for (int j = lane; j < (pre ? TPB : mine) * TS; j += 64) {
      const int q = (b + (j / TS) * G) * TS + (j % TS);
      const bool valid = j < mine * TS && q < cnt;
      float* slot = &U.pre[((size_t)k * TPB * TS + j) * (OBS + 4)];
      if (!valid) {
        if (pre) {  // padding: zero inputs (they meet zero gradients, never NaNs)
#pragma unroll
          for (int kk = 0; kk < OBS + 4; ++kk) slot[kk] = 0.0f;
          slot[OBS] = -1.0f;
        }
        continue;
      }
      const int idx = shuf_index(p.shuffle, keys, e, B, start + q);
      const float ret = p.returns[idx], oldv = p.old_values[idx];
      const float adv = ret - oldv;
      s1 += (double)adv;
      s2 += (double)adv * (double)adv;
      if (pre) {
#pragma unroll
        for (int kk = 0; kk < OBS; ++kk) slot[kk] = p.obs[(size_t)idx * OBS + kk];
        slot[OBS] = (float)p.actions[idx];
        slot[OBS + 1] = ret;
        slot[OBS + 2] = oldv;
        slot[OBS + 3] = p.old_logp[idx];
      }
    }
    s1 = xa_wave_sum_f64(s1);
    s2 = xa_wave_sum_f64(s2);
    if (lane == 0) st_d2_tagged(adv_r, (uint32_t)((k * G + b) * 16), s1, s2, epoch);
  }
  XA_TRACE_PT(b, kTraceSteps - 1, 1);  // advantage sums stored
  if (p.stats_words > 0) {
#pragma unroll
    for (int u = 0; u < kSW; ++u) {
      const int i = b * 256 + tid + u * G * 256;
      if (i < p.stats_words) st_dst[i] = st_w[u];
    }
    for (int i = b * 256 + tid + kSW * G * 256; i < p.stats_words; i += G * 256)
      st_dst[i] = st_src[i];
    if (b == 0 && tid == 0) st_dst[p.stats_words] = gen;
  }
  XA_STAMP(31);

  constexpr int NS = UpdLds<OBS, A, TS>::NS, NQ4 = UpdLds<OBS, A, TS>::NQ4;
  {  // the Adam moments live in LDS (register pressure of the step loop)
    float mm[4 * NQ4], vv[4 * NQ4];
#pragma unroll
    for (int q = 0; q < 4 * NQ4; ++q) {
      mm[q] = q < 16 ? mw[q] : q < NS ? mr[q - 16] : 0.0f;
      vv[q] = q < 16 ? vw[q] : q < NS ? vr[q - 16] : 0.0f;
    }
#pragma unroll
    for (int q4 = 0; q4 < NQ4; ++q4) {
      U.mv4[0][q4][tid] = make_float4(mm[4 * q4], mm[4 * q4 + 1], mm[4 * q4 + 2], mm[4 * q4 + 3]);
      U.mv4[1][q4][tid] = make_float4(vv[4 * q4], vv[4 * q4 + 1], vv[4 * q4 + 2], vv[4 * q4 + 3]);
    }
  }
  ps.to_lds(L, wv, rv);

  XA_STAMP(32);
  XA_TRACE_PT(b, kTraceSteps - 1, 2);  // signalled; m / v and the weights in LDS
  XA_TRACE_PT(b, kTraceSteps - 1, 7);  // (no counter hop: the sums are polled below)
  if (two_level) {
    // thread t reads block t's census granule; per XCD, the member blocks in ascending id
    // (fixed reduction order and column split) from wave ballots
    int xt = -1;
    bool bad = false;
    if (tid < G) {
      const uint32_t off[1] = {(uint32_t)(16 * tid)};
      f32x4v v[1];
      bad = !poll_gran<1>(cen_r, off, 1, epoch, v, ws.ctl, epoch, p.status);
      xt = (int)__float_as_uint(v[0][0]);
    }
    if (__syncthreads_or(bad)) return;
    int below = 0;  // lanes of this wave below this one on the same XCD
#pragma unroll
    for (int x = 0; x < kXcds; ++x) {
      const unsigned long long m = __ballot(xt == x);
      if (lane == 0) U.wx[w][x] = __popcll(m);
      if (xt == x) below = __popcll(m & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    if (tid < kXcds) U.xn[tid] = (U.wx[0][tid] + U.wx[1][tid]) + (U.wx[2][tid] + U.wx[3][tid]);
    if (xt == xcc) {
      int rank = below;
      for (int ww = 0; ww < w; ++ww) rank += U.wx[ww][xt];
      U.xmem[rank] = tid;
      if (tid == b) U.xrank = rank;
    }
    __syncthreads();
  }
  XA_STAMP(33);
  const int W = DP ? p.dp_world : 1;  // DP: compiled only into the data-parallel kernels
  const int CB0 = (padded(P) / 2 + G - 1) / G;
  const DpLayout dl = dp_layout(G, W, K, CB0);
  bool dp_bad = false;  // a phase-0 poll (or the DP exchange) timed out / aborted
  {
    // the blocks' per-minibatch advantage sums: wave w sums minibatches w, w + 4, ...; it
    // issues the 16-B {s1, s2} sc1 loads of up to kAB (minibatch, block) pairs at once (one
    // round trip per batch, not one per minibatch: 16 envs 3.7 -> see DESIGN.md), then adds
    // them per lane in ascending block order gi = lane, lane + 64, ... (the same f64 sums as
    // one load at a time) -> wave sums -> U.red (dead between phase 0 and phase B)
    constexpr int kAB = 16;
    const int LPK = (G + 63) / 64;         // loads per lane per minibatch
    const int nj = ((K - w + 3) / 4) * LPK;  // this wave's (minibatch, load) items
    double a1 = 0.0, a2 = 0.0;
    for (int j0 = 0; j0 < nj && !dp_bad; j0 += kAB) {
      double2 x[kAB];
      uint32_t off[kAB], valid = 0u;
#pragma unroll
      for (int u = 0; u < kAB; ++u) {
        const int j = j0 + u, kk = j / LPK, gi = lane + 64 * (j - kk * LPK);
        off[u] = (uint32_t)(((w + 4 * kk) * G + gi) * 16);
        if (j < nj && gi < G) valid |= 1u << u;
        x[u] = make_double2(0.0, 0.0);
      }
      dp_bad = !poll_d2<kAB>(adv_r, off, valid, epoch, x, ws.ctl, epoch, p.status);
#pragma unroll
      for (int u = 0; u < kAB; ++u) {
        const int j = j0 + u, kk = j / LPK, jj = j - kk * LPK;
        if (j < nj && lane + 64 * jj < G) {
          a1 += x[u].x;
          a2 += x[u].y;
        }
        if (j < nj && jj == LPK - 1) {
          a1 = xa_wave_sum_f64(a1);
          a2 = xa_wave_sum_f64(a2);
          if (lane == 0) {
            U.red[2 * (w + 4 * kk)] = a1;
            U.red[2 * (w + 4 * kk) + 1] = a2;
          }
          a1 = a2 = 0.0;
        }
      }
    }
    // (the wave reads back only its own LDS words, in issue order)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  XA_TRACE_PT(b, kTraceSteps - 1, 4);  // the advantage totals summed
  for (int k = w; DP && k < K; k += 4) {
    double s1 = U.red[2 * k], s2 = U.red[2 * k + 1];
    if constexpr (DP) {
      // lane q pushes this rank's totals to rank q (block b's slot); lane r then reads rank
      // r's totals from the own block; the sums run in rank order
      const unsigned long long u1 = (unsigned long long)__double_as_longlong(s1);
      const unsigned long long u2 = (unsigned long long)__double_as_longlong(s2);
      const size_t o_me = dl.adv + (((size_t)b * W + p.dp_rank) * K + k) * 32;
      if (lane < W) {
        void* blk = p.dp_blocks[lane];
        dp_st(blk, o_me, (uint32_t)u1, epoch);
        dp_st(blk, o_me + 8, (uint32_t)(u1 >> 32), epoch);
        dp_st(blk, o_me + 16, (uint32_t)u2, epoch);
        dp_st(blk, o_me + 24, (uint32_t)(u2 >> 32), epoch);
      }
      double v1 = 0.0, v2 = 0.0;
      if (lane < W) {
        const size_t o = dl.adv + (((size_t)b * W + lane) * K + k) * 32;
        const size_t off[4] = {o, o + 8, o + 16, o + 24};
        uint32_t x[4];
        dp_bad = dp_bad || !dp_poll<4>(p.dp_blocks[p.dp_rank], off, 4, epoch, x, ws.ctl, epoch,
                                       p.status);
        v1 = __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
        v2 = __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
      }
      s1 = 0.0;
      s2 = 0.0;
      for (int r = 0; r < W; ++r) {
        s1 += __shfl(v1, r);
        s2 += __shfl(v2, r);
      }
    }
    if (lane == 0) {
      U.red[2 * k] = s1;
      U.red[2 * k + 1] = s2;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // every minibatch's mean / population std on its own lane (lane j of wave w: minibatch
  // w + 4 j; the wave summed -- and, DP, exchanged -- exactly those), not one after another
  for (int k = w + 4 * lane; k < K; k += 256) {
    const int m = k % n_mb;
    const double n = (double)min(MB, B - m * MB) * (double)W;
    const double s1 = U.red[2 * k], s2 = U.red[2 * k + 1];
    const double mean = s1 / n;
    const double var = fmax(s2 / n - mean * mean, 0.0);
    const float sd = (float)sqrt(var);
    U.stat[k][0] = (float)mean;
    U.stat[k][1] = sd;
    U.stat[k][2] = 1.0f / (sd + p.adv_eps);
    U.stat[k][3] = 1.0f / (float)(min(MB, B - m * MB) * W);
  }

  if (__syncthreads_or(dp_bad)) return;
  XA_TRACE_PT(b, kTraceSteps - 1, 3);  // the minibatch statistics in LDS

  // per-sample inputs of the next tile (threads < TS), fetched one tile ahead -- across
  // minibatch boundaries too: they do not depend on the parameters. The next step's
  // first tile is fetched between the row hop's signal and wait (off the critical path).
  float nx[OBS], n_act = 0.0f, n_ret = 0.0f, n_oldv = 0.0f, n_oldlp = 0.0f;
  int n_valid = 0;
  auto fetch_tile = [&](int k, int tile) {
    if (pre || tid >= TS) return;
    long idx = -1;
    if (k < K) {
      const int e = k / n_mb, m = k - e * n_mb;
      const int start = m * MB, cnt = min(MB, B - start);
      const int q = tile * TS + tid;
      if (q < cnt) {
        const ShufKeys keys = shuf_keys(p.shuffle, ctr, e, B);
        idx = shuf_index(p.shuffle, keys, e, B, start + q);
      }
    }
    n_valid = idx >= 0;
    const size_t ix = idx >= 0 ? (size_t)idx : 0;
#pragma unroll
    for (int kk = 0; kk < OBS; ++kk) nx[kk] = idx >= 0 ? p.obs[ix * OBS + kk] : 0.0f;
    n_act = idx >= 0 ? (float)p.actions[ix] : 0.0f;
    n_ret = idx >= 0 ? p.returns[ix] : 0.0f;
    n_oldv = idx >= 0 ? p.old_values[ix] : 0.0f;
    n_oldlp = idx >= 0 ? p.old_logp[ix] : 0.0f;
  };
  fetch_tile(0, b);

  LossCfg cfg;
  cfg.is_ppo = true;
  cfg.has_adv_in = false;
  cfg.clip_norm = p.clip_norm;
  cfg.value_coef = p.value_coef;
  cfg.entropy_coef = p.entropy_coef;
  cfg.adv_eps = p.adv_eps;
  const float omb1 = 1.0f - p.adam.beta1, omb2 = 1.0f - p.adam.beta2;
  // rows are PP = P rounded up to 4 floats = PP/2 granule pairs (one pair per 16 B)
  const int PP = padded(P), NP2 = PP / 2;
  // phase B: block b reduces pair columns [c0, c0 + nc) of the gradient
  const int CB = (NP2 + G - 1) / G;
  const int c0 = min(NP2, b * CB), nc = min(NP2, c0 + CB) - c0;
  const __amdgpu_buffer_rsrc_t rows_r = rsrc(ws.rows_g, (uint32_t)((size_t)G * PP * 8));
  const __amdgpu_buffer_rsrc_t g_r = rsrc(ws.g_g, (uint32_t)(PP * 8 + G * 64));
  const __amdgpu_buffer_rsrc_t xp_r = rsrc(ws.xpart_g, (uint32_t)(kXcds * PP * 16));
  float* srow = U.row;
  for (int i = P + tid; i < PP; i += 256) srow[i] = 0.0f;  // the pad stays zero
  // granule tags: unique per (launch, step)
  auto tag_of = [&](int k) { return gen * (unsigned)K + (unsigned)k + 1u; };
  // Flat gather of nrow rows x ncol pair columns in ONE poll round (row r's pair column c
  // at byte offset base(r) + 16 c of `r`), staged as f32 pairs in LDS scratch (the W2
  // tiles: dead between the row write and phase C's refresh); summed afterwards in
  // ascending row order. Used when the rows x columns fit kBF granules per thread.
  float* const scr = U.scr();
  auto gather_rows = [&](__amdgpu_buffer_rsrc_t r, int nrow, int ncol, auto base,
                         unsigned tg) -> bool {
    const int total = nrow * ncol;
    uint32_t off[kBF];
    RowG x[kBF];
    int n = 0;
#pragma unroll
    for (int u = 0; u < kBF; ++u) {
      const int f = tid + 256 * u;
      const int rr = f / ncol;
      off[u] = f < total ? base(rr) + kRowPB * (uint32_t)(f - rr * ncol) : 0u;
      n += f < total;
    }
    const bool bad = !poll_row<kBF>(r, off, n, tg, x, ws.ctl, epoch, p.status);
#pragma unroll
    for (int u = 0; u < kBF; ++u)
      if (u < n) {
        const int f = tid + 256 * u;
        scr[2 * f] = row_v0(x[u]);
        scr[2 * f + 1] = row_v1(x[u]);
      }
    return bad;
  };

  PtAcc<OBS, A> acc;
  float w2r[16];  // dH1's B operand: W2 row 16 w + li, columns 16 lq .. (load_w2_rows)
  int k_tr = 0;  // the step the tile trace points belong to
  auto stampf = [&](int slot) {
    XA_STAMP(slot);
    // tile phases 50..55 -> points 8..13; H1 sub-points 47, 48, 49 -> 6, 7, 15
    XA_TRACE_PT(b, k_tr, slot == 49 ? 15 : slot == 48 ? 7 : slot == 47 ? 6 : 8 + (slot - 50));
  };
  (void)k_tr;
  (void)stampf;
  for (int k = 0; k < K; ++k) {
    const int m = k % n_mb;
    const int cnt = min(MB, B - m * MB);
    const int n_tiles = (cnt + TS - 1) / TS;
    const unsigned tag = tag_of(k);
    // the LDS weights of the previous step's Adam: with the layer-1 weights in registers
    // (kRegH1) the tile's first barrier orders them (H1 needs none of them), otherwise here
    if constexpr (!kRegH1<OBS, A>) __syncthreads();
    cfg.adv_mean = U.stat[k][0];
    cfg.adv_std = U.stat[k][1];
    cfg.adv_rstd = U.stat[k][2];
    cfg.loss_scale = U.stat[k][3];
    acc.zero();
    if constexpr (!kRegH1<OBS, A>) load_w2_rows(L, w2r);
    if (p.theta_trace && b == 0) ps.store(p.theta_trace + (size_t)k * P, wv, rv);  // diagnostic
    XA_STAMP(34);
    XA_TRACE_PT(b, k, 0);
    k_tr = k;
    // the block's gradient row in exchange order: the W2 part straight from the MFMA
    // accumulators as granule pairs (from the last tile, overlapping its dH1 phase), the
    // other parameters through LDS below
    const bool row_wt = kWt && !two_level;
    auto w2_out = [&](const PtAcc<OBS, A>& a) {
#ifndef XA_ABL_ROW
      pt_write_row_w2<OBS, A>(a, [&](int pr, float v0, float v1) {
        st_row(rows_r, (uint32_t)((size_t)b * NP2 + pr) * kRowPB, v0, v1, tag, row_wt);
      });
#endif
    };
    // ---- A: forward + loss + backward of this block's tiles ----
    for (int tile = b; tile < n_tiles; tile += G) {
      const bool last = tile + G >= n_tiles;
      if (pre) {
        // inputs straight from the phase-0 records (read-only: no staging, no barrier)
        XA_STAMP(35);
        const float* in = &U.pre[((size_t)k * TPB * TS + ((tile - b) / G) * TS) * (OBS + 4)];
#ifndef XA_ABL_TILE  // diagnostic ablation builds (tools/ablate_update.py) only
        pt_tile<OBS, A, TS>(L, acc, cfg, in, wv, w2r, rv[0], rv[1], stampf, last, w2_out);
#else
        if (last) w2_out(acc);
#endif
        XA_STAMP(36);
        XA_TRACE_PT(b, k, 14);
        continue;
      }
      __syncthreads();  // the previous tile's reads of the staged records are done
      if (tid < TS) {
        float* rec = &U.stage[tid * (OBS + 4)];
#pragma unroll
        for (int kk = 0; kk < OBS; ++kk) rec[kk] = nx[kk];
        rec[OBS] = n_valid ? n_act : -1.0f;
        rec[OBS + 1] = n_ret;
        rec[OBS + 2] = n_oldv;
        rec[OBS + 3] = n_oldlp;
      }
      if (tile + G < n_tiles) fetch_tile(k, tile + G);
      __syncthreads();
      XA_STAMP(35);
      pt_tile<OBS, A, TS>(L, acc, cfg, U.stage, wv, w2r, rv[0], rv[1], stampf, last, w2_out);
      XA_STAMP(36);
    }
    if (b >= n_tiles) w2_out(acc);  // no tile of this minibatch: a zero row
    // the rest of the row: 32-sample tiles store it straight from the lanes that hold its
    // values, one tagged word each, plus the pad words behind P (no LDS staging, no barrier:
    // C2 step 14.9 -> 14.4 us); 16-sample tiles stage it in LDS and store it coalesced
    // behind a barrier (the scattered word stores made their step slower: 7.5 -> 7.9 us,
    // profiles/r06v_ppo_update_trace.txt)
    constexpr bool kRowDirect = TS == S;
#ifndef XA_ABL_ROW
    if constexpr (kRowDirect) {
      pt_write_row_rest<OBS, A>(acc, [&](int x, float v) {
        st_row1(rows_r, (uint32_t)(((size_t)b * NP2 * 2 + x) * 4), v, tag, row_wt);
      }, p.loss_out != nullptr);
      if (tid < PP - P)
        st_row1(rows_r, (uint32_t)(((size_t)b * NP2 * 2 + P + tid) * 4), 0.0f, tag, row_wt);
    } else {
      pt_write_row_rest<OBS, A>(acc, [&](int x, float v) { srow[x] = v; }, p.loss_out != nullptr);
    }
#endif
    XA_STAMP(44);
    XA_TRACE_PT(b, k, 1);
    if (p.loss_out && tid == 0) {
      float* lo = p.loss_out + ((size_t)k * G + b) * 4;
      lo[0] = acc.l_pg;
      lo[1] = acc.l_v;
      lo[2] = acc.l_ent;
      lo[3] = acc.l_cnt;
    }
    if constexpr (!kRowDirect) {
      __syncthreads();
      for (int c = H * H / 2 + tid; c < NP2; c += 256)
        st_row(rows_r, (uint32_t)((size_t)b * NP2 + c) * kRowPB, srow[2 * c], srow[2 * c + 1], tag,
               row_wt);
    } else if constexpr (BF == 0) {
      // (the generic kernels' flat phase-B gather stages rows in the 32-sample tile's
      // activation buffers, which the slowest wave's dH1 phase may still read)
      __syncthreads();
    }
    XA_STAMP(45);
    XA_TRACE_PT(b, k, 2);
    fetch_tile(k + 1, b);  // the next step's first tile, while the other blocks finish
    XA_STAMP(37);
    if (two_level) {
      // ---- level 1, inside the XCD: its members' rows (in this XCD's L2) -> this XCD's
      // f64 partial of pair columns [xc0, xc0 + xnc), published write-through ----
      const int ng = U.xn[xcc];
      const int CBx = (NP2 + ng - 1) / ng;
      const int xc0 = min(NP2, U.xrank * CBx), xnc = min(NP2, xc0 + CBx) - xc0;
      const bool flat = false && ng * xnc <= 256 * kBF;  // measured slower at 32 rows (C2)
      if (flat && xnc > 0) {
        const bool bad = gather_rows(rows_r, ng, xnc, [&](int j) {
          return (uint32_t)((size_t)U.xmem[j] * NP2 + xc0) * kRowPB;
        }, tag);
        if (__syncthreads_or(bad)) return;
        for (int c = tid; c < xnc; c += 256) {
          double t0 = 0.0, t1 = 0.0;
          for (int j = 0; j < ng; ++j) {
            t0 += (double)scr[2 * (j * xnc + c)];
            t1 += (double)scr[2 * (j * xnc + c) + 1];
          }
          st_d2_tagged(xp_r, (uint32_t)(((size_t)xcc * NP2 + xc0 + c) * 16), t0, t1, tag);
        }
        __syncthreads();
      }
      const int ncol = max(1, min(xnc, 256)), RG = 256 / ncol;
      const int rg = tid / ncol, cq = tid - rg * ncol;
      for (int cb = 0; !flat && cb < xnc; cb += ncol) {
        bool bad = false;
        if (rg < RG && cb + cq < xnc) {
          const int c = xc0 + cb + cq;
          double a0 = 0.0, a1 = 0.0;
          constexpr int kB = kBF;  // 32 XCD members over 3 row groups: one poll round
          for (int j0 = rg; j0 < ng && !bad; j0 += RG * kB) {
            uint32_t off[kB];
            RowG x[kB];
            int n = 0;
#pragma unroll
            for (int u = 0; u < kB; ++u) {
              const int j = j0 + u * RG;
              off[u] = j < ng ? (uint32_t)((size_t)U.xmem[j] * NP2 + c) * kRowPB : 0u;
              n += j < ng;
            }
            bad = !poll_row<kB>(rows_r, off, n, tag, x, ws.ctl, epoch, p.status);
#pragma unroll
            for (int u = 0; u < kB; ++u)
              if (u < n) {
                a0 += (double)row_v0(x[u]);
                a1 += (double)row_v1(x[u]);
              }
          }
          U.red[(rg * ncol + cq) * 2] = a0;
          U.red[(rg * ncol + cq) * 2 + 1] = a1;
        }
        if (__syncthreads_or(bad)) return;
        if (tid < ncol && cb + tid < xnc) {
          double t0 = 0.0, t1 = 0.0;
          for (int r = 0; r < RG; ++r) {
            t0 += U.red[(r * ncol + tid) * 2];
            t1 += U.red[(r * ncol + tid) * 2 + 1];
          }
          st_d2_tagged(xp_r, (uint32_t)(((size_t)xcc * NP2 + xc0 + cb + tid) * 16), t0, t1, tag);
        }
        __syncthreads();
      }
    }
    XA_STAMP(38);

    // ---- B: pair columns [c0, c0 + nc): the fixed-order sum over the G rows, or
    // (two-level) over the XCD partials in XCD order -> g (granules) + f64 sum of squares ----
    double sq = 0.0;
    // pair column c of this block's slice: publish the final value (g granules, the last
    // step's raw gradient, the sum of squares), or -- data parallel -- stage the rank's local
    // value in srow for the cross-rank exchange below
    auto publish = [&](int c, float g0, float g1) {
      const int cc = c0 + c;
      st_row(g_r, (uint32_t)cc * kRowPB, g0, g1, tag, kWt);
      // canonical order for the caller (exchange index -> flat parameter index)
      if (p.grad_out && k == K - 1) {
        if (2 * cc < P) p.grad_out[canon_of_exchange<OBS, A>(2 * cc)] = g0;
        if (2 * cc + 1 < P) p.grad_out[canon_of_exchange<OBS, A>(2 * cc + 1)] = g1;
      }
      if (p.grad_trace) {  // diagnostic: every step's reduced gradient
        float* gt = p.grad_trace + (size_t)k * P;
        if (2 * cc < P) gt[canon_of_exchange<OBS, A>(2 * cc)] = g0;
        if (2 * cc + 1 < P) gt[canon_of_exchange<OBS, A>(2 * cc + 1)] = g1;
      }
      sq += (double)g0 * (double)g0 + (double)g1 * (double)g1;
    };
    auto emit = [&](int c, float g0, float g1) {
      if constexpr (DP) {
        srow[2 * c] = g0;
        srow[2 * c + 1] = g1;
      } else {
        publish(c, g0, g1);
      }
    };
    // few columns, few rows per part: thread (part, c) polls its own column's rows part,
    // part + parts, ... (<= kBF granules, one round trip) and sums them in registers in
    // that order -- the flat path's arithmetic without its LDS staging pass
    const int parts_b = nc <= 128 ? min(4, 256 / max(nc, 1)) : 1;
    const bool col_b = !two_level && nc > 0 && parts_b > 1 && (G + parts_b - 1) / parts_b <= kBF;
    if (col_b) {
      double t0 = 0.0, t1 = 0.0;
      bool bad = false;
      if (tid < parts_b * nc) {
        const int part = tid / nc, c = tid - part * nc;
        uint32_t off[kBF];
        RowG x[kBF];
        int n = 0;
#pragma unroll
        for (int u = 0; u < kBF; ++u) {
          const int r = part + parts_b * u;
          off[u] = r < G ? (uint32_t)((size_t)r * NP2 + c0 + c) * kRowPB : 0u;
          n += r < G;
        }
        bad = !poll_row<kBF>(rows_r, off, n, tag, x, ws.ctl, epoch, p.status);
#pragma unroll
        for (int u = 0; u < kBF; ++u)
          if (u < n) {
            t0 += (double)row_v0(x[u]);
            t1 += (double)row_v1(x[u]);
          }
        U.red[(part * nc + c) * 2] = t0;
        U.red[(part * nc + c) * 2 + 1] = t1;
      }
      if (__syncthreads_or(bad)) return;
      for (int c = tid; c < nc; c += 256) {
        double s0 = 0.0, s1 = 0.0;
        for (int part = 0; part < parts_b; ++part) {
          s0 += U.red[(part * nc + c) * 2];
          s1 += U.red[(part * nc + c) * 2 + 1];
        }
        const float g0 = (float)s0, g1 = (float)s1;
        emit(c, g0, g1);
      }
    }
    // (BF = 1: the host guarantees col_b wherever nc > 0; BF = 2: two_level everywhere)
    constexpr bool flat_ok = BF == 0, gen_ok = BF != 1 && BF != 3;
    const bool flat_b = flat_ok && !col_b && !two_level && G * nc <= 256 * kBF;
    if (nc > 0 && flat_b) {
      const bool bad = gather_rows(rows_r, G, nc, [&](int r) {
        return (uint32_t)((size_t)r * NP2 + c0) * kRowPB;
      }, tag);
      if (__syncthreads_or(bad)) return;
      // few columns: `parts` threads per column sum interleaved rows, combined in part
      // order (a shorter dependent f64 chain; fixed order)
      const int parts = nc <= 128 ? min(4, 256 / nc) : 1;
#ifdef XA_ABL_BSUM
      if (false) {
#else
      if (parts > 1) {
#endif
        if (tid < parts * nc) {
          const int part = tid / nc, c = tid - part * nc;
          double t0 = 0.0, t1 = 0.0;
          for (int r = part; r < G; r += parts) {
            t0 += (double)scr[2 * (r * nc + c)];
            t1 += (double)scr[2 * (r * nc + c) + 1];
          }
          U.red[(part * nc + c) * 2] = t0;
          U.red[(part * nc + c) * 2 + 1] = t1;
        }
        __syncthreads();
      }
      for (int c = tid; c < nc; c += 256) {
        double t0 = 0.0, t1 = 0.0;
#ifdef XA_ABL_BSUM
        if (true) {
          t0 = scr[2 * c]; t1 = scr[2 * c + 1];
        } else
#endif
        if (parts > 1) {
          for (int part = 0; part < parts; ++part) {
            t0 += U.red[(part * nc + c) * 2];
            t1 += U.red[(part * nc + c) * 2 + 1];
          }
        } else {
          for (int r = 0; r < G; ++r) {
            t0 += (double)scr[2 * (r * nc + c)];
            t1 += (double)scr[2 * (r * nc + c) + 1];
          }
        }
        const float g0 = (float)t0, g1 = (float)t1;
        emit(c, g0, g1);
      }
    }
    if (gen_ok && nc > 0 && !flat_b && !col_b) {
      const int SRC = two_level ? kXcds : G;  // sources summed per column
      const int ncol = min(nc, 256), RG = min(SRC, 256 / ncol);
      const int rg = tid / ncol, cq = tid - rg * ncol;
      for (int cb = 0; cb < nc; cb += ncol) {
        bool bad = false;
        if (rg < RG && cb + cq < nc) {
          const int c = c0 + cb + cq;
          double a0 = 0.0, a1 = 0.0;
          constexpr int kB = 8;
          for (int j0 = rg; j0 < SRC && !bad; j0 += RG * kB) {
            uint32_t off[kB];
            int n = 0;
            if (two_level) {
              // one tagged f64 pair per pair column and XCD
              double2 x[kB];
#pragma unroll
              for (int u = 0; u < kB; ++u) off[u] = 0u;
              for (int u = 0; u < kB; ++u) {
                const int xx = j0 + u * RG;
                if (xx < kXcds && U.xn[xx] > 0) off[n++] = (uint32_t)(((size_t)xx * NP2 + c) * 16);
              }
              bad = !poll_d2<kB>(xp_r, off, (1u << n) - 1u, tag, x, ws.ctl, epoch, p.status);
              for (int u = 0; u < n; ++u) {
                a0 += x[u].x;
                a1 += x[u].y;
              }
            } else {
              RowG xr[kB];
#pragma unroll
              for (int u = 0; u < kB; ++u) {
                const int r = j0 + u * RG;
                off[u] = r < G ? (uint32_t)((size_t)r * NP2 + c) * kRowPB : 0u;
                n += r < G;
              }
              bad = !poll_row<kB>(rows_r, off, n, tag, xr, ws.ctl, epoch, p.status);
#pragma unroll
              for (int u = 0; u < kB; ++u)
                if (u < n) {
                  a0 += (double)row_v0(xr[u]);
                  a1 += (double)row_v1(xr[u]);
                }
            }
          }
          U.red[(rg * ncol + cq) * 2] = a0;
          U.red[(rg * ncol + cq) * 2 + 1] = a1;
        }
        if (__syncthreads_or(bad)) return;
        if (tid < ncol && cb + tid < nc) {
          double t0 = 0.0, t1 = 0.0;
          for (int r = 0; r < RG; ++r) {
            t0 += U.red[(r * ncol + tid) * 2];
            t1 += U.red[(r * ncol + tid) * 2 + 1];
          }
          const float g0 = (float)t0, g1 = (float)t1;
          emit(cb + tid, g0, g1);
        }
        __syncthreads();
      }
    }
    if constexpr (DP) {
      // push this rank's slice to every rank (parity k & 1), then read every rank's slice
      // from the own block and sum in rank order (f64) -> the union's gradient slice
      __syncthreads();  // srow holds the local slice
      const int par = k & 1;
      for (int c = tid; c < nc; c += 256) {
        const size_t o = dl.gsl + ((((size_t)par * G + b) * W + p.dp_rank) * CB0 + c) * 16;
        const uint32_t w0 = __float_as_uint(srow[2 * c]), w1 = __float_as_uint(srow[2 * c + 1]);
        for (int q = 0; q < W; ++q) {
          dp_st(p.dp_blocks[q], o, w0, tag);
          dp_st(p.dp_blocks[q], o + 8, w1, tag);
        }
      }
      bool bad = false;
      for (int c = tid; c < nc; c += 256) {
        constexpr int kW2 = 2 * XA_PPO_DP_MAX;
        size_t off[kW2];
        uint32_t x[kW2];
#pragma unroll
        for (int u = 0; u < kW2; ++u) {
          const int r = u >> 1;
          off[u] = r < W ? dl.gsl + ((((size_t)par * G + b) * W + r) * CB0 + c) * 16 + 8 * (u & 1)
                         : 0;
        }
        bad = bad || !dp_poll<kW2>(p.dp_blocks[p.dp_rank], off, 2 * W, tag, x, ws.ctl, epoch,
                                   p.status);
        double s0 = 0.0, s1 = 0.0;
        for (int r = 0; r < W; ++r) {
          s0 += (double)__uint_as_float(x[2 * r]);
          s1 += (double)__uint_as_float(x[2 * r + 1]);
        }
        publish(c, (float)s0, (float)s1);
      }
      if (__syncthreads_or(bad)) return;
    }
    (void)sq;
    XA_STAMP(40);
    XA_TRACE_PT(b, k, 3);

    // ---- C: the g slice of this thread's parameters and the G norm partials (granules of
    // one buffer, one poll), global norm (identical in every wave of every block), clip +
    // Keras Adam ----
    float gw[16], gr[RPT];
    double tot = 0.0;
    bool bad = false;
    // the gradient-free half of the Adam moment updates, before the poll (its loads and
    // multiplies leave the critical path): b1 m and b2 v of the thread's slots
    float bm[4 * NQ4], bv[4 * NQ4];
#pragma unroll
    for (int q4 = 0; q4 < NQ4; ++q4) {
      const float4 a = U.mv4[0][q4][tid], c = U.mv4[1][q4][tid];
      const xa_f2 b1 = {p.adam.beta1, p.adam.beta1}, b2 = {p.adam.beta2, p.adam.beta2};
      const xa_f2 m01 = xa_f2{a.x, a.y} * b1, m23 = xa_f2{a.z, a.w} * b1;
      const xa_f2 v01 = xa_f2{c.x, c.y} * b2, v23 = xa_f2{c.z, c.w} * b2;
      bm[4 * q4] = m01.x; bm[4 * q4 + 1] = m01.y; bm[4 * q4 + 2] = m23.x; bm[4 * q4 + 3] = m23.y;
      bv[4 * q4] = v01.x; bv[4 * q4 + 1] = v01.y; bv[4 * q4 + 2] = v23.x; bv[4 * q4 + 3] = v23.y;
    }
    {
      // the thread's g values: 8 W2 pairs (exchange order: pairs 256 h + tid, coalesced) and
      // its rest pairs, as tagged pairs in one poll
      constexpr int NG = 8 + RPT;
      uint32_t off[NG];
      RowG x[NG];
#pragma unroll
      for (int h = 0; h < 8; ++h) off[h] = (uint32_t)((256 * h + tid) * kRowPB);
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        off[8 + q] = (uint32_t)((ps.rx[q] >= 0 ? ps.rx[q] / 2 : 0) * kRowPB);
      bad = !poll_row<NG>(g_r, off, NG, tag, x, ws.ctl, epoch, p.status);
      XA_STAMP(46);
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        gw[2 * h] = row_v0(x[h]);
        gw[2 * h + 1] = row_v1(x[h]);
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        gr[q] = ps.rx[q] >= 0 ? ((ps.rx[q] & 1) ? row_v1(x[8 + q]) : row_v0(x[8 + q])) : 0.0f;
    }
    {
      // the block holds all of g (each parameter on exactly one thread): its own f64 sum of
      // squares in a fixed thread / wave order, identical in every block
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        s0 = fma((double)gw[q], (double)gw[q], s0);
        s1 = fma((double)gw[q + 1], (double)gw[q + 1], s1);
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) s0 = fma((double)gr[q], (double)gr[q], s0);
      const double ws = xa_wave_sum_f64(s0 + s1);
      if (lane == 0) U.wsum[w] = ws;
    }
    if (__syncthreads_or(bad)) return;
    XA_STAMP(47);
    XA_TRACE_PT(b, k, 4);
#ifndef XA_ABL_CNORM
    tot = (U.wsum[0] + U.wsum[1]) + (U.wsum[2] + U.wsum[3]);
    // tf.clip_by_global_norm's scale clip * min(1 / norm, 1 / clip), on the hardware sqrt /
    // reciprocal units (the update is checked against float64 with a tolerance)
    const float gn = __builtin_amdgcn_sqrtf((float)tot);
    const float sc = p.adam.clip_norm > 0.0f
                         ? p.adam.clip_norm * fminf(frcp(gn), frcp(p.adam.clip_norm)) : 1.0f;
#else
    const float sc = (float)tot;
#endif
    const float alpha = U.alpha[k];
#ifndef XA_ABL_ADAM
    {
      // m' = b1 m + (1 - b1) sc g, v' = b2 v + (1 - b2) sc^2 g^2 (Keras ApplyAdam on the
      // clipped gradient sc g, regrouped: the update is checked against float64 with a
      // tolerance), theta -= alpha m' / (sqrt(v') + eps)
      const xa_f2 k1 = {sc * omb1, sc * omb1}, k2 = {(sc * sc) * omb2, (sc * sc) * omb2};
      const xa_f2 al = {alpha, alpha}, ep = {p.adam.eps, p.adam.eps};
      float th[4 * NQ4];
#pragma unroll
      for (int q = 0; q < 4 * NQ4; ++q) th[q] = q < 16 ? wv[q] : q < NS ? rv[q - 16] : 0.0f;
#pragma unroll
      for (int q = 0; q < NS; q += 2) {
        const xa_f2 g = {q < 16 ? gw[q] : gr[q - 16], q + 1 < 16 ? gw[q + 1] : q + 1 < NS ? gr[q + 1 - 16] : 0.0f};
        const xa_f2 mn = xa_fma2(g, k1, xa_f2{bm[q], bm[q + 1]});
        const xa_f2 vn = xa_fma2(g * g, k2, xa_f2{bv[q], bv[q + 1]});
        const xa_f2 step = mn * al;
        const xa_f2 den = xa_f2{__builtin_amdgcn_sqrtf(vn.x), __builtin_amdgcn_sqrtf(vn.y)} + ep;
        const xa_f2 r = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
        const xa_f2 tn = xa_fma2(-step, r, xa_f2{th[q], th[q + 1]});
        th[q] = tn.x;
        th[q + 1] = tn.y;
        bm[q] = mn.x;
        bm[q + 1] = mn.y;
        bv[q] = vn.x;
        bv[q + 1] = vn.y;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) wv[q] = th[q];
#pragma unroll
      for (int q = 0; q < RPT; ++q) rv[q] = th[16 + q];
#pragma unroll
      for (int q4 = 0; q4 < NQ4; ++q4) {
        U.mv4[0][q4][tid] = make_float4(bm[4 * q4], bm[4 * q4 + 1], bm[4 * q4 + 2], bm[4 * q4 + 3]);
        U.mv4[1][q4][tid] = make_float4(bv[4 * q4], bv[4 * q4 + 1], bv[4 * q4 + 2], bv[4 * q4 + 3]);
      }
    }
#endif
#ifndef XA_ABL_LDS
    ps.to_lds(L, wv, rv);
#endif
    XA_STAMP(43);
    XA_TRACE_PT(b, k, 5);
  }
  XA_TRACE_CLK(b, 1);
  XA_TRACE_FLUSH(b);
  if (b == 0 && tid == 0) {
    // zero the election slot of the next launch (this launch's slot is par; launch
    // gen + 1 uses par ^ 1, which launch gen - 1 used and nothing touches now)
    for (int x = 0; x < kXcds; ++x)
      __hip_atomic_store((gu32*)(ws.ctl + kElect + (par ^ 1u) * kXcds + x), 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32*)(ws.ctl + kWin + (par ^ 1u)), 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  // theta / m / v out: every block holds the same final values, so block b stores the
  // slices of threads tid = b, b + G, ... (all blocks share the stores instead of block 0
  // issuing every one of them at the launch's end); block 0 alone the counters
  if (tid % G == b % 256) {
    ps.store(p.theta, wv, rv);
    float mw[16], mr[RPT], vw[16], vr[RPT];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const float4 a = U.mv4[0][q >> 2][tid], c = U.mv4[1][q >> 2][tid];
      const float mq = (q & 3) == 0 ? a.x : (q & 3) == 1 ? a.y : (q & 3) == 2 ? a.z : a.w;
      const float vq = (q & 3) == 0 ? c.x : (q & 3) == 1 ? c.y : (q & 3) == 2 ? c.z : c.w;
      if (q < 16) {
        mw[q] = mq;
        vw[q] = vq;
      } else {
        mr[q - 16] = mq;
        vr[q - 16] = vq;
      }
    }
    ps.store(p.adam_m, mw, mr);
    ps.store(p.adam_v, vw, vr);
  }
  if (b == 0) {
    if (tid == 0) {
      *p.adam_step = t0 + K;
      // every block read the counter before its last gradient row, which block 0 has
      // consumed by now (phase B of the last step)
      if (p.bump_counter && p.shuffle.rng_counter)
        *const_cast<uint64_t*>(p.shuffle.rng_counter) = ctr + 1;
      // the next launch's generation, write-through (read at its start on every XCD)
      __hip_atomic_store((gu32*)ws.persist, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// resident capacity (blocks of one launch that are co-resident), per device: the
// minimum occupancy over every variant launch() may pick
template <int OBS, int A>
int occupancy_min() {
  void* const kernels[] = {
      (void*)ppo_update_kernel<OBS, A, S, false, false>, (void*)ppo_update_kernel<OBS, A, 16, false, false>,
      (void*)ppo_update_kernel<OBS, A, S, true, false>, (void*)ppo_update_kernel<OBS, A, 16, true, false>,
      (void*)ppo_update_kernel<OBS, A, S, false, true>, (void*)ppo_update_kernel<OBS, A, 16, false, true>,
      (void*)ppo_update_kernel<OBS, A, S, true, true>, (void*)ppo_update_kernel<OBS, A, 16, true, true>,
      (void*)ppo_update_kernel<OBS, A, 16, false, false, 1>,
      (void*)ppo_update_kernel<OBS, A, 16, true, false, 1>,
      (void*)ppo_update_kernel<OBS, A, 16, false, true, 1>,
      (void*)ppo_update_kernel<OBS, A, 16, true, true, 1>,
      (void*)ppo_update_kernel<OBS, A, 16, false, true, 3>,
      (void*)ppo_update_kernel<OBS, A, S, false, true, 4>,
      (void*)ppo_update_kernel<OBS, A, 16, true, true, 3>,
      (void*)ppo_update_kernel<OBS, A, S, true, true, 4>,
      (void*)ppo_update_kernel<OBS, A, S, false, false, 2>,
      (void*)ppo_update_kernel<OBS, A, S, true, false, 2>,
      (void*)ppo_update_kernel<OBS, A, S, false, true, 2>,
      (void*)ppo_update_kernel<OBS, A, S, true, true, 2>};
  // (template flags: DP, PRE, BF)
  int occ = 1 << 30;
  for (void* k : kernels) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, 256, 0) != hipSuccess) return 0;
    occ = min(occ, o);
  }
  return occ;
}

template <int OBS, int A>
int capacity() {
  static int cap[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cap[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    cap[dev] = cus * occupancy_min<OBS, A>();
  }
  return cap[dev];
}


// samples per tile: 16 when there are more blocks than 32-sample tiles of a minibatch
// (xa_ppo_update_blocks picks that for minibatches of <= 16 such tiles), else 32
int tile_samples(int mb_size, int G) { return G > (mb_size + S - 1) / S ? 16 : S; }

// XCD-local mode (elect_local): small grids (one level, G <= 32 at one block per CU), when
// kXcds G blocks are co-resident; data-parallel launches only when every rank owns its GPU
// (ranks sharing one GPU could strand each other's elections). XA_PPO_LOCAL=0 disables it.
bool use_local(const XaPpoUpdateArgs* a, int G, int cap) {
  static const int env = [] {
    const char* e = getenv("XA_PPO_LOCAL");
    return e && e[0] == '0' ? 0 : 1;
  }();
  if (!env || a->placement == XA_PPO_PLACE_SPREAD) return false;
  if (a->dp_world > 1 && a->placement != XA_PPO_PLACE_LOCAL) return false;
  return G < kTwoLevelMinG && (long)G * kXcds <= (long)cap;
}

// every block's phase-B slice (pair columns [b CB, (b + 1) CB) of NP2) takes the kernel's
// column form -- the kernel's own col_b test, per block (single-level reduce only)
bool col_b_everywhere(int G, int P) {
  const int NP2 = padded(P) / 2, CB = (NP2 + G - 1) / G;
  for (int b = 0; b < G; ++b) {
    const int c0 = min(NP2, b * CB), nc = min(NP2, c0 + CB) - c0;
    if (nc <= 0) continue;
    const int parts = nc <= 128 ? min(4, 256 / nc) : 1;
    if (!(parts > 1 && (G + parts - 1) / parts <= kBF)) return false;
  }
  return true;
}

template <int OBS, int A, int TS>
void launch_ts(const XaPpoUpdateArgs* a, int G, bool dp, bool loc, const Ws& ws, int K, int n_mb,
               hipStream_t s) {
  const dim3 grid(loc ? G * kXcds : G);
  // the tile inputs of every step fit the block's LDS records (same test as the kernel's)
  const int n_tiles_max = (min(a->mb_size, a->batch) + TS - 1) / TS;
  const int TPB = (n_tiles_max + G - 1) / G;
  const bool pre = K * TPB * TS <= pre_max<OBS>();
  const int l = loc ? 1 : 0;
  // the fixed-shape instantiations (BF 3 / 4) for exactly their shape; XA_PPO_FIXED_SHAPE=0
  // forces the generic ones (A/B)
  static const bool fix_on = [] {
    const char* e = getenv("XA_PPO_FIXED_SHAPE");
    return !(e && e[0] == '0');
  }();
  auto is_fix = [&](auto fs) {
    typedef decltype(fs) F;
    return fix_on && pre && G == F::G && K == F::K && n_mb == F::NMB && a->batch == F::B &&
           a->mb_size == F::MB;
  };
  if constexpr (TS == 16) {  // 16-sample tiles: small grids, one-level reduce
    if (col_b_everywhere(G, offs(OBS, A).P)) {
      if (is_fix(FixShape<3>{}) && dp)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, true, 3>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (is_fix(FixShape<3>{}))
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, true, 3>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (dp && pre)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, true, 1>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (dp)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, false, 1>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (pre)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, true, 1>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, false, 1>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      return;
    }
  } else {  // 32-sample tiles on a spread grid of >= kTwoLevelMinG blocks: two-level only
    if (!loc && G >= kTwoLevelMinG) {
      if (is_fix(FixShape<4>{}) && dp)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, true, 4>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (is_fix(FixShape<4>{}))
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, true, 4>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (dp && pre)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, true, 2>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (dp)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, false, 2>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else if (pre)
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, true, 2>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      else
        hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, false, 2>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
      return;
    }
  }
  if (dp && pre)
    hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, true>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
  else if (dp)
    hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, true, false>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
  else if (pre)
    hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, true>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
  else
    hipLaunchKernelGGL((ppo_update_kernel<OBS, A, TS, false, false>), grid, dim3(256), 0, s, *a, ws, K, n_mb, l);
}

template <int OBS, int A>
int launch(const XaPpoUpdateArgs* a, int G, int K, int n_mb, hipStream_t s) {
  const int P = offs(OBS, A).P;
  const Ws ws = carve(a->workspace, G, P, K);
  const bool loc = use_local(a, G, capacity<OBS, A>());
  if (tile_samples(a->mb_size, G) == 16)
    launch_ts<OBS, A, 16>(a, G, a->dp_world > 1, loc, ws, K, n_mb, s);
  else
    launch_ts<OBS, A, S>(a, G, a->dp_world > 1, loc, ws, K, n_mb, s);
  XA_CHECK_LAUNCH("xa_ppo_update");
  return 0;
}

}  // namespace

// the capacity / launch entry points of one (obs, actions) shape's instantiations, defined
// in that shape's translation unit (ppo_update_oXY.hip) and dispatched by ppo_update.hip
#define XA_PPO_SHAPE_TU(O, A_)                                                               \
  int xa_ppo_capacity_##O##_##A_() { return capacity<O, A_>(); }                            \
  int xa_ppo_launch_##O##_##A_(const XaPpoUpdateArgs* a, int G, int K, int n_mb,            \
                               hipStream_t s) {                                             \
    return launch<O, A_>(a, G, K, n_mb, s);                                                  \
  }
#define XA_PPO_SHAPE_DECL(O, A_)          \
  int xa_ppo_capacity_##O##_##A_();       \
  int xa_ppo_launch_##O##_##A_(const XaPpoUpdateArgs* a, int G, int K, int n_mb, hipStream_t s);

