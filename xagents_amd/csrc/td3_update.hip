// TD3 / DDPG gradient step in ONE persistent launch (xa_td3_update): the sample gather,
// both critics' forward / TD head / backward / Keras Adam and, on policy-delay steps, the
// actor's forward / -mean Q backward through the UPDATED critic 1 / Keras Adam and the
// Polyak sync of every target network. Replaces DDPG.update_critic_weights +
// update_actor_weights + sync_target_models (xagents/ddpg/agent.py:73-147) and TD3's twin
// critic / target-smoothing update (xagents/td3/agent.py:66-110) -- at batch 64 those are
// ~90 small launches of 4-12 us each (profiles/r04a_c5_grad_step_kernel_shapes.txt).
//
// Networks: the 3-layer MLPs of the .cfg models (in -> H1 relu -> H2 relu -> out; the
// actor's output tanh, the critics' linear), parameters in Keras order (W1 [in][H1], b1,
// W2 [H1][H2], b2, W3 [H2][out], b3), batch rows r = the sampled transitions.
//
// G resident workgroups of 256 threads run the phases below; a phase's jobs are dealt
// round-robin (job j -> workgroup j mod G) and a grid barrier separates the phases. A
// forward / input-gradient job is one 32-row x 16-column output tile: both operands staged
// in LDS by LDS-DMA (zero padded to a multiple of 16 along K), wave w computes rows
// 16 (w & 1) .. + 15 over half w >> 1 of the k chunks on v_mfma_f32_16x16x4f32 (lane (i, q)
// reads k0 + 4q .. 4q + 3 of its row / column as one float4, component s feeding MFMA step
// s: one consistent k order for A and B), the halves summed in LDS. A weight-gradient job
// is 64 in-features x up to 4 column tiles of 16 sharing the staged A.
//   P1  L1 forward: target actor (s'), critic 1 / 2 ([s, a]), actor (s, policy steps)
//   P2  L2 forward of the same networks, + each tile's partial of the narrow L3 product;
//       the last job of a row tile finishes L3: target actor tanh (+ TD3 smoothing noise,
//       clip) -> a'; critics -> v1, v2; actor tanh -> pi(s)
//   P4  target critics L1 on [s', a'];  P5  L2 (+ the L3 partials; the row tile's last job
//       runs the TD head y = r + (1 - d) gamma min(tv1, tv2), dv = 2 (v - y) (MSE) or
//       clip(v - y, +-delta) (opt-in Huber), per-sample loss)
//   P7  critics backward: dW2 / db2 (dZ2 = dv W3^T gate(h2) formed while staging), dH1,
//       dW3 / db3
//   P8  critics: dW1 / db1 with the Keras Adam step applied in the same job, Adam of every
//       other critic parameter (+ Polyak of the critic targets on policy steps)
//   policy steps only:
//   P9  critic 1 L1 on [s, pi(s)] (updated critic 1);  P10 L2
//   P11 dH1 of -mean Q (dZ2 = -W3^T gate(h2) / B), + the partials of d pi = dH1 W1[s..s+A]^T;
//       the row tile's last job forms the actor's output gradient d pi (1 - pi^2)
//   P13 actor backward: dW2 / db2, dH1, dW3 / db3
//   P14 actor dW1 / db1 + Adam + Polyak, Adam + Polyak of the other actor parameters
// (the phases once numbered P3, P6 and P12 -- the narrow L3 / TD-head / d pi products --
// run as the row tiles' last jobs of P2, P5 and P11: a ticket per row tile, no barrier)
// Hand-offs follow MI355X_MICROARCH.md's visibility table row 1: every in-launch produced
// word (activations, gradients, updated parameters) is stored write-through (sc1) and
// loaded with sc1 loads; a barrier drains (vmcnt 0), joins the workgroup and ONE lane adds
// to an agent-scope counter that ONE lane polls. The counter is never reset: the workspace
// keeps the value the previous launch left (`base`), so graph replays need no memset.
#include <math.h>

#include "../../include/xagents_hip.h"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kRsrcWord3 = 0x00020000;  // raw buffer, gfx9-family resource word 3
constexpr int kAuxSc1 = 16;             // buffer instruction aux bits: write-through (sc1)
constexpr uint64_t kSpinTicks = 1000000000;  // 10 s of the 100 MHz wall clock per barrier
constexpr int kRows = 64, kCols = 16;   // weight-gradient / narrow job rows, tile columns
constexpr int kTR = 32;                 // rows of a forward / input-gradient job
constexpr int kMaxK = 416;              // largest GEMM depth (H1, H2, batch, in)
constexpr int kAux = 2048 + 1024;       // LDS floats: W3 slice + dZ3 rows of the dZ2 former

XA_DEV f32x4v mfma4(float a, float b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- write-through hand-off accesses ----
XA_DEV float ldc(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
XA_DEV void stc(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (the base is made wave-uniform explicitly: a buffer resource lives in scalar registers)
XA_DEV __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  const uint64_t u = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* ub = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFF0, kRsrcWord3);
}
XA_DEV float4 ld4c(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAuxSc1);
  return make_float4(v[0], v[1], v[2], v[3]);
}
// 16 bytes through the cache hierarchy (parameters no phase of this launch has written yet)
XA_DEV float4 ld4p(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return make_float4(v[0], v[1], v[2], v[3]);
}
// plain loads / stores through the GLOBAL address space: a generic (flat) access in an
// out-of-line function would also count on lgkmcnt, so every later LDS wait would wait for it
typedef __attribute__((address_space(1))) float gf32;
typedef __attribute__((address_space(1))) f32x4v gv4;
XA_DEV float ldg(const float* p) { return *(const gf32*)p; }
XA_DEV void stg(float* p, float v) { *(gf32*)p = v; }
XA_DEV float4 ldg4(const float* p) {
  const f32x4v v = *(const gv4*)p;
  return make_float4(v[0], v[1], v[2], v[3]);
}
XA_DEV void stg4(float* p, float4 v) { *(gv4*)p = f32x4v{v.x, v.y, v.z, v.w}; }
XA_DEV float ldw(const float* p, bool coh) { return coh ? ldc(p) : ldg(p); }
// one 16-B write-through store (a vector store)
XA_DEV void st4c(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, f32x4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, kAuxSc1);
}

XA_DEV float philox_normal(uint32_t i, uint32_t j, uint64_t ctr, uint64_t seed) {
  // the same draw as xa_noisy_actions (offpolicy.hip)
  const xa_u4 r = xa_philox(i, j, (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)seed,
                            (uint32_t)(seed >> 32));
  const float u1 = ((float)(r.x >> 8) + 1.0f) * 5.9604644775390625e-08f;
  const float u2 = (float)(r.y >> 8) * 5.9604644775390625e-08f;
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// ---- network views ----
struct Net {
  float* th;
  float* m;
  float* v;
  int in, out;
  int w1, b1, w2, b2, w3, b3, P;
  float alpha;  // Adam step size of this launch's step (online networks)
};

XA_DEV Net make_net(const XaTdNet& d, int in, int H1, int H2, int out, bool adam) {
  Net n;
  n.th = d.theta;
  n.m = d.m;
  n.v = d.v;
  n.in = in;
  n.out = out;
  n.w1 = 0;
  n.b1 = in * H1;
  n.w2 = n.b1 + H1;
  n.b2 = n.w2 + H1 * H2;
  n.w3 = n.b2 + H2;
  n.b3 = n.w3 + H2 * out;
  n.P = n.b3 + out;
  n.alpha = adam ? adam_alpha(d.lr, d.beta1, d.beta2, *d.step + 1) : 0.0f;
  return n;
}

// A row source: row r of X = [src0 row | src1 row] (src1 optional), each source either a
// dense [rows][ld] buffer or a replay ring addressed through the sample slots
struct XSrc {
  const float* p0;
  int w0, ld0;
  bool slot0, coh0;
  const float* p1;
  int w1, ld1;
  bool slot1, coh1;
};
XA_DEV XSrc xsrc(const float* p, int w, int ld, bool slot, bool coh) {
  XSrc x;
  x.p0 = p;
  x.w0 = w;
  x.ld0 = ld;
  x.slot0 = slot;
  x.coh0 = coh;
  x.p1 = nullptr;
  x.w1 = 0;
  x.ld1 = 0;
  x.slot1 = false;
  x.coh1 = false;
  return x;
}
XA_DEV XSrc xcat(XSrc a, const float* p, int w, int ld, bool slot, bool coh) {
  a.p1 = p;
  a.w1 = w;
  a.ld1 = ld;
  a.slot1 = slot;
  a.coh1 = coh;
  return a;
}
// the batch's ring rows, copied to LDS at launch start (read per element by xload)
__shared__ int64_t td3_slots[256];

XA_DEV float xload(const XSrc& x, const int64_t* slots, int r, int k) {
  (void)slots;
  if (k < x.w0) {
    const int64_t row = x.slot0 ? td3_slots[r] : r;
    const float* p = x.p0 + row * x.ld0 + k;
    return x.coh0 ? ldc(p) : ldg(p);
  }
  const int64_t row = x.slot1 ? td3_slots[r] : r;
  const float* p = x.p1 + row * x.ld1 + (k - x.w0);
  return x.coh1 ? ldc(p) : ldg(p);
}

// A gradient source dZ [rows][cols]: a dense buffer (ld), or the layer-2 output gradient
// formed on the fly: dZ[r][k] = (sum_a d3[r][a] W3[k][a]) (h2[r][k] > 0), with d3 [rows][n3]
// (or the constant c3 when d3 is null: the actor loss -mean Q gives -1 / B)
struct DZ {
  const float* buf;
  int ld;
  const float* h2;
  int H2;
  const float* w3;
  int n3;
  const float* d3;
  float c3;
};
XA_DEV DZ dz_buf(const float* p, int ld) {
  DZ d;
  d.buf = p;
  d.ld = ld;
  d.h2 = nullptr;
  d.H2 = 0;
  d.w3 = nullptr;
  d.n3 = 0;
  d.d3 = nullptr;
  d.c3 = 0.0f;
  return d;
}
XA_DEV DZ dz_h2(const float* h2, int H2, const float* w3, int n3, const float* d3, float c3) {
  DZ d;
  d.buf = nullptr;
  d.ld = H2;
  d.h2 = h2;
  d.H2 = H2;
  d.w3 = w3;
  d.n3 = n3;
  d.d3 = d3;
  d.c3 = c3;
  return d;
}

struct Lds {
  float* A;    // 64 x Kp floats: chunked rows (CR) or k-major rows of 64 (KM)
  float* B;    // 16 x Kp floats: CR (16 rows) or k-major rows of 16 (KM)
  float* aux;  // [kAux]
};
// the dynamic LDS of the launch (named at file scope so the out-of-line job functions
// address it directly as LDS)
extern __shared__ __attribute__((aligned(16))) float td3_smem[];
XA_DEV Lds lds() {
  return Lds{td3_smem, td3_smem + kRows * kMaxK, td3_smem + (kRows + kCols) * kMaxK};
}

XA_DEV int pad16(int k) { return (k + 15) & ~15; }
// the two k halves of a forward / input-gradient tile, row-major [kTR][16] each
__shared__ __attribute__((aligned(16))) float td3_part[2 * 32 * 16];

// (diagnostic) block 0 stamps the wall clock at points of the first job of every phase into
// the workspace's detail trace (tools/td3_grad_steps.py): slot 8 p + point
// (diagnostic builds only: -DXA_TD3_TRACE=1, tools/build_variant.py; a trace store in the
// product would hold block 0 one store round trip at every barrier, so the product build
// compiles no trace code at all)
#ifndef XA_TD3_TRACE
#define XA_TD3_TRACE 0
#endif
#if XA_TD3_TRACE
__shared__ int td3_dslot;
__shared__ unsigned long long* td3_dbuf;
XA_DEV void dstamp(int point) {
  if (threadIdx.x == 0 && td3_dslot >= 0)
    *((__attribute__((address_space(1))) unsigned long long*)td3_dbuf + td3_dslot + point) =
        wall_clock64();
}
#define XA_TD3_DSLOT(v) \
  do {                  \
    if (threadIdx.x == 0) td3_dslot = (v); \
  } while (0)
#define XA_TD3_CLOCK(dst) ((dst) = wall_clock64())
#else
#define dstamp(point) ((void)0)
#define XA_TD3_DSLOT(v) ((void)0)
#define XA_TD3_CLOCK(dst) ((void)0)
#endif

// Operand layouts in LDS (both written by LDS-DMA, 1 KB per wave instruction):
//   CR  chunked rows: element (row r, k) at (k / 16 * nrow + r) * 16 + k % 16 -- a 16-row x
//       16-k chunk is one DMA instruction; MFMA lane (i, q) reads k0 + 4q .. + 3 of its row as
//       one float4 (the 64 lanes read 1 KB of consecutive 16-B slots)
//   KM  k-major: element (k, c) at k * width + c (width 64 or 16) -- rows of the global
//       matrix as they lie; MFMA lane (i, q) reads element (k0 + 4q + s, i) for step s
XA_DEV int cr_idx(int r, int k, int nrow) { return ((k >> 4) * nrow + r) * 16 + (k & 15); }

typedef __attribute__((address_space(3))) void lds_void;
constexpr uint32_t kOob = 0xFFFFFFF0u;  // a buffer offset past every range: the DMA lands zeros

XA_DEV __amdgpu_buffer_rsrc_t rsrc_dma(const void* base) {
  const uint64_t u = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* ub = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFF0, kRsrcWord3);
}
// one wave instruction: 64 lanes x 16 B into LDS at dst (wave-uniform) + 16 lane
XA_DEV void dma16(__amdgpu_buffer_rsrc_t r, float* dst, uint32_t voff, bool coh) {
  lds_void* d = (lds_void*)dst;
  if (coh) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, d, 16, voff, 0, 0, kAuxSc1);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, d, 16, voff, 0, 0, 0);
}
XA_DEV void dma_wait() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// (the row map is the block's LDS slot table td3_slots, filled once at the launch start: the
// sampled slots may live in mapped host memory, read once per block; it is read BEFORE the
// first DMA is issued)

// CR tile of nrow (64 / 16) rows: tile row r = source row (rowmap ? rowmap[r] : r0 + r) of a
// row-major matrix (ld floats, K % 4 == 0 and ld % 4 == 0), k < K; rows >= vrows and k >= K
// are zeros up to Kp
XA_DEV void dma_cr(float* dst, int nrow, const float* base, int64_t ld, int r0,
                   const int64_t* rowmap, int vrows, int K, int Kp, bool coh) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_dma(base);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nrb = nrow >> 4, ninst = nrb * (Kp >> 4);
  const int rr = lane >> 2, kk = 4 * (lane & 3);
  int64_t gr[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int row = 16 * rb + rr;
    gr[rb] = (rb < nrb && row < vrows) ? (rowmap ? rowmap[row] : (int64_t)(r0 + row)) : -1;
  }
  for (int t = w; t < ninst; t += 4) {
    const int kc = t / nrb, rb = t - kc * nrb, k = 16 * kc + kk;
    const int64_t g = rb == 0 ? gr[0] : rb == 1 ? gr[1] : rb == 2 ? gr[2] : gr[3];
    const uint32_t voff = (g >= 0 && k < K) ? (uint32_t)((g * ld + k) * 4) : kOob;
    dma16(rs, dst + (kc * nrow + 16 * rb) * 16, voff, coh);
  }
}

constexpr int kKmMax = 16;  // k-major DMA instructions per wave with a row map (batch <= 256)

// KM tile of width wd (64 / 16) floats: row k = source row (rowmap ? rowmap[k] : k) columns
// c0 .. c0 + wd (ld % 4 == 0, c0 % 4 == 0), k < vK, column < vc (vc % 4 == 0); zeros elsewhere
// up to Kp rows
XA_DEV void dma_km(float* dst, int wd, const float* base, int64_t ld, int c0,
                   const int64_t* rowmap, int vK, int vc, int Kp, bool coh) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_dma(base);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int per = wd >> 2, rows_per = 64 / per, ninst = Kp / rows_per;
  const int kr = lane / per, c = 4 * (lane - kr * per);
  if (rowmap) {
    int64_t gr[kKmMax];
#pragma unroll
    for (int m = 0; m < kKmMax; ++m) {
      const int k = (w + 4 * m) * rows_per + kr;
      gr[m] = (w + 4 * m < ninst && k < vK) ? rowmap[k] : -1;
    }
#pragma unroll
    for (int m = 0; m < kKmMax; ++m) {
      const int t = w + 4 * m;
      if (t < ninst) {
        const uint32_t voff = (gr[m] >= 0 && c < vc) ? (uint32_t)((gr[m] * ld + c0 + c) * 4) : kOob;
        dma16(rs, dst + t * 256, voff, coh);
      }
    }
    return;
  }
  for (int t = w; t < ninst; t += 4) {
    const int k = t * rows_per + kr;
    const uint32_t voff = (k < vK && c < vc) ? (uint32_t)(((int64_t)k * ld + c0 + c) * 4) : kOob;
    dma16(rs, dst + t * 256, voff, coh);
  }
}

// scalar loads into registers (concatenated or gathered rows the DMA cannot take), all issued
// before the first LDS write: element (a, b) of an na x nb grid, value x(a, b) when a < va and
// b < vb (else 0), dst(a, b, v)
template <class Ld, class Dst>
XA_DEV void sload(int na, int nb, int va, int vb, Ld ld, Dst dst) {
  constexpr int kS = 16;
  const int total = na * nb;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * kS) {
    float v[kS];
#pragma unroll
    for (int u = 0; u < kS; ++u) {
      const int e = e0 + 256 * u, a = e / nb, b = e - a * nb;
      v[u] = (e < total && a < va && b < vb) ? ld(a, b) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kS; ++u) {
      const int e = e0 + 256 * u, a = e / nb, b = e - a * nb;
      if (e < total) dst(a, b, v[u]);
    }
  }
}

// [src0 | src1] rows as float4 quads (every width and ld a multiple of 4): quad q of an
// nr x (Kp / 4) grid, tile row r (source row r0 + r, through the slots for ring sources)
// and features k0 + k .. + 3 (k < K; zeros for r >= vr, k >= K), all of a thread's loads
// issued before its first LDS write. Ring rows are plain 16-B loads (64-bit addresses);
// in-launch hand-off sources are 16-B sc1 buffer loads
XA_DEV bool quad_src(const XSrc& x, int k0) {
  return (x.w0 & 3) == 0 && (x.ld0 & 3) == 0 && (k0 & 3) == 0 &&
         (x.p1 == nullptr || ((x.w1 & 3) == 0 && (x.ld1 & 3) == 0));
}
template <class Dst>
XA_DEV void xgather4(const XSrc& x, int r0, int nr, int vr, int k0, int K, int Kp, Dst dst) {
  constexpr int kQ = 4;
  const __amdgpu_buffer_rsrc_t rs0 = rsrc(x.p0), rs1 = rsrc(x.p1 ? x.p1 : x.p0);
  const int nq = Kp >> 2, total = nr * nq;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * kQ) {
    f32x4v v[kQ];
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const int e = e0 + 256 * u, r = e / nq, k = 4 * (e - r * nq);
      v[u] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      if (e < total && r < vr && k < K) {
        const int f = k0 + k;
        const bool first = f < x.w0;
        const float* pb = first ? x.p0 : x.p1;
        const bool slot = first ? x.slot0 : x.slot1, coh = first ? x.coh0 : x.coh1;
        const int ld = first ? x.ld0 : x.ld1, c = first ? f : f - x.w0;
        const int64_t row = slot ? td3_slots[r0 + r] : (int64_t)(r0 + r);
        if (coh) {
          const uint32_t off = (uint32_t)((row * ld + c) * 4);
          v[u] = first ? __builtin_amdgcn_raw_buffer_load_b128(rs0, off, 0, kAuxSc1)
                       : __builtin_amdgcn_raw_buffer_load_b128(rs1, off, 0, kAuxSc1);
        } else {
          v[u] = *(const gv4*)(pb + row * ld + c);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const int e = e0 + 256 * u, r = e / nq, k = 4 * (e - r * nq);
      if (e < total) dst(r, k, v[u]);
    }
  }
}

XA_DEV bool dma_src(const XSrc& x) {
  return x.p1 == nullptr && (x.w0 & 3) == 0 && (x.ld0 & 3) == 0;
}

// the dZ2 former's LDS inputs: W3 rows [k0, k0 + nk) (n3 each, nk n3 <= 2048) and d3 rows
// [r0, r0 + nr) (nr n3 <= 1024), loaded into registers by aux_load BEFORE the tile's DMA is
// issued and written to LDS by aux_store after it (only the aux loads are waited for there)
struct AuxRegs {
  float w[8], d[4];
};
XA_DEV AuxRegs aux_load(const DZ& d, int k0, int nk, int r0, int nr) {
  AuxRegs a;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = threadIdx.x + 256 * u;
    a.w[u] = (d.h2 && e < nk * d.n3) ? ldc(d.w3 + k0 * d.n3 + e) : 0.0f;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = threadIdx.x + 256 * u;
    a.d[u] = (d.h2 && d.d3 && e < nr * d.n3) ? ldc(d.d3 + r0 * d.n3 + e) : 0.0f;
  }
  return a;
}
XA_DEV void aux_store(const Lds& s, const DZ& d, const AuxRegs& a, int nk, int nr) {
  if (!d.h2) return;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = threadIdx.x + 256 * u;
    if (e < nk * d.n3) s.aux[e] = a.w[u];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = threadIdx.x + 256 * u;
    if (d.d3 && e < nr * d.n3) s.aux[2048 + e] = a.d[u];
  }
}
// dZ2 = g(r, k) (h > 0) for 4 consecutive values of one row / one sample (the aux tables
// indexed relative to the tile: kk = first of the 4 columns, rr = the row)
template <int N3>  // N3 = 0: the width d.n3 at run time
XA_DEV float4 dz_form4(const Lds& s, const DZ& d, float4 h, int rr, int kk) {
  const int n3 = N3 > 0 ? N3 : d.n3;
  float g[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float* w = s.aux + (kk + u) * n3;
    if (d.d3) {
      const float* dr = s.aux + 2048 + rr * n3;
      float t = dr[0] * w[0];
      if constexpr (N3 > 0) {
#pragma unroll
        for (int a = 1; a < N3; ++a) t = fmaf(dr[a], w[a], t);
      } else {
        for (int a = 1; a < n3; ++a) t = fmaf(dr[a], w[a], t);
      }
      g[u] = t;
    } else {
      g[u] = d.c3 * w[0];
    }
  }
  return make_float4(h.x > 0.0f ? g[0] : 0.0f, h.y > 0.0f ? g[1] : 0.0f,
                     h.z > 0.0f ? g[2] : 0.0f, h.w > 0.0f ? g[3] : 0.0f);
}
XA_DEV float4 dz_form4(const Lds& s, const DZ& d, float4 h, int rr, int kk) {
  return d.n3 == 1 ? dz_form4<1>(s, d, h, rr, kk)
         : d.n3 == 4 ? dz_form4<4>(s, d, h, rr, kk) : dz_form4<0>(s, d, h, rr, kk);
}
// scalar form (the non-vector staging paths)
XA_DEV float dz_form(const Lds& s, const DZ& d, float h, int rr, int kk) {
  float g;
  if (d.d3) {
    const float* sd = s.aux + 2048 + rr * d.n3;
    const float* w = s.aux + kk * d.n3;
    g = sd[0] * w[0];
    for (int a = 1; a < d.n3; ++a) g = fmaf(sd[a], w[a], g);
  } else {
    g = d.c3 * s.aux[kk * d.n3];
  }
  return h > 0.0f ? g : 0.0f;
}

// ---- the tile product: wave w, rows 16 w .. 16 w + 15, 16 columns; K padded to 16 ----
template <bool A_CR, bool B_CR>
XA_DEV float4 mma_a(const Lds& s, int k0, int w, int i, int q) {
  if constexpr (A_CR) {
    return *reinterpret_cast<const float4*>(s.A + ((k0 >> 4) * kRows + 16 * w + i) * 16 + 4 * q);
  } else {
    const float* pa = s.A + (k0 + 4 * q) * kRows + 16 * w + i;
    return make_float4(pa[0], pa[kRows], pa[2 * kRows], pa[3 * kRows]);
  }
}
template <bool A_CR, bool B_CR>
XA_DEV float4 mma_b(const Lds& s, int k0, int i, int q) {
  if constexpr (B_CR) {
    return *reinterpret_cast<const float4*>(s.B + ((k0 >> 4) * kCols + i) * 16 + 4 * q);
  } else {
    const float* pb = s.B + (k0 + 4 * q) * kCols + i;
    return make_float4(pb[0], pb[kCols], pb[2 * kCols], pb[3 * kCols]);
  }
}
// the next 16-deep chunk's operands are read from LDS while the current chunk's 4 MFMAs run
template <bool A_CR, bool B_CR>
XA_DEV f32x4v tile_mma(const Lds& s, int Kp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4;
  f32x4v c0 = {0.0f, 0.0f, 0.0f, 0.0f}, c1 = {0.0f, 0.0f, 0.0f, 0.0f};
  float4 a = mma_a<A_CR, B_CR>(s, 0, w, i, q), b = mma_b<A_CR, B_CR>(s, 0, i, q);
  for (int k0 = 0; k0 < Kp; k0 += 16) {
    const int kn = k0 + 16 < Kp ? k0 + 16 : k0;
    const float4 an = mma_a<A_CR, B_CR>(s, kn, w, i, q), bn = mma_b<A_CR, B_CR>(s, kn, i, q);
    c0 = mfma4(a.x, b.x, c0);
    c1 = mfma4(a.y, b.y, c1);
    c0 = mfma4(a.z, b.z, c0);
    c1 = mfma4(a.w, b.w, c1);
    a = an;
    b = bn;
  }
  return c0 + c1;
}

// ---- epilogue helpers: lane l holds D[4 (l >> 4) + r][l & 15] of the wave's 16 rows ----
XA_DEV int out_row(int r) { return 16 * (threadIdx.x >> 6) + 4 * ((threadIdx.x & 63) >> 4) + r; }
XA_DEV int out_col() { return threadIdx.x & 15; }

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

XA_DEV float act_f(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.0f);
  if (act == ACT_TANH) return xa_tanhf(v);
  return v;
}

// ---- narrow follow-on products (the L3 heads, d pi) as column-tile partials: a forward /
// input-gradient job also sums its 16 columns' share of out[r][n] = sum_c y[r][c] Wh(c, n)
// (Wh(c, n) = w[c sc + n sn], n < nh <= 4) into hp[(ct B + r) nh + n]; the job that
// completes a row tile's set (its add to the tile's ticket returned per - 1) finishes the
// product from the partials (fixed column-tile order) before it reaches the grid barrier,
// so the phase that used to compute these products is gone ----
struct Head {
  const float* w;  // null: no head
  float* hp;
  unsigned* ticket;
  int sc, sn, nh, ct, per;
  bool coh;
};
XA_DEV Head no_head() { return Head{nullptr, nullptr, nullptr, 0, 0, 0, 0, 1, false}; }
__shared__ int td3_last;
// B operand of the block's first job in the next phase, staged by LDS-DMA while the grid
// barrier waits (the weights of that job were last written before the barrier the block is
// in); td3_bpre tells the job to skip its own B staging
__shared__ int td3_bpre;
struct PreB {
  const float* W;
  int kind;  // 0 none; 1 forward (KM rows k < K, columns c0 .. of W [K][N]); 2 input
             // gradient (CR rows c0 .. c0 + nc of W [in][K])
  int N, K, c0, nc;
  bool coh;
};
XA_DEV PreB no_preb() { return PreB{nullptr, 0, 0, 0, 0, 0, false}; }
// thread t < 4 kTR holds y[row][c .. c + 3] (zeros outside the tile): its quad's sum
// (lanes t ^ 1, t ^ 2) is the 16-column partial of every n; lane n of the quad stores n
XA_DEV bool head_partial(const Head& h, const float (&wv)[4][4], float4 y, int row, int B) {
  if (!h.w) return false;
  const int t = threadIdx.x;
  float pn[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    float a = y.x * wv[n][0];
    a = fmaf(y.y, wv[n][1], a);
    a = fmaf(y.z, wv[n][2], a);
    a = fmaf(y.w, wv[n][3], a);
    a = a + __shfl_xor(a, 1);
    a = a + __shfl_xor(a, 2);
    pn[n] = a;
  }
  const int q = t & 3;
  if (t < 4 * kTR && row < B && q < h.nh)
    stc(h.hp + ((int64_t)h.ct * B + row) * h.nh + q,
        q == 0 ? pn[0] : q == 1 ? pn[1] : q == 2 ? pn[2] : pn[3]);
  // the ticket: every storing wave drained, then one add for the workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned old = __hip_atomic_fetch_add((gu32*)h.ticket, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old + 1u == (unsigned)h.per;
    // the set is complete: the next launch's adds start from zero
    if (last) __hip_atomic_store((gu32*)h.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    td3_last = last;
  }
  __syncthreads();
  return td3_last != 0;
}
XA_DEV void head_weights(const Head& h, int c, bool on, float (&wv)[4][4]) {
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      wv[n][u] = (h.w && on && n < h.nh) ? ldw(h.w + (int64_t)(c + u) * h.sc + (int64_t)n * h.sn, h.coh)
                                          : 0.0f;
}
constexpr int kMaxCT = (kMaxK + 15) / 16;
// the finished product of (row, n): the column-tile partials summed in tile order
__device__ __noinline__ float head_total(const float* hp, int CT, int B, int nh, int row, int n) {
  float v[kMaxCT];
#pragma unroll
  for (int u = 0; u < kMaxCT; ++u)
    v[u] = u < CT ? ldc(hp + ((int64_t)u * B + row) * nh + n) : 0.0f;
  float a = v[0];
#pragma unroll
  for (int u = 1; u < kMaxCT; ++u)
    if (u < CT) a = a + v[u];
  return a;
}

// ---- forward / input-gradient jobs: a kTR-row x 16-column output tile; wave w computes
// rows 16 (w & 1) .. + 15 over the k chunks of half w >> 1 (the halves meet in LDS, summed
// in a fixed order), then 128 threads finish one float4 of a row each: bias + activation or
// the relu gate, one 16-B write-through store. Operands and the epilogue's inputs are all in
// flight before the first wait ----
XA_DEV float4 mma_a_tr(const Lds& s, int k0, int rb, int i, int q) {
  return *reinterpret_cast<const float4*>(s.A + ((k0 >> 4) * kTR + 16 * rb + i) * 16 + 4 * q);
}
template <bool B_CR>
XA_DEV void tile_mma_split(const Lds& s, int Kp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, q = lane >> 4, rb = w & 1, kh = w >> 1;
  const int nch = Kp >> 4, h0 = (nch + 1) >> 1;
  const int lo = kh ? h0 : 0, hi = kh ? nch : h0;
  f32x4v c0 = {0.0f, 0.0f, 0.0f, 0.0f}, c1 = {0.0f, 0.0f, 0.0f, 0.0f};
  if (lo < hi) {
    float4 a = mma_a_tr(s, 16 * lo, rb, i, q), b = mma_b<false, B_CR>(s, 16 * lo, i, q);
    for (int c = lo; c < hi; ++c) {
      const int kn = 16 * (c + 1 < hi ? c + 1 : c);
      const float4 an = mma_a_tr(s, kn, rb, i, q), bn = mma_b<false, B_CR>(s, kn, i, q);
      c0 = mfma4(a.x, b.x, c0);
      c1 = mfma4(a.y, b.y, c1);
      c0 = mfma4(a.z, b.z, c0);
      c1 = mfma4(a.w, b.w, c1);
      a = an;
      b = bn;
    }
  }
  const f32x4v acc = c0 + c1;
  float* part = td3_part + kh * (kTR * kCols);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(16 * rb + 4 * q + r) * kCols + i] = acc[r];
  __syncthreads();
}
// the tile's float4 of thread t < 128: row t / 4, columns 4 (t % 4) .. + 3 (both halves)
XA_DEV float4 tile_out4() {
  const int t = threadIdx.x;
  const float4 u = *reinterpret_cast<const float4*>(td3_part + 4 * t);
  const float4 v = *reinterpret_cast<const float4*>(td3_part + kTR * kCols + 4 * t);
  return make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
}

// forward job: out[r][c] = act(X W + b) on rows [r0, r0 + kTR) x cols [c0, c0 + 16)
// (A = X rows (CR), B = W[k][c0 ..] (KM); N % 4 == 0; the job functions are out of line:
// one copy each instead of one per call site)
// (the job functions take their arguments through LDS, written by every wave of the
// calling workgroup just before the call: a by-value struct argument would travel through
// scratch memory, one store / load round trip on every call)
struct FwdArgs {
  XSrc x;
  const float* W;
  const float* bias;
  float* out;
  Head h;
  int r0, B, K, N, c0, act;
  bool coh;
};
__shared__ FwdArgs td3_fa;
__device__ __noinline__ bool fwd_tile(const int64_t* slots) {
  const FwdArgs fa = td3_fa;
  const XSrc x = fa.x;
  const Head h = fa.h;
  const float *W = fa.W, *bias = fa.bias;
  float* out = fa.out;
  const int r0 = fa.r0, B = fa.B, K = fa.K, N = fa.N, c0 = fa.c0, act = fa.act;
  const bool coh = fa.coh;
  const Lds s = lds();
  dstamp(0);
  const int Kp = pad16(K), nrows = min(kTR, B - r0), nc = min(kCols, N - c0);
  const int t = threadIdx.x, row = r0 + (t >> 2), c = c0 + 4 * (t & 3);
  const bool st = t < 4 * kTR && row < B && c < N;
  float4 bv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (st) bv = coh ? ld4c(rsrc(bias), (uint32_t)(c * 4)) : ldg4(bias + c);
  float wv[4][4];
  head_weights(h, c, st, wv);
  if (dma_src(x) && (K & 3) == 0)
    dma_cr(s.A, kTR, x.p0, x.ld0, r0, x.slot0 ? td3_slots + r0 : nullptr, nrows, K, Kp, x.coh0);
  else if (quad_src(x, 0) && (K & 3) == 0)
    xgather4(x, r0, kTR, nrows, 0, K, Kp, [&](int r, int k, f32x4v v) {
      *reinterpret_cast<f32x4v*>(s.A + cr_idx(r, k, kTR)) = v;
    });
  else
    sload(kTR, Kp, nrows, K, [&](int r, int k) { return xload(x, slots, r0 + r, k); },
          [&](int r, int k, float v) { s.A[cr_idx(r, k, kTR)] = v; });
  const bool bpre = td3_bpre != 0;  // (staged during the barrier: the same DMA)
  if (bpre) {
  } else if ((N & 3) == 0 && (c0 & 3) == 0 && (nc & 3) == 0)
    dma_km(s.B, kCols, W, N, c0, nullptr, K, nc, Kp, coh);
  else
    sload(Kp, kCols, K, nc, [&](int k, int j) { return ldw(W + (int64_t)k * N + c0 + j, coh); },
          [&](int k, int j, float v) { s.B[k * kCols + j] = v; });
  dstamp(1);
  dma_wait();
  if (bpre && threadIdx.x == 0) td3_bpre = 0;
  dstamp(2);
  tile_mma_split<false>(s, Kp);
  dstamp(3);
  float4 y = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (st) {
    const float4 z = tile_out4();
    y = make_float4(act_f(z.x + bv.x, act), act_f(z.y + bv.y, act), act_f(z.z + bv.z, act),
                    act_f(z.w + bv.w, act));
    st4c(rsrc(out), (uint32_t)(((int64_t)row * N + c) * 4), f32x4v{y.x, y.y, y.z, y.w});
  }
  return head_partial(h, wv, y, row, B);
}

XA_DEV bool fwd_job(const XSrc& x, const int64_t* slots, int r0, int B, const float* W,
                    const float* bias, int K, int N, int c0, int act, float* out,
                    bool coh = false, const Head& h = no_head()) {
  td3_fa = FwdArgs{x, W, bias, out, h, r0, B, K, N, c0, act, coh};
  return fwd_tile(slots);
}

// input-gradient job: out[r][c] = (dZ W^T)[r][c] (gate[r][c] > 0) on rows [r0, r0 + kTR) x
// cols [c0, c0 + 16) of the layer input (W row-major [in][K], out / gate [B][ld]):
// A = dZ rows (CR, the dZ2 former applied in LDS), B = W rows c0 .. (CR)
struct DxArgs {
  DZ d;
  const float* W;
  const float* gate;
  float* out;
  Head h;
  int r0, B, K, c0, nc, ld;
  bool coh;
};
__shared__ DxArgs td3_xa;
__device__ __noinline__ bool dx_tile_lds() {
  const DxArgs xa = td3_xa;
  const DZ d = xa.d;
  const Head h = xa.h;
  const float *W = xa.W, *gate = xa.gate;
  float* out = xa.out;
  const int r0 = xa.r0, B = xa.B, K = xa.K, c0 = xa.c0, nc = xa.nc, ld = xa.ld;
  const bool coh = xa.coh;
  const Lds s = lds();
  dstamp(0);
  const int Kp = pad16(K), nrows = min(kTR, B - r0);
  const int t = threadIdx.x, row = r0 + (t >> 2), c = c0 + 4 * (t & 3);
  const bool st = t < 4 * kTR && row < B && c < c0 + nc;
  float4 gv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (st) gv = ld4c(rsrc(gate), (uint32_t)(((int64_t)row * ld + c) * 4));
  float wv[4][4];
  head_weights(h, c, st, wv);
  const float* src = d.h2 ? d.h2 : d.buf;
  const AuxRegs ax = aux_load(d, 0, K, r0, nrows);
  if ((K & 3) == 0 && (d.ld & 3) == 0)
    dma_cr(s.A, kTR, src, d.ld, r0, nullptr, nrows, K, Kp, true);
  else
    sload(kTR, Kp, nrows, K, [&](int r, int k) { return ldc(src + (int64_t)(r0 + r) * d.ld + k); },
          [&](int r, int k, float v) { s.A[cr_idx(r, k, kTR)] = v; });
  const bool bpre = td3_bpre != 0;  // (staged during the barrier: the same DMA)
  if (bpre) {
  } else if ((K & 3) == 0)
    dma_cr(s.B, kCols, W, K, c0, nullptr, nc, K, Kp, coh);
  else
    sload(kCols, Kp, nc, K, [&](int j, int k) { return ldw(W + (int64_t)(c0 + j) * K + k, coh); },
          [&](int j, int k, float v) { s.B[cr_idx(j, k, kCols)] = v; });
  aux_store(s, d, ax, K, nrows);
  dstamp(1);
  dma_wait();
  if (bpre && threadIdx.x == 0) td3_bpre = 0;
  if (d.h2) {
    // 4 consecutive k of one row per float4 (K % 4 == 0 on this path)
    for (int e4 = threadIdx.x; e4 < kTR * Kp / 4; e4 += 256) {
      const int e = 4 * e4, kc = e / (kTR * 16), r = (e >> 4) & (kTR - 1), k = 16 * kc + (e & 15);
      if (r < nrows && k < K) {
        float4* p = reinterpret_cast<float4*>(s.A + e);
        *p = dz_form4(s, d, *p, r, k);
      }
    }
    __syncthreads();
  }
  dstamp(2);
  tile_mma_split<true>(s, Kp);
  dstamp(3);
  float4 y = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (st) {
    const float4 z = tile_out4();
    y = make_float4(gv.x > 0.0f ? z.x : 0.0f, gv.y > 0.0f ? z.y : 0.0f,
                    gv.z > 0.0f ? z.z : 0.0f, gv.w > 0.0f ? z.w : 0.0f);
    st4c(rsrc(out), (uint32_t)(((int64_t)row * ld + c) * 4), f32x4v{y.x, y.y, y.z, y.w});
  }
  return head_partial(h, wv, y, row, B);
}

// weight-gradient tiles: D_t[i][j] = sum_k X[k][i0 + i] dZ[k][j0 + 16 t + j] for nt <= 4
// column tiles t sharing the staged A (i < ni, columns < nc of the nt x 16, k < B):
// A = X rows (KM, width 64), B = dZ rows (nt KM tiles of width 16); the bias gradients
// sum_k dZ[k][j0 + j] (fixed k order) land in td3_bsum[j] when want_b (each by thread j)
XA_DEV bool dx_tile(const DZ& d, int r0, int B, const float* W, int K, int c0, int nc, bool coh,
                    const float* gate, float* out, int ld, const Head& h) {
  td3_xa = DxArgs{d, W, gate, out, h, r0, B, K, c0, nc, ld, coh};
  return dx_tile_lds();
}

__shared__ float td3_bsum[kCols * 4];  // the bias gradients of a weight-gradient job
struct Acc4 {
  f32x4v t[4];
};
constexpr int kMaxDwTiles = 4;
struct DwArgs {
  XSrc x;
  DZ d;
  int i0, ni, j0, nc, nt, B;
  bool want_b;
};
__shared__ DwArgs td3_wa;
__device__ __noinline__ Acc4 dw_tile_lds(const int64_t* slots) {
  const DwArgs wa = td3_wa;
  const XSrc x = wa.x;
  const DZ d = wa.d;
  const int i0 = wa.i0, ni = wa.ni, j0 = wa.j0, nc = wa.nc, nt = wa.nt, B = wa.B;
  const bool want_b = wa.want_b;
  const Lds s = lds();
  dstamp(0);
  const int Kp = pad16(B);
  const AuxRegs ax = aux_load(d, j0, nc, 0, B);
  if (dma_src(x) && (ni & 3) == 0 && (i0 & 3) == 0)
    dma_km(s.A, kRows, x.p0, x.ld0, i0, x.slot0 ? td3_slots : nullptr, B, ni, Kp, x.coh0);
  else if (quad_src(x, i0) && (ni & 3) == 0)
    xgather4(x, 0, Kp, B, i0, ni, kRows, [&](int k, int i, f32x4v v) {
      *reinterpret_cast<f32x4v*>(s.A + k * kRows + i) = v;
    });
  else
    sload(Kp, kRows, B, ni, [&](int k, int i) { return xload(x, slots, k, i0 + i); },
          [&](int k, int i, float v) { s.A[k * kRows + i] = v; });
  const float* src = d.h2 ? d.h2 : d.buf;
  const bool vec = (d.ld & 3) == 0 && (j0 & 3) == 0 && (nc & 3) == 0;
  for (int t = 0; t < nt; ++t) {
    float* bt = s.B + t * Kp * kCols;
    const int jt = j0 + kCols * t, nct = min(kCols, nc - kCols * t);
    if (vec)
      dma_km(bt, kCols, src, d.ld, jt, nullptr, B, nct, Kp, true);
    else
      sload(Kp, kCols, B, nct, [&](int k, int j) { return ldc(src + (int64_t)k * d.ld + jt + j); },
            [&](int k, int j, float v) { bt[k * kCols + j] = v; });
  }
  aux_store(s, d, ax, nc, B);
  dstamp(1);
  dma_wait();
  if (d.h2) {
    // 4 consecutive columns of one sample per float4 (nc % 4 == 0 on this path)
    for (int e4 = threadIdx.x; e4 < nt * Kp * kCols / 4; e4 += 256) {
      const int t = e4 / (Kp * kCols / 4), r4 = e4 - t * (Kp * kCols / 4);
      const int k = r4 >> 2, j = kCols * t + 4 * (r4 & 3);
      if (k < B && j < nc) {
        float4* p = reinterpret_cast<float4*>(s.B + 4 * e4);
        *p = dz_form4(s, d, *p, k, j);
      }
    }
    __syncthreads();
  }
  if (want_b && (int)threadIdx.x < nc) {
    const int t = threadIdx.x >> 4, j = threadIdx.x & 15;
    const float* bt = s.B + t * Kp * kCols;
    float acc = 0.0f;
    for (int k = 0; k < B; ++k) acc += bt[k * kCols + j];
    td3_bsum[threadIdx.x] = acc;
  }
  dstamp(2);
  // one pass over k for every column tile: A's 4 k-major words per chunk read once, each
  // tile's B words and 4 MFMAs per chunk, the next chunk's words read during this chunk's
  // MFMAs
  Acc4 r;
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane & 15, q = lane >> 4;
    const int tstride = Kp * kCols;
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t) r.t[t] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    float4 a = mma_a<false, false>(s, 0, w, i, q);
    float4 bb[kMaxDwTiles];
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t) {
      const float* pb = s.B + t * tstride + 4 * q * kCols + i;
      bb[t] = t < nt ? make_float4(pb[0], pb[kCols], pb[2 * kCols], pb[3 * kCols])
                     : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    for (int k0 = 0; k0 < Kp; k0 += 16) {
      const int kn = k0 + 16 < Kp ? k0 + 16 : k0;
      const float4 an = mma_a<false, false>(s, kn, w, i, q);
      float4 bn[kMaxDwTiles];
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t) {
        const float* pb = s.B + t * tstride + (kn + 4 * q) * kCols + i;
        bn[t] = t < nt ? make_float4(pb[0], pb[kCols], pb[2 * kCols], pb[3 * kCols]) : bb[t];
      }
      // (k step outer, tile inner: consecutive MFMAs on independent accumulators)
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t)
        if (t < nt) r.t[t] = mfma4(a.x, bb[t].x, r.t[t]);
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t)
        if (t < nt) r.t[t] = mfma4(a.y, bb[t].y, r.t[t]);
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t)
        if (t < nt) r.t[t] = mfma4(a.z, bb[t].z, r.t[t]);
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t)
        if (t < nt) r.t[t] = mfma4(a.w, bb[t].w, r.t[t]);
      a = an;
#pragma unroll
      for (int t = 0; t < kMaxDwTiles; ++t) bb[t] = bn[t];
    }
  }
  dstamp(3);
  return r;
}

// Keras Adam (+ Polyak into the target) of one parameter from its raw gradient
XA_DEV void adam_one(const Net& n, float g, int i, float omb1, float omb2, float eps,
                     float* target, float tau) {
  float th = ldc(n.th + i), m = ldg(n.m + i), v = ldg(n.v + i);
  adam_elem(g, th, m, v, n.alpha, omb1, omb2, eps);
  stc(n.th + i, th);
  stg(n.m + i, m);
  stg(n.v + i, v);
  if (target) {
    const float y = ldg(target + i);
    stg(target + i, tau == 1.0f ? th : (1.0f - tau) * y + tau * th);
  }
}

// Adam (+ Polyak) of parameters [lo, hi) from their raw gradients (lo % 4 == 0 and every
// array 16-B aligned): float4 groups, every load of a thread's groups issued before the
// first update (one memory round trip, not one per element); the < 4 trailing elements
// of the network scalar
constexpr int kAdamG = 4;  // float4 groups per thread per round
XA_DEV int adam_chunk(int rest, int jobs) {
  const int per = 4 * 256;  // one group per thread
  const int c = (rest + jobs - 1) / jobs;
  return max(per, (c + per - 1) / per * per);
}
__device__ __noinline__ void adam_range(Net n, const float* grad, int lo, int hi, float omb1,
                                        float omb2, float eps, float* target, float tau,
                                        float gs = 1.0f) {
  const int hi4 = lo + ((hi - lo) & ~3);
  const __amdgpu_buffer_rsrc_t rg = rsrc(grad), rt = rsrc(n.th);
  for (int g0 = lo / 4 + (int)threadIdx.x; 4 * g0 < hi4; g0 += 256 * kAdamG) {
    float4 g[kAdamG], th[kAdamG], m[kAdamG], v[kAdamG], tg[kAdamG];
#pragma unroll
    for (int u = 0; u < kAdamG; ++u) {
      const int i = 4 * min(g0 + 256 * u, hi4 / 4 - 1);
      g[u] = ld4c(rg, (uint32_t)i * 4u);
      th[u] = ld4c(rt, (uint32_t)i * 4u);
      m[u] = ldg4(n.m + i);
      v[u] = ldg4(n.v + i);
      tg[u] = target ? ldg4(target + i) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kAdamG; ++u) {
      const int i = 4 * (g0 + 256 * u);
      if (i >= hi4) break;
      float* gp = &g[u].x;
      float* tp = &th[u].x;
      float* mp = &m[u].x;
      float* vp = &v[u].x;
      float* yp = &tg[u].x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        adam_elem(gp[c] * gs, tp[c], mp[c], vp[c], n.alpha, omb1, omb2, eps);
        yp[c] = tau == 1.0f ? tp[c] : (1.0f - tau) * yp[c] + tau * tp[c];
      }
      st4c(rt, (uint32_t)i * 4u, f32x4v{th[u].x, th[u].y, th[u].z, th[u].w});
      stg4(n.m + i, m[u]);
      stg4(n.v + i, v[u]);
      if (target) stg4(target + i, tg[u]);
    }
  }
  if ((int)threadIdx.x < hi - hi4) {
    const int i = hi4 + threadIdx.x;
    adam_one(n, ldc(grad + i) * gs, i, omb1, omb2, eps, target, tau);
  }
}

// weight-gradient job over columns [j0, j0 + 16 nt) of W [nin][N] (offset w; the bias at b
// when the job holds the first in-feature tile): the raw gradient into grad, optionally the
// Adam step (+ Polyak) of those elements
// (the Adam options by value: no pointer into the kernel's private frame)
struct AdamOpt {
  float omb1, omb2, eps, tau;
  float* target;
  bool on;
};
XA_DEV AdamOpt adam_opt(const XaTdNet& o, float* target, float tau) {
  return AdamOpt{1.0f - o.beta1, 1.0f - o.beta2, o.eps, tau, target, true};
}
XA_DEV AdamOpt no_adam() { return AdamOpt{0.0f, 0.0f, 0.0f, 0.0f, nullptr, false}; }
XA_DEV void dw_job(const XSrc& x, const int64_t* slots, const DZ& d, int nin, int N, int i0,
                   int j0, int nt, int B, float* grad, int w, int b, const Net& an,
                   const AdamOpt& ao) {
  const int ni = min(kRows, nin - i0), nc = min(kCols * nt, N - j0);
  nt = (nc + kCols - 1) / kCols;
  const bool first = i0 == 0;
  td3_wa = DwArgs{x, d, i0, ni, j0, nc, nt, B, first};
  const Acc4 acc = dw_tile_lds(slots);
  const float omb1 = ao.omb1, omb2 = ao.omb2, eps = ao.eps, tau = ao.tau;
  float* const target = ao.target;
  // (the bias gradient of column threadIdx.x < nc was summed by this same thread)
  const bool has_b = first && (int)threadIdx.x < nc;
  if ((N & 3) == 0 && (j0 & 3) == 0 && (w & 3) == 0) {
    // the tile through LDS, row-major [64 in-features][64 (+ 4 pad)]: every thread then owns
    // whole float4 groups -- 16-B loads and write-through stores instead of scattered words
    constexpr int kTS = kRows + 4;
    float* T = lds().A;
    __syncthreads();  // every wave's MFMA reads of the staged operands are done
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (t < nt) T[out_row(r) * kTS + kCols * t + out_col()] = acc.t[t][r];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rg = rsrc(grad), rt = rsrc(an.th);
    float4 gq[4], thq[4], mq[4], vq[4], tq[4];
    int eq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = (int)threadIdx.x + 256 * u, i = f >> 4, c = 4 * (f & 15);
      const bool ok = i < ni && c < nc;
      eq[u] = ok ? w + (i0 + i) * N + j0 + c : -1;
      const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      gq[u] = ok ? *reinterpret_cast<const float4*>(T + i * kTS + c) : z;
      thq[u] = mq[u] = vq[u] = tq[u] = z;
      if (ao.on && ok) {
        thq[u] = ld4c(rt, (uint32_t)eq[u] * 4u);
        mq[u] = ldg4(an.m + eq[u]);
        vq[u] = ldg4(an.v + eq[u]);
        if (target) tq[u] = ldg4(target + eq[u]);
      }
    }
    const int eb = b + j0 + (has_b ? (int)threadIdx.x : 0);
    float bth = 0.0f, bm = 0.0f, bv = 0.0f, btg = 0.0f;
    if (ao.on && has_b) {
      bth = ldc(an.th + eb);
      bm = ldg(an.m + eb);
      bv = ldg(an.v + eb);
      btg = target ? ldg(target + eb) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (eq[u] < 0) continue;
      st4c(rg, (uint32_t)eq[u] * 4u, f32x4v{gq[u].x, gq[u].y, gq[u].z, gq[u].w});
      if (!ao.on) continue;
      float* gp = &gq[u].x;
      float* tp = &thq[u].x;
      float* mp = &mq[u].x;
      float* vp = &vq[u].x;
      float* yp = &tq[u].x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        adam_elem(gp[c], tp[c], mp[c], vp[c], an.alpha, omb1, omb2, eps);
        yp[c] = tau == 1.0f ? tp[c] : (1.0f - tau) * yp[c] + tau * tp[c];
      }
      st4c(rt, (uint32_t)eq[u] * 4u, f32x4v{thq[u].x, thq[u].y, thq[u].z, thq[u].w});
      stg4(an.m + eq[u], mq[u]);
      stg4(an.v + eq[u], vq[u]);
      if (target) stg4(target + eq[u], tq[u]);
    }
    if (has_b) {
      const float g = td3_bsum[threadIdx.x];
      stc(grad + eb, g);
      if (ao.on) {
        adam_elem(g, bth, bm, bv, an.alpha, omb1, omb2, eps);
        stc(an.th + eb, bth);
        stg(an.m + eb, bm);
        stg(an.v + eb, bv);
        if (target) stg(target + eb, tau == 1.0f ? bth : (1.0f - tau) * btg + tau * bth);
      }
    }
  } else if (ao.on) {
    // every parameter / moment / target load of the thread's nt x 4 elements and of its
    // bias element in flight before the first update: one memory round trip
    float th[kMaxDwTiles][4], m[kMaxDwTiles][4], v[kMaxDwTiles][4], tg[kMaxDwTiles][4];
    int ee[kMaxDwTiles][4];
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t) {
      const int j = kCols * t + out_col();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = out_row(r);
        const bool ok = t < nt && i < ni && j < nc;
        ee[t][r] = ok ? w + (i0 + i) * N + j0 + j : -1;
        const int e = ok ? ee[t][r] : w;
        th[t][r] = t < nt ? ldc(an.th + e) : 0.0f;
        m[t][r] = t < nt ? an.m[e] : 0.0f;
        v[t][r] = t < nt ? an.v[e] : 0.0f;
        tg[t][r] = (t < nt && target) ? target[e] : 0.0f;
      }
    }
    const int eb = b + j0 + (has_b ? (int)threadIdx.x : 0);
    float bth = 0.0f, bm = 0.0f, bv = 0.0f, btg = 0.0f;
    if (has_b) {
      bth = ldc(an.th + eb);
      bm = an.m[eb];
      bv = an.v[eb];
      btg = target ? target[eb] : 0.0f;
    }
    auto upd = [&](int e, float g, float th_, float m_, float v_, float tg_) {
      stc(grad + e, g);
      adam_elem(g, th_, m_, v_, an.alpha, omb1, omb2, eps);
      stc(an.th + e, th_);
      an.m[e] = m_;
      an.v[e] = v_;
      if (target) target[e] = tau == 1.0f ? th_ : (1.0f - tau) * tg_ + tau * th_;
    };
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (ee[t][r] >= 0) upd(ee[t][r], acc.t[t][r], th[t][r], m[t][r], v[t][r], tg[t][r]);
    if (has_b) upd(eb, td3_bsum[threadIdx.x], bth, bm, bv, btg);
  } else {
#pragma unroll
    for (int t = 0; t < kMaxDwTiles; ++t) {
      if (t >= nt) continue;
      const int j = kCols * t + out_col();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = out_row(r);
        if (i < ni && j < nc) stc(grad + w + (i0 + i) * N + j0 + j, acc.t[t][r]);
      }
    }
    if (has_b) stc(grad + b + j0 + threadIdx.x, td3_bsum[threadIdx.x]);
  }
}

// ---- the grid barrier: a counter sharded over 8 lines (block b adds to shard b % 8: 32
// arrivals per line instead of 256 on one), polled by one lane per block as the sum of the
// shards; only the blocks that held a job in the phase arrive (the rest only wait), so the
// target grows by min(G, jobs) per barrier ----
constexpr int kShards = 8, kShardStride = 32;  // u32 words between shards (128 B)
struct Sync {
  unsigned* cnt;
  unsigned* abort_w;
  unsigned target, G, n, epoch;
  int* status;
  unsigned long long* trace;  // block 0 only: the wall clock as each barrier completes
  // launch-entry rendezvous (block 0 only): every block adds 1 to *ent once it holds the
  // launch-start words in registers; block 0 writes the next launch's start words only
  // after *ent reached ent_target (seen while it waits at a barrier, or polled at the end)
  unsigned* ent;
  unsigned ent_target;
  int ent_ok;
};

// block 0, thread 0: has every block of the launch entered (read its start words)?
XA_DEV bool entered_all(const Sync& y) {
  return (int)(__hip_atomic_load((gu32*)y.ent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
               y.ent_target) >= 0;
}

// Every block, once its launch-start words (barrier base, epoch, step / noise / entry
// counters) are in registers: drain the loads, then one lane counts the block in. Contains a
// __syncthreads().
XA_DEV void enter_launch(unsigned* ent) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add((gu32*)ent, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// block 0, thread 0, before it writes the next launch's start words: wait (bounded) until
// every block entered. False on timeout / abort.
XA_DEV bool wait_entered(Sync& y) {
  const uint64_t t0 = wall_clock64();
  while (!y.ent_ok) {
    if (entered_all(y)) {
      y.ent_ok = 1;
      break;
    }
    if (__hip_atomic_load((gu32*)y.abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == y.epoch)
      return false;
    if (wall_clock64() - t0 > kSpinTicks) {
      __hip_atomic_store((gu32*)y.abort_w, y.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (y.status) __hip_atomic_store((gu32*)y.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

XA_DEV unsigned shard_sum(const unsigned* cnt) {
  unsigned v[kShards];
#pragma unroll
  for (int s = 0; s < kShards; ++s)
    v[s] = __hip_atomic_load((gu32*)(cnt + kShardStride * s), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  unsigned t = 0;
#pragma unroll
  for (int s = 0; s < kShards; ++s) t += v[s];
  return t;
}

struct NoMid {
  XA_DEV void operator()() const {}
};
// mid: work every thread does after the arrival, while thread 0 waits (the Adam step sizes)
template <class Mid = NoMid>
XA_DEV bool grid_sync(Sync& y, int& lds_flag, int jobs, const PreB& pb = no_preb(),
                      const Mid& mid = Mid()) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  y.n += 1;
  // only the blocks that held a job arrive (a block dispatched late never holds up a
  // barrier it has no work before); block 0's end-of-launch writes are ordered behind every
  // block's reads of the launch-start words by the entry counter instead (enter_launch /
  // wait_entered; ADVICE r04's hazard)
  const unsigned m = (unsigned)min((int)y.G, max(jobs, 0));
  y.target += m;
  if (threadIdx.x == 0 && blockIdx.x < m)
    __hip_atomic_fetch_add((gu32*)(y.cnt + kShardStride * (blockIdx.x % kShards)), 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the next job's weights into LDS while the barrier waits (every wave issues its share)
  if (pb.kind == 1 && (pb.N & 3) == 0 && (pb.c0 & 3) == 0) {
    const int nc = min(kCols, pb.N - pb.c0);
    if ((nc & 3) == 0) {
      dma_km(lds().B, kCols, pb.W, pb.N, pb.c0, nullptr, pb.K, nc, pad16(pb.K), pb.coh);
      if (threadIdx.x == 0) td3_bpre = 1;
    }
  } else if (pb.kind == 2 && (pb.K & 3) == 0) {
    dma_cr(lds().B, kCols, pb.W, pb.K, pb.c0, nullptr, pb.nc, pb.K, pad16(pb.K), pb.coh);
    if (threadIdx.x == 0) td3_bpre = 1;
  }
  mid();
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t t0 = wall_clock64();
    for (unsigned it = 0;; ++it) {
      // block 0 checks the entry counter while it waits anyway (same round trip)
      if (y.ent && !y.ent_ok && entered_all(y)) y.ent_ok = 1;
      if ((int)(shard_sum(y.cnt) - y.target) >= 0) break;  // wrap-safe: the shards only grow
      if ((it & 15u) == 15u) {
        if (__hip_atomic_load((gu32*)y.abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            y.epoch) {
          ok = 0;
          break;
        }
        if (wall_clock64() - t0 > kSpinTicks) {
          __hip_atomic_store((gu32*)y.abort_w, y.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (y.status)
            __hip_atomic_store((gu32*)y.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
    lds_flag = ok;
    if (XA_TD3_TRACE && y.trace && y.n < 15) y.trace[y.n] = wall_clock64();
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  return lds_flag != 0;
}

// workspace: control words, then the activations / gradients of the step (floats)
struct Ws {
  unsigned* cnt;      // barrier counter shards (monotonic)
  unsigned* base;     // the shards' sum at the start of the next launch
  unsigned* abort_w;  // the epoch of a launch that timed out
  unsigned* epoch;    // launches so far
  unsigned* ent;      // launch-entry counter: every block of every launch adds 1
  unsigned* ent_base;  // the entry counter at the start of the next launch
  unsigned long long* dtrace;  // [16][8] points inside block 0's first job of each phase
  unsigned long long* trace;  // [16] wall clock at launch start and after every barrier
                              // (block 0; tools/td3_grad_steps.py reads it)
  float* h1all;       // [6][B][H1] per network slot: target actor, critic 1, critic 2,
  float* h2all;       // [6][B][H2]   actor, target critic 1, target critic 2
  __host__ __device__ float* h1(int id) const { return h1all + (size_t)id * h1s; }
  __host__ __device__ float* h2(int id) const { return h2all + (size_t)id * h2s; }
  size_t h1s, h2s;
  float* q1;          // critic 1 on [s, pi(s)]: h1
  float* q2;          //                         h2
  float* ta;          // a' [B][A] (smoothed target action)
  float* pa;          // pi(s) [B][A]
  float* v1;          // critic values [B]
  float* v2;
  float* dh1all;      // critics' dH1 [2][B][H1]
  __host__ __device__ float* dh1(int c) const { return dh1all + (size_t)c * h1s; }
  float* dq1;         // dH1 of -mean Q [B][H1]
  float* dz3;         // actor output gradient [B][A]
  float* dh1a;        // actor dH1 [B][H1]
  float* hp3all;      // head partials [6][CT2][B][4] per network slot (L3 of each network)
  __host__ __device__ float* hp3(int id) const { return hp3all + (size_t)id * hp3s; }
  size_t hp3s;
  float* hpp;         // d pi partials [CT1][B][A]
  unsigned* tickets;  // [7 slots][8 row tiles], 128 B apart: the head tickets
  __device__ unsigned* ticket(int slot, int rt) const { return tickets + 32 * (8 * slot + rt); }
  size_t total;
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

__host__ __device__ inline Ws carve(void* base_p, int B, int H1, int H2, int A) {
  Ws w;
  char* c = (char*)base_p;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = c + off;
    off = align_up(off + bytes, 256);
    return q;
  };
  unsigned* ctl = (unsigned*)take(2048);  // bytes: [0, 1024) counter shards, 1024 base,
  w.cnt = ctl;                              // 1152 abort, 1280 epoch, [1536, 1664) trace
  w.base = ctl + 256;
  w.abort_w = ctl + 288;
  w.epoch = ctl + 320;
  w.trace = (unsigned long long*)(ctl + 384);
  w.ent = ctl + 448;       // byte 1792: the launch-entry counter (monotonic)
  w.ent_base = ctl + 480;  // byte 1920: its value at the start of the next launch
  w.dtrace = (unsigned long long*)take(8192);
  w.h1s = align_up((size_t)B * H1, 64);
  w.h2s = align_up((size_t)B * H2, 64);
  w.h1all = (float*)take(6 * w.h1s * 4);
  w.h2all = (float*)take(6 * w.h2s * 4);
  w.q1 = (float*)take((size_t)B * H1 * 4);
  w.q2 = (float*)take((size_t)B * H2 * 4);
  w.ta = (float*)take((size_t)B * A * 4);
  w.pa = (float*)take((size_t)B * A * 4);
  w.v1 = (float*)take((size_t)B * 4);
  w.v2 = (float*)take((size_t)B * 4);
  w.dh1all = (float*)take(2 * w.h1s * 4);
  w.dq1 = (float*)take((size_t)B * H1 * 4);
  w.dz3 = (float*)take((size_t)B * A * 4);
  w.dh1a = (float*)take((size_t)B * H1 * 4);
  const int CT1 = (H1 + 15) / 16, CT2 = (H2 + 15) / 16;
  w.hp3s = align_up((size_t)CT2 * B * 4, 64);
  w.hp3all = (float*)take(6 * w.hp3s * 4);
  w.hpp = (float*)take((size_t)CT1 * B * A * 4);
  w.tickets = (unsigned*)take(7 * 8 * 128);
  w.total = off;
  return w;
}

enum { N_TA = 0, N_C1 = 1, N_C2 = 2, N_AC = 3, N_TC1 = 4, N_TC2 = 5 };

__global__ __launch_bounds__(256) void td3_update_kernel(XaTd3UpdateArgs p) {
  __shared__ int s_flag;
  // a launch whose barrier timed out left the control words inconsistent (a stale barrier
  // base, partial arrivals in the shards): every later launch is a no-op until the caller
  // re-zeroes the workspace and the status word (it raises on the status)
  if (p.status && *(const volatile int*)p.status != 0) return;
  const int G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  const int B = p.batch, S = p.obs_dim, A = p.act_dim, H1 = p.h1, H2 = p.h2;
  const int C = S + A;
  const bool twin = p.twin != 0, pol = p.actor_update != 0;
  // 0: the whole gradient step; data parallel (the gradients all-reduced between launches):
  // 1 critics' forward / backward -> raw gradients, 2 critics' Adam (+ Polyak) and, on
  // policy steps, the actor's forward / backward through the updated critic 1 -> raw
  // gradient, 3 the actor's Adam + Polyak
  const int stage = p.stage;
  const Ws ws = carve(p.workspace, B, H1, H2, A);
  Sync y;
  y.cnt = ws.cnt;
  y.abort_w = ws.abort_w;
  y.target = *ws.base;
  y.epoch = *ws.epoch + 1u;
  y.G = (unsigned)G;
  y.n = 0;
  y.status = p.status;
  y.trace = b == 0 ? ws.trace : nullptr;
  y.ent = b == 0 && tid == 0 ? ws.ent : nullptr;
  y.ent_target = *ws.ent_base + (unsigned)G;
  y.ent_ok = 0;
  if (XA_TD3_TRACE && b == 0 && tid == 0) ws.trace[0] = wall_clock64();
  if (tid == 0) td3_bpre = 0;
#if XA_TD3_TRACE
  if (tid == 0) {
    td3_dslot = b == 0 ? 8 * 15 : -1;  // (diagnostic) the prologue's points in slot 15
    td3_dbuf = ws.dtrace;
  }
#endif
  dstamp(0);
  // networks; the step counters as the launch finds them are read here (in flight with the
  // slot loads) and the Adam step sizes formed only where the optimizer steps run
  Net c1 = make_net(p.critic1, C, H1, H2, 1, false);
  Net c2 = make_net(twin ? p.critic2 : p.critic1, C, H1, H2, 1, false);
  Net ac = make_net(p.actor, S, H1, H2, A, false);
  const int step_c1 = *p.critic1.step, step_c2 = twin ? *p.critic2.step : 0;
  const int step_ac = pol ? *p.actor.step : 0;
  if (tid < p.batch) td3_slots[tid] = p.slots[tid];  // (batch <= 256)
  dstamp(1);
  enter_launch(ws.ent);  // (the launch-start words are in registers; contains the barrier)
  dstamp(2);
  const Net tc1 = make_net(p.target_critic1, C, H1, H2, 1, false);
  const Net tc2 = make_net(twin ? p.target_critic2 : p.target_critic1, C, H1, H2, 1, false);
  const int64_t* slots = p.slots;
  const int RTT = (B + kTR - 1) / kTR;
  const int CT1 = (H1 + kCols - 1) / kCols, CT2 = (H2 + kCols - 1) / kCols;
  // column tiles per weight-gradient job (they share the staged A; the B region holds
  // kCols x kMaxK floats, one k-major [pad16(B)][16] tile per column tile)
  const int NTW = max(1, min(kMaxDwTiles, (kCols * kMaxK) / (pad16(B) * kCols)));
  const int CTW2 = (CT2 + NTW - 1) / NTW, CTW1 = (CT1 + NTW - 1) / NTW;
  const float* rs = p.ring_states;
  const float* rn = p.ring_new_states;
  const float* ra = p.ring_actions;

  // the sampled batch for the caller (concat_buffer_samples' arrays), from the last block:
  // element e of [s | s' | a | r | d], every load of a thread in flight before its stores
  if (stage <= 1 && b == G - 1) {
    const int nS = B * S, nA = B * A, tot = 2 * nS + nA + 2 * B;
    constexpr int kGu = 16;
    for (int e0 = tid; e0 < tot; e0 += 256 * kGu) {
      float v[kGu];
#pragma unroll
      for (int u = 0; u < kGu; ++u) {
        int e = e0 + 256 * u;
        float x = 0.0f;
        if (e < nS) {
          x = rs[td3_slots[e / S] * S + e % S];
        } else if ((e -= nS) < nS) {
          x = rn[td3_slots[e / S] * S + e % S];
        } else if ((e -= nS) < nA) {
          x = ra[td3_slots[e / A] * A + e % A];
        } else if ((e -= nA) < B) {
          x = p.ring_rewards[td3_slots[e]];
        } else if ((e -= B) < B) {
          x = p.ring_dones[td3_slots[e]];
        }
        v[u] = x;
      }
#pragma unroll
      for (int u = 0; u < kGu; ++u) {
        int e = e0 + 256 * u;
        // (s, s', a write-through: later phases read them back as dense rows)
        if (e < nS) stc(p.out_s + e, v[u]);
        else if ((e -= nS) < nS) stc(p.out_s2 + e, v[u]);
        else if ((e -= nS) < nA) stc(p.out_a + e, v[u]);
        else if ((e -= nA) < B) p.out_r[e] = v[u];
        else if ((e -= B) < B) p.out_d[e] = v[u];
      }
    }
  }

  dstamp(3);

  // ---- P1 / P2: L1 and L2 forward of the target actor, the critics (and the actor) ----
  // the networks of P1 - P3: target actor, critic 1, [critic 2], [actor]
  const int nn = 2 + (twin ? 1 : 0) + (pol ? 1 : 0);
  auto net_id = [&](int t) { return t < 2 ? t : (t == 2 && twin) ? N_C2 : N_AC; };
  // a network's view by slot id (by value from the kernel arguments: no stack arrays)
  auto net_of = [&](int id) -> Net {
    const bool actor_like = id == N_TA || id == N_AC;
    const XaTdNet& d = id == N_TA ? p.target_actor : id == N_C1 ? p.critic1
                     : id == N_C2 ? p.critic2 : id == N_AC ? p.actor
                     : id == N_TC1 ? p.target_critic1 : p.target_critic2;
    return make_net(d, actor_like ? S : C, H1, H2, actor_like ? A : 1, false);
  };
  // the sampled batch as dense rows (the caller's copies, written through by the last block
  // before its first barrier): what every phase after P1 stages instead of ring rows
  const XSrc sa_dense = xcat(xsrc(p.out_s, S, S, false, true), p.out_a, A, A, false, true);
  auto in_of = [&](int id) -> XSrc {
    if (id == N_TA) return xsrc(rn, S, S, true, false);            // s'
    if (id == N_AC) return xsrc(rs, S, S, true, false);            // s
    return xcat(xsrc(rs, S, S, true, false), ra, A, A, true, false);  // [s, a]
  };
  const uint64_t ctr = p.rng_counter ? *p.rng_counter : 0ull;
  // the B operand of this block's first job in the next phase (prefetched at the barrier;
  // the same job enumeration as the phase loops below)
  auto pre_fwd = [&](const float* W, int N, int K, int ct, bool coh) {
    return PreB{W, 1, N, K, ct * kCols, min(kCols, N - ct * kCols), coh};
  };
  auto pre_dx = [&](const float* W, int K, int ct, bool coh) {
    return PreB{W, 2, 0, K, ct * kCols, min(kCols, H1 - ct * kCols), coh};
  };
  auto pre_p2 = [&]() {
    const int per = RTT * CT2;
    if (b >= nn * per) return no_preb();
    const Net n = net_of(net_id(b / per));
    return pre_fwd(n.th + n.w2, H2, H1, (b % per) % CT2, false);
  };
  auto pre_p5 = [&]() {
    const int per = RTT * CT2, ntc = twin ? 2 : 1;
    if (b >= ntc * per) return no_preb();
    const Net n = net_of(N_TC1 + b / per);
    return pre_fwd(n.th + n.w2, H2, H1, (b % per) % CT2, false);
  };
  auto pre_p7 = [&]() {
    const int IT1 = (H1 + kRows - 1) / kRows, IT2 = (H2 + kRows - 1) / kRows;
    const int n_dx = RTT * CT1, per = n_dx + IT1 * CTW2 + IT2, ntc = twin ? 2 : 1;
    const int ci = b / per, q = b % per;
    if (b >= ntc * per || q >= n_dx) return no_preb();
    const Net n = ci ? c2 : c1;
    return pre_dx(n.th + n.w2, H2, q % CT1, false);
  };
  auto pre_p10 = [&]() {
    if (b >= RTT * CT2) return no_preb();
    return pre_fwd(c1.th + c1.w2, H2, H1, b % CT2, true);
  };
  auto pre_p11 = [&]() {
    if (b >= RTT * CT1) return no_preb();
    return pre_dx(c1.th + c1.w2, H2, b % CT1, true);
  };
  auto pre_p13 = [&]() {
    if (b >= RTT * CT1) return no_preb();  // (the input-gradient jobs come first)
    return pre_dx(ac.th + ac.w2, H2, b % CT1, false);
  };
  const int nt = twin ? 2 : 1;
  int p8_jobs = 0;
  if (stage <= 1) {
  for (int layer = 1; layer <= 2; ++layer) {
    const int CT = layer == 1 ? CT1 : CT2, per = RTT * CT;
    for (int j = b; j < nn * per; j += G) {
      XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
      const int id = net_id(j / per), rem = j % per, rt = rem / CT, ct = rem % CT;
      const Net n = net_of(id);
      if (layer == 1) {
        fwd_job(in_of(id), slots, rt * kTR, B, n.th + n.w1, n.th + n.b1, n.in, H1, ct * kCols,
                ACT_RELU, ws.h1(id));
      } else {
        // + the L3 partials of the tile's 16 units; the row tile's last job finishes L3:
        // target actor tanh (+ TD3 smoothing noise, clip) -> a', critics -> v1, v2,
        // actor tanh -> pi(s)
        const Head hd{n.th + n.w3, ws.hp3(id), ws.ticket(id, rt), n.out, 1, n.out, ct, CT2,
                      false};
        if (fwd_job(xsrc(ws.h1(id), H1, H1, false, true), slots, rt * kTR, B, n.th + n.w2,
                    n.th + n.b2, H1, H2, ct * kCols, ACT_RELU, ws.h2(id), false, hd)) {
          const int N = n.out, r0 = rt * kTR, nr = min(kTR, B - r0);
          for (int e = tid; e < nr * N; e += 256) {
            const int row = r0 + e / N, c = e % N;
            const float z = head_total(ws.hp3(id), CT2, B, N, row, c) + n.th[n.b3 + c];
            if (id == N_TA) {
              float a = xa_tanhf(z);
              if (p.smooth) {
                float nz = 0.0f;
                if (p.noise_sigma != 0.0f) {
                  nz = philox_normal((uint32_t)row, (uint32_t)c, ctr, p.seed) * p.noise_sigma;
                  nz = fminf(fmaxf(nz, -p.noise_clip), p.noise_clip);
                }
                if (p.noise_out) p.noise_out[row * A + c] = nz;
                a = fminf(fmaxf(a + nz, -1.0f), 1.0f);
              }
              stc(ws.ta + row * A + c, a);
            } else if (id == N_AC) {
              stc(ws.pa + row * A + c, xa_tanhf(z));
            } else {
              stc((id == N_C1 ? ws.v1 : ws.v2) + row, z);
            }
          }
        }
      }
      __syncthreads();
    }
    if (!grid_sync(y, s_flag, nn * per, layer == 1 ? pre_p2() : no_preb())) return;
  }

  // ---- P4 / P5: target critics L1 on [s', a'], L2 (+ the target values' partials; the
  // row tile's last job runs the TD head: y = r + (1 - d) gamma min(tv1, tv2),
  // dv = 2 (v - y) (MSE) or clip(v - y, +-delta) (opt-in Huber), per-sample loss) ----
  for (int layer = 1; layer <= 2; ++layer) {
    const int CT = layer == 1 ? CT1 : CT2, per = RTT * CT;
    for (int j = b; j < nt * per; j += G) {
      XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
      const int id = N_TC1 + j / per, rem = j % per, rt = rem / CT, ct = rem % CT;
      const Net n = net_of(id);
      if (layer == 1) {
        fwd_job(xcat(xsrc(p.out_s2, S, S, false, true), ws.ta, A, A, false, true), slots,
                rt * kTR, B, n.th + n.w1, n.th + n.b1, C, H1, ct * kCols, ACT_RELU, ws.h1(id));
      } else {
        const Head hd{n.th + n.w3, ws.hp3(id), ws.ticket(N_TC1, rt), 1, 1, 1, ct, nt * CT2,
                      false};
        if (fwd_job(xsrc(ws.h1(id), H1, H1, false, true), slots, rt * kTR, B, n.th + n.w2,
                    n.th + n.b2, H1, H2, ct * kCols, ACT_RELU, ws.h2(id), false, hd)) {
          const int r0 = rt * kTR, nr = min(kTR, B - r0);
          if (tid < nr) {
            const int row = r0 + tid;
            const float t1 = head_total(ws.hp3(N_TC1), CT2, B, 1, row, 0) + tc1.th[tc1.b3];
            const float tv = twin
                ? fminf(t1, head_total(ws.hp3(N_TC2), CT2, B, 1, row, 0) + tc2.th[tc2.b3])
                : t1;
            const int64_t sl = td3_slots[row];
            const float yv = p.ring_rewards[sl] + ((1.0f - p.ring_dones[sl]) * p.gamma) * tv;
            const float hdl = p.huber_delta;
            auto term = [hdl](float e, float& d) {
              if (hdl > 0.0f) {
                d = fminf(fmaxf(e, -hdl), hdl);
                const float ae = fabsf(e);
                return ae <= hdl ? 0.5f * (e * e) : hdl * (ae - 0.5f * hdl);
              }
              d = 2.0f * e;
              return e * e;
            };
            float d1;
            float l = term(ldc(ws.v1 + row) - yv, d1);
            stc(p.dv1 + row, d1);
            if (twin) {
              float d2;
              l = l + term(ldc(ws.v2 + row) - yv, d2);
              stc(p.dv2 + row, d2);
            }
            if (p.loss_out) p.loss_out[row] = l;
          }
        }
      }
      __syncthreads();
    }
    if (!grid_sync(y, s_flag, nt * per, layer == 1 ? pre_p5() : pre_p7())) return;
  }

  // ---- P7: critics backward (dW2 / db2, dH1, dW3 / db3) ----
  {
    const int IT1 = (H1 + kRows - 1) / kRows, IT2 = (H2 + kRows - 1) / kRows;
    const int n_dx = RTT * CT1, n_dw2 = IT1 * CTW2, n_dw3 = IT2;
    const int per = n_dx + n_dw2 + n_dw3;  // the heavy input-gradient jobs first
    for (int j = b; j < nt * per; j += G) {
      XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
      const int ci = j / per, q = j % per;
      const Net n = ci ? c2 : c1;
      const int id = ci ? N_C2 : N_C1;
      float* dv = ci ? p.dv2 : p.dv1;
      float* grad = ci ? p.g_critic2 : p.g_critic1;
      const DZ d2 = dz_h2(ws.h2(id), H2, n.th + n.w3, 1, dv, 0.0f);
      if (q < n_dx) {
        const int rt = q / CT1, ct = q % CT1, c0 = ct * kCols;
        dx_tile(d2, rt * kTR, B, n.th + n.w2, H2, c0, min(kCols, H1 - c0), false, ws.h1(id),
                ws.dh1(ci), H1, no_head());
      } else if (q < n_dx + n_dw2) {
        const int t = q - n_dx, it = t / CTW2, ct = t % CTW2;
        dw_job(xsrc(ws.h1(id), H1, H1, false, true), slots, d2, H1, H2, it * kRows,
               ct * NTW * kCols, NTW, B, grad, n.w2, n.b2, n, no_adam());
      } else {
        const int it = q - n_dx - n_dw2;
        dw_job(xsrc(ws.h2(id), H2, H2, false, true), slots, dz_buf(dv, 1), H2, 1, it * kRows,
               0, 1, B, grad, n.w3, n.b3, n, no_adam());
      }
      __syncthreads();
    }
    // (the critics' Adam step sizes formed while the barrier waits)
    auto alphas = [&]() {
      c1.alpha = adam_alpha(p.critic1.lr, p.critic1.beta1, p.critic1.beta2, step_c1 + 1);
      if (twin) c2.alpha = adam_alpha(p.critic2.lr, p.critic2.beta1, p.critic2.beta2, step_c2 + 1);
    };
    if (!grid_sync(y, s_flag, nt * per, no_preb(), alphas)) return;
  }

  // ---- P8: critics dW1 / db1 + Adam, Adam of the rest (+ Polyak on policy steps); the
  // rest in chunks sized so the phase's jobs fill the grid. Stage 1: dW1 / db1 only ----
  {
    const int n_w1 = CTW1;                      // one in-feature tile (C <= 64)
    const int rest = c1.P - c1.w2, chunk = adam_chunk(rest, max(1, (G - nt * n_w1) / nt));
    const int n_ad = stage == 1 ? 0 : (rest + chunk - 1) / chunk;
    const int per = n_w1 + n_ad;
    p8_jobs = nt * per;
    for (int j = b; j < nt * per; j += G) {
      XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
      const int ci = j / per, q = j % per;
      const Net n = ci ? c2 : c1;
      const XaTdNet& opt = ci ? p.critic2 : p.critic1;
      float* grad = ci ? p.g_critic2 : p.g_critic1;
      float* tgt = pol ? (ci ? p.target_critic2.theta : p.target_critic1.theta) : nullptr;
      if (q < n_w1) {
        dw_job(sa_dense, slots, dz_buf(ws.dh1(ci), H1), C, H1, 0, q * NTW * kCols, NTW, B,
               grad, n.w1, n.b1, n, stage == 1 ? no_adam() : adam_opt(opt, tgt, p.tau));
      } else {
        const int lo = n.w2 + (q - n_w1) * chunk, hi = min(n.P, lo + chunk);
        const float omb1 = 1.0f - opt.beta1, omb2 = 1.0f - opt.beta2;
        adam_range(n, grad, lo, hi, omb1, omb2, opt.eps, tgt, p.tau);
      }
      __syncthreads();
    }
  }
  }  // stage <= 1

  // ---- stage 2, P8': the critics' Keras Adam (+ Polyak of their targets on policy steps)
  // from the all-reduced gradients, every parameter in chunks that fill the grid ----
  if (stage == 2) {
    c1.alpha = adam_alpha(p.critic1.lr, p.critic1.beta1, p.critic1.beta2, step_c1 + 1);
    if (twin) c2.alpha = adam_alpha(p.critic2.lr, p.critic2.beta1, p.critic2.beta2, step_c2 + 1);
    const int chunk = adam_chunk(c1.P, max(1, G / nt)), per = (c1.P + chunk - 1) / chunk;
    p8_jobs = nt * per;
    for (int j = b; j < nt * per; j += G) {
      const int ci = j / per, q = j % per;
      const Net n = ci ? c2 : c1;
      const XaTdNet& opt = ci ? p.critic2 : p.critic1;
      float* tgt = pol ? (ci ? p.target_critic2.theta : p.target_critic1.theta) : nullptr;
      const int lo = q * chunk, hi = min(n.P, lo + chunk);
      adam_range(n, ci ? p.g_critic2 : p.g_critic1, lo, hi, 1.0f - opt.beta1, 1.0f - opt.beta2,
                 opt.eps, tgt, p.tau, p.critic_grad_scale);
      __syncthreads();
    }
  }

  if (pol && (stage == 0 || stage == 2)) {
    if (!grid_sync(y, s_flag, p8_jobs)) return;
    // ---- P9 / P10: critic 1 (updated) on [s, pi(s)] ----
    const XSrc spa = xcat(xsrc(p.out_s, S, S, false, true), ws.pa, A, A, false, true);
    for (int layer = 1; layer <= 2; ++layer) {
      const int CT = layer == 1 ? CT1 : CT2;
      for (int j = b; j < RTT * CT; j += G) {
        XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
        const int rt = j / CT, ct = j % CT;
        if (layer == 1)
          fwd_job(spa, slots, rt * kTR, B, c1.th + c1.w1, c1.th + c1.b1, C, H1, ct * kCols,
                  ACT_RELU, ws.q1, true);
        else
          fwd_job(xsrc(ws.q1, H1, H1, false, true), slots, rt * kTR, B, c1.th + c1.w2,
                  c1.th + c1.b2, H1, H2, ct * kCols, ACT_RELU, ws.q2, true);
        __syncthreads();
      }
      if (!grid_sync(y, s_flag, RTT * CT, layer == 1 ? pre_p10() : pre_p11())) return;
    }
    // ---- P11: dH1 of -mean Q (dQ / dv = -1 / B per row), + the partials of
    // d pi(s) = dH1 W1[S + a][:]^T; the row tile's last job forms the actor's output
    // gradient d pi (1 - pi^2) ----
    const DZ dq2 = dz_h2(ws.q2, H2, c1.th + c1.w3, 1, nullptr, -1.0f / (float)B);
    for (int j = b; j < RTT * CT1; j += G) {
      XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
      const int rt = j / CT1, ct = j % CT1, c0 = ct * kCols;
      const Head hd{c1.th + c1.w1 + (size_t)S * H1, ws.hpp, ws.ticket(6, rt), 1, H1, A, ct, CT1,
                    true};
      if (dx_tile(dq2, rt * kTR, B, c1.th + c1.w2, H2, c0, min(kCols, H1 - c0), true, ws.q1,
                  ws.dq1, H1, hd)) {
        const int r0 = rt * kTR, nr = min(kTR, B - r0);
        for (int e = tid; e < nr * A; e += 256) {
          const int row = r0 + e / A, c = e % A;
          const float dp = head_total(ws.hpp, CT1, B, A, row, c);
          const float pv = ldc(ws.pa + row * A + c);
          stc(ws.dz3 + row * A + c, dp * (1.0f - pv * pv));
        }
      }
      __syncthreads();
    }
    if (!grid_sync(y, s_flag, RTT * CT1, pre_p13())) return;
    // ---- P13: actor backward (dW2 / db2, dH1, dW3 / db3) ----
    {
      const int IT1 = (H1 + kRows - 1) / kRows, IT2 = (H2 + kRows - 1) / kRows;
      const int n_dx = RTT * CT1, n_dw2 = IT1 * CTW2, n_dw3 = IT2;
      const DZ d2 = dz_h2(ws.h2(N_AC), H2, ac.th + ac.w3, A, ws.dz3, 0.0f);
      for (int j = b; j < n_dx + n_dw2 + n_dw3; j += G) {
        XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
        if (j < n_dx) {
          const int rt = j / CT1, ct = j % CT1, c0 = ct * kCols;
          dx_tile(d2, rt * kTR, B, ac.th + ac.w2, H2, c0, min(kCols, H1 - c0), false,
                  ws.h1(N_AC), ws.dh1a, H1, no_head());
        } else if (j < n_dx + n_dw2) {
          const int t = j - n_dx, it = t / CTW2, ct = t % CTW2;
          dw_job(xsrc(ws.h1(N_AC), H1, H1, false, true), slots, d2, H1, H2, it * kRows,
                 ct * NTW * kCols, NTW, B, p.g_actor, ac.w2, ac.b2, ac, no_adam());
        } else {
          const int it = j - n_dx - n_dw2;
          dw_job(xsrc(ws.h2(N_AC), H2, H2, false, true), slots, dz_buf(ws.dz3, A), H2, A,
                 it * kRows, 0, 1, B, p.g_actor, ac.w3, ac.b3, ac, no_adam());
        }
        __syncthreads();
      }
      auto alpha_ac = [&]() {
        ac.alpha = adam_alpha(p.actor.lr, p.actor.beta1, p.actor.beta2, step_ac + 1);
      };
      if (!grid_sync(y, s_flag, n_dx + n_dw2 + n_dw3, no_preb(), alpha_ac)) return;
    }
    // ---- P14: actor dW1 / db1 + Adam + Polyak, Adam + Polyak of the rest (stage 2:
    // dW1 / db1 only) ----
    {
      const int rest = ac.P - ac.w2, chunk = adam_chunk(rest, max(1, G - CTW1));
      const int n_ad = stage == 2 ? 0 : (rest + chunk - 1) / chunk;
      for (int j = b; j < CTW1 + n_ad; j += G) {
        XA_TD3_DSLOT((b == 0 && j == b) ? 8 * (int)y.n : -1);
        if (j < CTW1) {
          dw_job(xsrc(p.out_s, S, S, false, true), slots, dz_buf(ws.dh1a, H1), S, H1, 0,
                 j * NTW * kCols, NTW, B, p.g_actor, ac.w1, ac.b1, ac,
                 stage == 2 ? no_adam() : adam_opt(p.actor, p.target_actor.theta, p.tau));
        } else {
          const int lo = ac.w2 + (j - CTW1) * chunk, hi = min(ac.P, lo + chunk);
          const float omb1 = 1.0f - p.actor.beta1, omb2 = 1.0f - p.actor.beta2;
          adam_range(ac, p.g_actor, lo, hi, omb1, omb2, p.actor.eps, p.target_actor.theta, p.tau);
        }
        __syncthreads();
      }
    }
  }

  // ---- stage 3: the actor's Keras Adam + Polyak of the target actor from the all-reduced
  // gradient (scaled: the ranks' -mean Q gradients are summed) ----
  if (stage == 3) {
    ac.alpha = adam_alpha(p.actor.lr, p.actor.beta1, p.actor.beta2, step_ac + 1);
    const int chunk = adam_chunk(ac.P, G), per = (ac.P + chunk - 1) / chunk;
    for (int j = b; j < per; j += G) {
      const int lo = j * chunk, hi = min(ac.P, lo + chunk);
      adam_range(ac, p.g_actor, lo, hi, 1.0f - p.actor.beta1, 1.0f - p.actor.beta2, p.actor.eps,
                 p.target_actor.theta, p.tau, p.actor_grad_scale);
      __syncthreads();
    }
  }

  // the step counters, the noise counter and the next launch's barrier base and entry
  // base: written once every block of the launch has entered (read them)
  if (b == 0 && tid == 0) {
    if (!wait_entered(y)) return;
    *ws.ent_base = y.ent_target;
    if (stage == 0 || stage == 2) {
      *p.critic1.step += 1;
      if (twin) *p.critic2.step += 1;
    }
    if (pol && (stage == 0 || stage == 3)) *p.actor.step += 1;
    if (p.smooth && p.rng_counter && stage <= 1) *p.rng_counter += 1ull;
    *ws.base = y.target;
    *ws.epoch = y.epoch;
    // block 0's end (the last phase's tail may run on)
    if (XA_TD3_TRACE) ws.trace[15] = wall_clock64();
  }
}

// ---- the exploration step's actions (DDPG.get_step_actions, ddpg/agent.py:60-71):
// clip(tanh(actor(s)) + N(0, sigma) clipped, lo, hi) for the env states in ONE launch -- P1
// actor L1 on the states, P2 actor L2 with the L3 partials; each row tile's last job
// finishes tanh + noise (the same Philox draw as xa_noisy_actions) + clip. One grid
// barrier; block 0 bumps the noise counter at the end (every block read it at launch
// start) ----
__global__ __launch_bounds__(256) void td3_act_kernel(XaTd3ActArgs p) {
  __shared__ int s_flag;
  if (p.status && *(const volatile int*)p.status != 0) return;  // (as td3_update_kernel)
  const int G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  const int n = p.n, S = p.obs_dim, A = p.act_dim, H1 = p.h1, H2 = p.h2;
  const Ws ws = carve(p.workspace, n, H1, H2, A);
  Sync y;
  y.cnt = ws.cnt;
  y.abort_w = ws.abort_w;
  y.target = *ws.base;
  y.epoch = *ws.epoch + 1u;
  y.G = (unsigned)G;
  y.n = 0;
  y.status = p.status;
  y.trace = nullptr;
  y.ent = b == 0 && tid == 0 ? ws.ent : nullptr;
  y.ent_target = *ws.ent_base + (unsigned)G;
  y.ent_ok = 0;
  if (tid == 0) td3_bpre = 0;
#if XA_TD3_TRACE
  if (tid == 0) {
    td3_dslot = -1;
    td3_dbuf = ws.dtrace;
  }
#endif
  const uint64_t ctr = p.rng_counter ? *p.rng_counter : 0ull;
  XaTdNet d{};
  d.theta = const_cast<float*>(p.theta);
  const Net ac = make_net(d, S, H1, H2, A, false);
  const int RTT = (n + kTR - 1) / kTR;
  const int CT1 = (H1 + kCols - 1) / kCols, CT2 = (H2 + kCols - 1) / kCols;
  enter_launch(ws.ent);
  for (int j = b; j < RTT * CT1; j += G) {
    const int rt = j / CT1, ct = j % CT1;
    fwd_job(xsrc(p.states, S, S, false, false), nullptr, rt * kTR, n, ac.th + ac.w1,
            ac.th + ac.b1, S, H1, ct * kCols, ACT_RELU, ws.h1(N_AC));
    __syncthreads();
  }
  auto pre_act2 = [&]() {
    if (b >= RTT * CT2) return no_preb();
    const int ct = b % CT2;
    return PreB{ac.th + ac.w2, 1, H2, H1, ct * kCols, min(kCols, H2 - ct * kCols), false};
  };
  if (!grid_sync(y, s_flag, RTT * CT1, pre_act2())) return;
  for (int j = b; j < RTT * CT2; j += G) {
    const int rt = j / CT2, ct = j % CT2;
    const Head hd{ac.th + ac.w3, ws.hp3(N_AC), ws.ticket(N_AC, rt), A, 1, A, ct, CT2, false};
    if (fwd_job(xsrc(ws.h1(N_AC), H1, H1, false, true), nullptr, rt * kTR, n, ac.th + ac.w2,
                ac.th + ac.b2, H1, H2, ct * kCols, ACT_RELU, ws.h2(N_AC), false, hd)) {
      const int r0 = rt * kTR, nr = min(kTR, n - r0);
      for (int e = tid; e < nr * A; e += 256) {
        const int row = r0 + e / A, c = e % A;
        const float z = head_total(ws.hp3(N_AC), CT2, n, A, row, c) + ac.th[ac.b3 + c];
        float nz = 0.0f;
        if (p.sigma != 0.0f) {
          nz = philox_normal((uint32_t)row, (uint32_t)c, ctr, p.seed) * p.sigma;
          nz = fminf(fmaxf(nz, -p.noise_clip), p.noise_clip);
        }
        if (p.noise_out) p.noise_out[row * A + c] = nz;
        p.out[(int64_t)row * p.ld_out + c] = fminf(fmaxf(xa_tanhf(z) + nz, p.lo), p.hi);
      }
    }
    __syncthreads();
  }
  if (b == 0 && tid == 0) {
    if (!wait_entered(y)) return;
    *ws.ent_base = y.ent_target;
    if (p.bump && p.rng_counter) *p.rng_counter += 1ull;
    *ws.base = y.target;
    *ws.epoch = y.epoch;
  }
}

}  // namespace

extern "C" size_t xa_td3_update_workspace_bytes(int batch, int obs_dim, int act_dim, int h1,
                                                int h2) {
  (void)obs_dim;
  return carve(nullptr, batch, h1, h2, act_dim).total;
}

extern "C" int xa_td3_update(const XaTd3UpdateArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_td3_update: null args");
  const XaTd3UpdateArgs& a = *p;
  XA_CHECK_ARG(a.batch > 0 && a.obs_dim > 0 && a.act_dim > 0 && a.act_dim <= 4 && a.h1 > 0 &&
                   a.h2 > 0,
               "xa_td3_update: bad sizes");
  XA_CHECK_ARG(a.batch <= 256 && a.h1 <= kMaxK && a.h2 <= kMaxK && a.h1 % 4 == 0 &&
                   a.h2 % 4 == 0 &&
                   a.obs_dim + a.act_dim <= 64 && a.h2 * a.act_dim <= 2048 &&
                   a.batch * a.act_dim <= 1024,
               "xa_td3_update: sizes beyond the kernel's tiles (batch <= 256; h1, h2 <= %d and "
               "multiples of 4; act <= 4; obs + act <= 64; h2 act, batch act <= 2048, 1024)",
               kMaxK);
  XA_CHECK_ARG(a.ring_states && a.ring_new_states && a.ring_actions && a.ring_rewards &&
                   a.ring_dones && a.slots && a.workspace && a.dv1 && a.g_critic1 &&
                   (!a.twin || (a.dv2 && a.g_critic2 && a.critic2.theta && a.target_critic2.theta)) &&
                   (!a.actor_update || a.g_actor) && a.out_s && a.out_a && a.out_r && a.out_d &&
                   a.out_s2,
               "xa_td3_update: missing buffers");
  XA_CHECK_ARG(a.workspace_bytes >= carve(nullptr, a.batch, a.h1, a.h2, a.act_dim).total,
               "xa_td3_update: workspace too small");
  XA_CHECK_ARG(a.stage >= 0 && a.stage <= 3 && (a.stage != 3 || (a.actor_update && a.g_actor)),
               "xa_td3_update: stage must be 0 (whole step) or 1 / 2 / 3 (data parallel; "
               "stage 3 needs actor_update)");
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int G = a.n_blocks > 0 ? min(a.n_blocks, cus) : min(256, cus);
  const size_t lds = sizeof(float) * ((size_t)(kRows + kCols) * kMaxK + kAux);
  hipLaunchKernelGGL(td3_update_kernel, dim3(G), dim3(256), lds, (hipStream_t)stream, a);
  XA_CHECK_LAUNCH("xa_td3_update");
  return 0;
}

extern "C" size_t xa_td3_act_workspace_bytes(int n, int obs_dim, int act_dim, int h1, int h2) {
  (void)obs_dim;
  return carve(nullptr, n, h1, h2, act_dim).total;
}

extern "C" int xa_td3_act(const XaTd3ActArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_td3_act: null args");
  const XaTd3ActArgs& a = *p;
  XA_CHECK_ARG(a.n > 0 && a.n <= 256 && a.obs_dim > 0 && a.act_dim > 0 && a.act_dim <= 4 &&
                   a.h1 > 0 && a.h2 > 0 && a.h1 <= kMaxK && a.h2 <= kMaxK && a.h1 % 4 == 0 &&
                   a.h2 % 4 == 0 && a.obs_dim <= 64 && a.ld_out >= a.act_dim,
               "xa_td3_act: sizes beyond the kernel's tiles (n <= 256; h1, h2 <= %d and "
               "multiples of 4; act <= 4; obs <= 64)",
               kMaxK);
  XA_CHECK_ARG(a.states && a.theta && a.out && a.workspace &&
                   a.workspace_bytes >= carve(nullptr, a.n, a.h1, a.h2, a.act_dim).total,
               "xa_td3_act: missing buffers or workspace too small");
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // jobs per phase: (n / 32) x (h / 16); no more workgroups than the wider phase holds
  const int jobs = ((a.n + kTR - 1) / kTR) * ((max(a.h1, a.h2) + kCols - 1) / kCols);
  const int G = a.n_blocks > 0 ? min(a.n_blocks, cus) : min(min(jobs, 256), cus);
  const size_t lds = sizeof(float) * ((size_t)(kRows + kCols) * kMaxK + kAux);
  hipLaunchKernelGGL(td3_act_kernel, dim3(G), dim3(256), lds, (hipStream_t)stream, a);
  XA_CHECK_LAUNCH("xa_td3_act");
  return 0;
}
