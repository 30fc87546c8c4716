// f32 GEMM on v_mfma_f32_16x16x4_f32 with grouped-affine operand addressing, the
// building block of the CNN (NatureCNN-Conv1D, xagents/*/models/cnn*.cfg) and wide-MLP
// (TD3 / DDPG) forward and backward passes.
//
//   C(m, n) [+]= act( sum_k A(m, k) B(k, n) + bias(n) ) * gate(m, n)
//   A(m, k) = a[f(m) + g(k)],  f(m) = (m / a_pm) a_rm + (m % a_pm) a_sm,
//                              g(k) = (k / a_pk) a_rk + (k % a_pk) a_sk
//   B(k, n) = b[k b_ks + n b_ns]
//
// The grouped-affine A covers, without materialising anything:
//   * Keras Conv1D on (B, H, W, C) input (conv along W, H folded into the batch,
//     SURVEY Appendix B): rows m = (row, position p), columns k = (tap t, channel c)
//     and A(m, k) = act[row][stride p + t][c] = a[row W C + p stride C + k]
//   * its weight gradient (the im2col on the reduction index instead),
//   * transposed operands (plain strides) for dX = dY W^T and dW = X^T dY.
// u8 A operands (Atari frames) are scaled as the reference does,
// tf.cast(x, f32) / 255.0 (xagents/base.py:505-506).
//
// Tiles: 64 x 64 per 256-thread workgroup, 4 waves of 32 x 32 (2 x 2 MFMA tiles),
// K in steps of 16 staged through double-buffered LDS. K may be split over
// blockIdx.z; split partial sums are reduced in fixed order by a second kernel that
// applies the epilogue (deterministic, no atomics).
#include <algorithm>
#include <cstdlib>

#include "../../include/xagents_hip.h"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

constexpr int BM = 64, BN = 64, BK = 16, LDA = BM + 4, LDB = BN + 4;

typedef float f32x4 __attribute__((ext_vector_type(4)));

XA_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// (i / p) r + (i % p) s with 32-bit division (indices and group sizes fit in 31 bits;
// a 64-bit divide in the loader costs more than the MFMA work of a K step)
XA_DEV int64_t grouped(int i, int p, int64_t r, int64_t s) {
  if (p == 1) return (int64_t)i * r;
  const unsigned q = (unsigned)i / (unsigned)p;
  const unsigned m = (unsigned)i - q * (unsigned)p;
  return (int64_t)q * r + (int64_t)m * s;
}

XA_DEV float epilogue(float v, int n, const XaGemmArgs& g) {
  if (g.bias) v = v + g.bias[n];
  if (g.act == XA_ACT_RELU) v = fmaxf(v, 0.0f);
  else if (g.act == XA_ACT_TANH) v = xa_tanhf(v);
  return v;
}

XA_DEV void store_c(float v, int m, int n, const XaGemmArgs& g) {
  if (g.gate && !(g.gate[(int64_t)m * g.ld_gate + n] > 0.0f)) v = 0.0f;
  float* c = g.c + (int64_t)m * g.ldc + n;
  *c = g.beta ? *c + v : v;
}

// kernel argument: the public args plus the host's vectorisation verdicts. vec_a / vec_b:
// every 4-run a thread loads (along k for k-major A, along m otherwise; along n for n-major
// B, along k otherwise) is contiguous, aligned and entirely in or out of bounds, so it is
// one 16-B (f32) or 4-B (u8) load
struct XaGemmK {
  XaGemmArgs g;
  int vec_a, vec_b;
  int ones_m;  // a_ones_row: the constant-one row (M - 1), else -1 (gemm_kernel only)
  XaAdamApply ad;  // (gemm_kernel<..., ADAM = true> only) the epilogue's Adam step
  // (ADAM only) > 0: 1-D grid, XCD-aware tile order over xmap_nt column tiles (below)
  int xmap_nt;
};

template <bool U8>
XA_DEV void ld4(const void* base, int64_t off, float* d) {
  if (U8) {
    const uchar4 v = *reinterpret_cast<const uchar4*>(static_cast<const uint8_t*>(base) + off);
    d[0] = (float)v.x / 255.0f;
    d[1] = (float)v.y / 255.0f;
    d[2] = (float)v.z / 255.0f;
    d[3] = (float)v.w / 255.0f;
  } else {
    const f32x4 v = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + off);
    d[0] = v[0];
    d[1] = v[1];
    d[2] = v[2];
    d[3] = v[3];
  }
}

XA_DEV void zero4(float* d) { d[0] = d[1] = d[2] = d[3] = 0.0f; }

// A_KMAJOR: g(k) is unit stride (loader reads along k); otherwise along m.
// B_NMAJOR: b_ns == 1 (loader reads along n); otherwise along k.
// ADAM: the epilogue applies Keras Adam to the parameters the tile is the gradient of
// (xa_gemm_adam; one K split, no bias / activation / gate / beta, N % 4 == 0)
template <bool A_KMAJOR, bool B_NMAJOR, bool A_U8, bool ADAM = false>
// (ADAM: 4 blocks per CU -- the parameter / moment prefetch fits 121 VGPRs instead of 184)
__global__ __launch_bounds__(256, ADAM ? 4 : 1) void gemm_kernel(XaGemmK kargs) {
  const XaGemmArgs& g = kargs.g;
  const bool vec_a = kargs.vec_a, vec_b = kargs.vec_b;
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  int bx = (int)blockIdx.x, by = (int)blockIdx.y;
  if constexpr (ADAM) {
    if (kargs.xmap_nt > 0) {
      // consecutive workgroups go to consecutive XCDs, so ids x + 8 (n + xmap_nt j) all run
      // on XCD x: give them the xmap_nt column tiles of row tile x + 8 j -- the row tile's A
      // slice (the layer input, shared by every column tile) is then read into one L2, not
      // once per column tile from the fabric
      const int id = (int)blockIdx.x, r = id >> 3;
      by = r % kargs.xmap_nt;
      bx = (id & 7) + 8 * (r / kargs.xmap_nt);
      if (bx * BM >= g.M) return;
    }
  }
  const int m0 = bx * BM, n0 = by * BN;
  const int tiles_k = (g.K + BK - 1) / BK;
  const int per = (tiles_k + (int)gridDim.z - 1) / (int)gridDim.z;
  const int k_begin = blockIdx.z * per * BK;
  const int k_end = min(g.K, k_begin + per * BK);

  // this thread's load slots (4 A elements, 4 B elements per K tile)
  const int a_m = A_KMAJOR ? tid >> 2 : (tid & 15) * 4;
  const int a_k = A_KMAJOR ? (tid & 3) * 4 : tid >> 4;
  const int b_k = B_NMAJOR ? tid >> 4 : (tid & 3) * 4;
  const int b_n = B_NMAJOR ? (tid & 15) * 4 : tid >> 2;
  // a_ones_row: row ones_m of A is constant 1 (never read); runs start on 4-aligned m, and the
  // host's vec_a verdict is taken on the M - 1 real rows, so a 4-m run either lies below
  // ones_m or starts at it
  const int ones_m = kargs.ones_m;
  int64_t a_row[4];
  bool a_ok[4], a_one[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + a_m + (A_KMAJOR ? 0 : i);
    a_ok[i] = m < g.M;
    a_one[i] = m == ones_m;
    a_row[i] = a_ok[i] && !a_one[i] ? grouped(m, (int)g.a_pm, g.a_rm, g.a_sm) : 0;
  }
  const float* af = static_cast<const float*>(g.a);
  const uint8_t* au = static_cast<const uint8_t*>(g.a);

  float ra[4], rb[4];

  // interior fast path (as gemm_tile_kernel): fixed bases + k strides, no bounds tests
  const int m_real = ones_m >= 0 ? ones_m : g.M;
  const bool fast = vec_a && vec_b && (A_KMAJOR || g.a_pk == 1) && m0 + BM <= m_real &&
                    n0 + BN <= g.N && (k_end - k_begin) % BK == 0;
  int64_t fa = 0, fb = 0;
  const int64_t fa_k = A_KMAJOR ? 1 : g.a_rk, fb_k = g.b_ks;
  if (fast) {
    fa = A_KMAJOR ? a_row[0] + k_begin + a_k : a_row[0] + (int64_t)(k_begin + a_k) * g.a_rk;
    fb = (int64_t)(k_begin + b_k) * g.b_ks + (int64_t)(n0 + b_n) * g.b_ns;
  }
  auto load_fast = [&](int kt) {
    const int64_t dk = kt - k_begin;
    ld4<A_U8>(g.a, fa + dk * fa_k, ra);
    ld4<false>(g.b, fb + dk * fb_k, rb);
  };
  auto load = [&](int kt) {
    if (vec_a) {
      // one run: 4 k of row a_m (k-major) or 4 m at column a_k
      const int k = kt + a_k;
      if (a_ok[0] && k < k_end) {
        if (a_one[0]) {
          ra[0] = 1.0f;
          ra[1] = ra[2] = ra[3] = A_KMAJOR ? 1.0f : 0.0f;
        } else {
          ld4<A_U8>(g.a, a_row[0] + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk), ra);
        }
      } else {
        zero4(ra);
      }
    } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kt + a_k + (A_KMAJOR ? i : 0);
      const int ai = A_KMAJOR ? 0 : i;
      float v = 0.0f;
      if (a_ok[ai] && k < k_end) {
        if (g.a == nullptr || a_one[ai]) {
          v = 1.0f;
        } else {
          const int64_t off = a_row[ai] + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk);
          v = A_U8 ? (float)au[off] / 255.0f : af[off];
        }
      }
      ra[i] = v;
    }
    }
    if (vec_b) {
      const int k = kt + b_k, n = n0 + b_n;
      if (k < k_end && n < g.N) ld4<false>(g.b, (int64_t)k * g.b_ks + (int64_t)n * g.b_ns, rb);
      else zero4(rb);
    } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kt + b_k + (B_NMAJOR ? 0 : i);
      const int n = n0 + b_n + (B_NMAJOR ? i : 0);
      rb[i] = (k < k_end && n < g.N) ? g.b[(int64_t)k * g.b_ks + (int64_t)n * g.b_ns] : 0.0f;
    }
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      As[buf][(a_k + (A_KMAJOR ? i : 0)) * LDA + a_m + (A_KMAJOR ? 0 : i)] = ra[i];
      Bs[buf][(b_k + (B_NMAJOR ? 0 : i)) * LDB + b_n + (B_NMAJOR ? i : 0)] = rb[i];
    }
  };

  // ADAM: the parameters / moments of this thread's four float4 groups of the tile (group
  // f = tid + 256 q: row f / 16, columns 4 (f % 16) .. + 3; a wave's load covers 4 rows x
  // 256 contiguous bytes) are loaded before the main loop, in flight under the GEMM
  f32x4 pth[ADAM ? 4 : 1], pm[ADAM ? 4 : 1], pv[ADAM ? 4 : 1];
  int64_t pe[ADAM ? 4 : 1];
  if (ADAM) {
    const XaAdamApply& ad = kargs.ad;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = tid + 256 * q, m = m0 + (f >> 4), n = n0 + 4 * (f & 15);
      pe[q] = (m < g.M && n < g.N) ? (int64_t)m * g.ldc + n : -1;
      if (pe[q] >= 0) {
        pth[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ad.theta + pe[q]));
        pm[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ad.m + pe[q]));
        pv[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ad.v + pe[q]));
      }
    }
  }

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if (k_begin < k_end) {
    if (fast) load_fast(k_begin);
    else load(k_begin);
    stash(0);
    __syncthreads();
    int buf = 0;
    for (int kt = k_begin; kt < k_end; kt += BK) {
      const bool more = kt + BK < k_end;
      if (more) {
        if (fast) load_fast(kt + BK);
        else load(kt + BK);
      }
      const float* as = As[buf];
      const float* bs = Bs[buf];
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        const int kk = 4 * s + (lane >> 4);
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = as[kk * LDA + wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = bs[kk * LDB + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      if (more) stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  if (ADAM) {
    // the tile through LDS (the main loop ended on a barrier; the tile reuses the operand
    // stash), then every thread updates its four prefetched float4 groups
    constexpr int LDT = BN + 4;
    static_assert(2 * BK * LDA >= BM * LDT / 2 && 2 * BK * LDB >= BM * LDT / 2, "tile stash");
    float* const Ta = &As[0][0];  // rows 0 .. 31 (both stash buffers, contiguous)
    float* const Tb = &Bs[0][0];  // rows 32 .. 63
    auto T = [&](int r, int c) -> float& {
      return r < BM / 2 ? Ta[r * LDT + c] : Tb[(r - BM / 2) * LDT + c];
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          T(wm * 32 + i * 16 + 4 * (lane >> 4) + r, wn * 32 + j * 16 + (lane & 15)) = acc[i][j][r];
    __syncthreads();
    const XaAdamApply& ad = kargs.ad;
    const float alpha = adam_alpha(ad.lr, ad.beta1, ad.beta2, *ad.step);
    const float omb1 = 1.0f - ad.beta1, omb2 = 1.0f - ad.beta2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (pe[q] < 0) continue;
      const int f = tid + 256 * q, r = f >> 4, c = 4 * (f & 15);
      const f32x4 gq = *reinterpret_cast<const f32x4*>(&T(r, c));
      if (g.c) __builtin_nontemporal_store(gq, reinterpret_cast<f32x4*>(g.c + pe[q]));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = pth[q][u], mm = pm[q][u], vv = pv[q][u];
        adam_elem(gq[u] * ad.grad_scale, t, mm, vv, alpha, omb1, omb2, ad.eps);
        pth[q][u] = t;
        pm[q][u] = mm;
        pv[q][u] = vv;
      }
      __builtin_nontemporal_store(pth[q], reinterpret_cast<f32x4*>(ad.theta + pe[q]));
      __builtin_nontemporal_store(pm[q], reinterpret_cast<f32x4*>(ad.m + pe[q]));
      __builtin_nontemporal_store(pv[q], reinterpret_cast<f32x4*>(ad.v + pe[q]));
    }
    return;
  }
  // D(row = 4 (lane >> 4) + r, col = lane & 15) of each 16 x 16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= g.M || n >= g.N) continue;
        if (gridDim.z > 1) {
          g.partials[((int64_t)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][r];
        } else {
          store_c(epilogue(acc[i][j][r], n, g), m, n, g);
        }
      }
}

// ---------------------------------------------------------------------------
// Large-tile path: v_mfma_f32_32x32x2_f32 (A[i = l&31][k = l>>5], B[k = l>>5][j = l&31];
// D col = l&31, row = (r&3) + 8 (r>>2) + 4 (l>>5)), 4 waves of 64 x 64 (2 x 2 tiles of
// 32 x 32, 4 independent accumulators per wave), block (64 WM) x (64 WN) with
// WM WN = 4, K in steps of 32 through double-buffered LDS.
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int TBK = 32;

XA_DEV f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int WM, int WN, bool A_KMAJOR, bool B_NMAJOR, bool A_U8>
__global__ __launch_bounds__(256) void gemm_tile_kernel(XaGemmK kargs) {
  const XaGemmArgs& g = kargs.g;
  const bool vec_a = kargs.vec_a, vec_b = kargs.vec_b;
  // LDS row pitch: a k-major operand is stashed one float per row (4 rows per thread), so
  // a pitch = 1 (mod 8) spreads a wave's 32-lane write group over all 32 banks; an m- /
  // n-major operand is stashed as one 16-B write per thread (pitch a multiple of 4)
  constexpr int TBM = 64 * WM, TBN = 64 * WN;
  constexpr int TLA = A_KMAJOR ? TBM + 1 : TBM + 4, TLB = B_NMAJOR ? TBN + 4 : TBN + 1;
  constexpr int EA = TBM * TBK / 256, EB = TBN * TBK / 256;  // elements per thread
  __shared__ __attribute__((aligned(16))) float As[2][TBK * TLA];
  __shared__ __attribute__((aligned(16))) float Bs[2][TBK * TLB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int m0 = blockIdx.x * TBM, n0 = blockIdx.y * TBN;
  const int tiles_k = (g.K + TBK - 1) / TBK;
  const int per = (tiles_k + (int)gridDim.z - 1) / (int)gridDim.z;
  const int k_begin = blockIdx.z * per * TBK;
  const int k_end = min(g.K, k_begin + per * TBK);

  // A slots: k-major -> rows (tid >> 3) + 32 r, k quad (tid & 7);
  //          m-major -> m quad (tid % (TBM/4)) * 4, k rows tid / (TBM/4) + (1024/TBM) r
  constexpr int AQ = TBM / 4, AKR = 256 / AQ;  // m-major: threads per k row, k rows per pass
  constexpr int NA = A_KMAJOR ? TBM / 32 : 4;   // distinct m per thread
  int64_t a_row[NA];
  bool a_ok[NA];
#pragma unroll
  for (int r = 0; r < NA; ++r) {
    const int m = m0 + (A_KMAJOR ? (tid >> 3) + 32 * r : (tid % AQ) * 4 + r);
    a_ok[r] = m < g.M;
    a_row[r] = a_ok[r] ? grouped(m, (int)g.a_pm, g.a_rm, g.a_sm) : 0;
  }
  constexpr int BQ = TBN / 4, BKR = 256 / BQ;
  const float* af = static_cast<const float*>(g.a);
  const uint8_t* au = static_cast<const uint8_t*>(g.a);
  float ra[EA], rb[EB];

  // Interior fast path: every row / column of the tile exists, the split's K range is whole
  // K steps, both operands load as 16-B runs and A's k offset is linear (no im2col on k).
  // Then each run's address is a base fixed at k_begin plus (kt - k_begin) x its k stride,
  // and the loads need no bounds tests or index arithmetic per step.
  const bool a_lin = A_KMAJOR || g.a_pk == 1;
  const bool fast = vec_a && vec_b && a_lin && m0 + TBM <= g.M && n0 + TBN <= g.N &&
                    (k_end - k_begin) % TBK == 0;
  constexpr int RA = EA / 4, RB = EB / 4;
  int64_t a_base[RA], b_base[RB];
  int64_t a_kstride = 1, b_kstride = g.b_ks;
  if (fast) {
#pragma unroll
    for (int r = 0; r < RA; ++r) {
      if (A_KMAJOR) {
        a_base[r] = a_row[r] + k_begin + (tid & 7) * 4;
      } else {
        a_base[r] = a_row[0] + (int64_t)(k_begin + tid / AQ + AKR * r) * g.a_rk;
      }
    }
    a_kstride = A_KMAJOR ? 1 : g.a_rk;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int n = B_NMAJOR ? n0 + (tid % BQ) * 4 : n0 + (tid >> 3) + 32 * r;
      const int k = B_NMAJOR ? k_begin + tid / BQ + BKR * r : k_begin + (tid & 7) * 4;
      b_base[r] = (int64_t)k * g.b_ks + (int64_t)n * g.b_ns;
    }
  }
  auto load_fast = [&](int kt) {
    const int64_t dk = kt - k_begin;
#pragma unroll
    for (int r = 0; r < RA; ++r) ld4<A_U8>(g.a, a_base[r] + dk * a_kstride, ra + 4 * r);
#pragma unroll
    for (int r = 0; r < RB; ++r) ld4<false>(g.b, b_base[r] + dk * b_kstride, rb + 4 * r);
  };

  auto load = [&](int kt) {
    if (vec_a) {
#pragma unroll
      for (int r = 0; r < EA / 4; ++r) {
        // k-major: row r, k quad (tid & 7); m-major: 4 m from (tid % AQ) 4, k row r
        const int mi = A_KMAJOR ? r : 0;
        const int k = A_KMAJOR ? kt + (tid & 7) * 4 : kt + tid / AQ + AKR * r;
        if (a_ok[mi] && k < k_end)
          ld4<A_U8>(g.a, a_row[mi] + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk), ra + 4 * r);
        else zero4(ra + 4 * r);
      }
    } else {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      int mi, k;
      if (A_KMAJOR) {
        mi = e >> 2;
        k = kt + (tid & 7) * 4 + (e & 3);
      } else {
        mi = e & 3;
        k = kt + tid / AQ + AKR * (e >> 2);
      }
      float v = 0.0f;
      if (a_ok[mi] && k < k_end) {
        if (g.a == nullptr) {
          v = 1.0f;
        } else {
          const int64_t off = a_row[mi] + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk);
          v = A_U8 ? (float)au[off] / 255.0f : af[off];
        }
      }
      ra[e] = v;
    }
    }
    if (vec_b) {
#pragma unroll
      for (int r = 0; r < EB / 4; ++r) {
        const int n = B_NMAJOR ? n0 + (tid % BQ) * 4 : n0 + (tid >> 3) + 32 * r;
        const int k = B_NMAJOR ? kt + tid / BQ + BKR * r : kt + (tid & 7) * 4;
        if (k < k_end && n < g.N) ld4<false>(g.b, (int64_t)k * g.b_ks + (int64_t)n * g.b_ns, rb + 4 * r);
        else zero4(rb + 4 * r);
      }
    } else {
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      int n, k;
      if (B_NMAJOR) {
        n = n0 + (tid % BQ) * 4 + (e & 3);
        k = kt + tid / BQ + BKR * (e >> 2);
      } else {
        n = n0 + (tid >> 3) + 32 * (e >> 2);
        k = kt + (tid & 7) * 4 + (e & 3);
      }
      rb[e] = (k < k_end && n < g.N) ? g.b[(int64_t)k * g.b_ks + (int64_t)n * g.b_ns] : 0.0f;
    }
    }
  };
  auto stash = [&](int buf) {
    if (A_KMAJOR) {
#pragma unroll
      for (int e = 0; e < EA; ++e)
        As[buf][((tid & 7) * 4 + (e & 3)) * TLA + (tid >> 3) + 32 * (e >> 2)] = ra[e];
    } else {
#pragma unroll
      for (int r = 0; r < EA / 4; ++r)
        *reinterpret_cast<f32x4*>(&As[buf][(tid / AQ + AKR * r) * TLA + (tid % AQ) * 4]) =
            f32x4{ra[4 * r], ra[4 * r + 1], ra[4 * r + 2], ra[4 * r + 3]};
    }
    if (B_NMAJOR) {
#pragma unroll
      for (int r = 0; r < EB / 4; ++r)
        *reinterpret_cast<f32x4*>(&Bs[buf][(tid / BQ + BKR * r) * TLB + (tid % BQ) * 4]) =
            f32x4{rb[4 * r], rb[4 * r + 1], rb[4 * r + 2], rb[4 * r + 3]};
    } else {
#pragma unroll
      for (int e = 0; e < EB; ++e)
        Bs[buf][((tid & 7) * 4 + (e & 3)) * TLB + (tid >> 3) + 32 * (e >> 2)] = rb[e];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  if (k_begin < k_end) {
    if (fast) load_fast(k_begin);
    else load(k_begin);
    stash(0);
    __syncthreads();
    int buf = 0;
    for (int kt = k_begin; kt < k_end; kt += TBK) {
      const bool more = kt + TBK < k_end;
      if (more) {
        if (fast) load_fast(kt + TBK);
        else load(kt + TBK);
      }
      const float* as = As[buf] + wm * 64 + (lane & 31);
      const float* bs = Bs[buf] + wn * 64 + (lane & 31);
#pragma unroll
      for (int s2 = 0; s2 < TBK / 2; ++s2) {
        const int kk = 2 * s2 + (lane >> 5);
        const float a0 = as[kk * TLA], a1 = as[kk * TLA + 32];
        const float b0 = bs[kk * TLB], b1 = bs[kk * TLB + 32];
        acc[0][0] = mfma32(a0, b0, acc[0][0]);
        acc[0][1] = mfma32(a0, b1, acc[0][1]);
        acc[1][0] = mfma32(a1, b0, acc[1][0]);
        acc[1][1] = mfma32(a1, b1, acc[1][1]);
      }
      if (more) stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int n = n0 + wn * 64 + 32 * j + (lane & 31);
        if (m >= g.M || n >= g.N) continue;
        if (gridDim.z > 1) {
          g.partials[((int64_t)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][r];
        } else {
          store_c(epilogue(acc[i][j][r], n, g), m, n, g);
        }
      }
}

// ---------------------------------------------------------------------------
// Small-M path, both operands k-major: C[M, N] = A[M, K] B[K, N] with A(m, k) = a[m lda + k]
// and B(k, n) = b[n ldb + k] -- the dense layer's input gradient dX = dY W^T at batch
// M <= 64 (DQN's 64), where 64-row M tiles leave most CUs idle. K = 128 CH.
// A unit is a strip of 16 columns n x every row m; the wave that owns a unit's K part
// streams its 16 rows of b along k from HBM straight into MFMA operand registers (lane
// (q = l >> 4, i = l & 15) loads b[n0 + i][k0 + 4q .. 4q + 3], one float4 that feeds the 4
// MFMAs of a 16-k step in a permuted k order: no LDS staging, no transpose) and reads A, in
// the same k order, from LDS, where ALL of A stays resident: no A load sits in the K loop,
// so nothing queues behind the B prefetches in the in-order memory counter.
// 512 threads = 8 waves = 2 units x 4 K parts; the grid is persistent (<= one workgroup
// per CU) and walks rounds of 2 units per workgroup; each wave's B ring spans two rounds'
// chunks and runs 2 CH - 1 chunks ahead. At a round's end the 4 K parts are combined through LDS in part order and wave p finishes m
// tile p (gate values fetched when the round started, ahead of the prefetches).
// ---------------------------------------------------------------------------
constexpr int RS_KP = 4, RS_UPR = 2;
// rounds the B ring spans (the round loop is unrolled by this): 2 keeps 2 CH - 1 chunks of B
// in flight per wave (3 / 4 measured slower, profiles/r04m_smallm_ring_and_k_ab.txt)
constexpr int RS_NR = 2;
// Resident-A row layout, conflict-free for the lane groups of ds_read_b128 (MI355X_MICROARCH.md
// LDS table: 4 groups of 16 lanes, bank (a/4) mod 64): element k = 16 b + 4 q + j of a row
// sits at q SR + 4 b + j -- the k quads q = 0..3 of every 16-k step in 4 sub-rows whose
// stride SR is a multiple of 256 B -- and rows are PA = 4 SR + 4 floats apart, so lane
// (lq, li) reads its quad at 16-B slot li + b (mod 16) of the bank row: 16 distinct slots in
// every lane group (the plain k-major row with a +4 pad put two lanes of every group on
// one slot).
template <int K>
constexpr int rs_sr() { return K / 4 > 64 ? K / 4 : 64; }
template <int K>
constexpr int rs_pa() { return 4 * rs_sr<K>() + 4; }

template <int MT, int CH, bool GATE>
__global__ __launch_bounds__(512) void gemm_smallm_res_kernel(XaGemmArgs g, int rounds) {
  constexpr int K = 128 * CH, KQ = K / RS_KP, SR = rs_sr<K>(), PA = rs_pa<K>();
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* As = sm;                       // [MT 16][PA], sub-row layout above
  float* red = sm + MT * 16 * PA;       // [RS_UPR][MT][RS_KP - 1][256] (a tile's own part stays in registers)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kp = w % RS_KP, us = w / RS_KP;
  const int li = lane & 15, lq = lane >> 4;
  const int M = g.M, N = g.N;
  const int units = (N + 15) / 16;
  const float* af = static_cast<const float*>(g.a);
  // A into LDS: every thread's PER float4 loads issued before the B ring's first loads and
  // before any LDS write (a load -> wait -> write loop serialised PER round trips: 17.5k
  // cycles of prologue at M = 64, profiles/r04y_smallm_stamps.txt)
  constexpr int PER = MT * 16 * (K / 4) / 512;
  static_assert(PER * 512 == MT * 16 * (K / 4), "A slots per thread");
  f32x4 va[PER];
  int va_at[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    // 32 consecutive threads: 8 blocks b x the 4 quads q, b fastest -- 512 contiguous bytes
    // of the global row, and every 8-lane group of the ds_write_b128 one 128-B run of a
    // sub-row
    const int sl = tid + 512 * i;
    const int m = sl / (K / 4), rem = sl - m * (K / 4);
    const int q = (rem >> 3) & 3, b = ((rem >> 5) << 3) + (rem & 7);
    va_at[i] = m * PA + q * SR + 4 * b;
    va[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (m < M) va[i] = *reinterpret_cast<const f32x4*>(af + (int64_t)m * g.a_rm + 16 * b + 4 * q);
  }
  auto unit_of = [&](int r) { return (r * (int)gridDim.x + (int)blockIdx.x) * RS_UPR + us; };
  auto brow = [&](int r) {
    const int n = min(unit_of(r) * 16 + li, N - 1);
    return g.b + (int64_t)n * g.b_ns + kp * KQ + 4 * lq;
  };
  // B ring over the flattened chunk sequence gi = r CH + c of this wave's rounds: RS_R slots
  // (RS_NR rounds), chunk gi + RS_R - 1 fetched while chunk gi is computed
  constexpr int RS_R = RS_NR * CH;
  f32x4 rb[RS_R][2];
  auto load_b = [&](int gi, f32x4 (&dst)[2]) {
    const float* p = brow(gi / CH) + 32 * (gi % CH);
    dst[0] = *reinterpret_cast<const f32x4*>(p);
    dst[1] = *reinterpret_cast<const f32x4*>(p + 16);
  };
#pragma unroll
  for (int gi = 0; gi < RS_R - 1; ++gi) load_b(gi, rb[gi]);
#pragma unroll
  for (int i = 0; i < PER; ++i) *reinterpret_cast<f32x4*>(As + va_at[i]) = va[i];
  __syncthreads();
  const float* as = As + li * PA + lq * SR + kp * (KQ / 4);  // k = kp KQ + 16 b' + 4 lq + j
  const int mt_fin = min(kp, MT - 1);  // the m tile this wave finishes (kp < MT)
  for (int r0 = 0; r0 < rounds; r0 += RS_NR) {
#pragma unroll
    for (int par = 0; par < RS_NR; ++par) {
      const int r = r0 + par;
      const int unit = unit_of(r);
      const bool live = unit < units;
      const int n = unit * 16 + li;
      float gt[4] = {1.0f, 1.0f, 1.0f, 1.0f};
      if (GATE) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = min(16 * mt_fin + 4 * lq + q, M - 1);
          gt[q] = g.gate[(int64_t)m * g.ld_gate + min(n, N - 1)];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int u = par * CH + c;  // this chunk's slot
        // chunk gi + RS_R - 1 (clamped rows past the last round; unused) into the slot
        // the previous chunk freed
        load_b(r * CH + c + RS_R - 1, rb[(u + RS_R - 1) % RS_R]);
        __builtin_amdgcn_sched_barrier(0);
        if (live) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 aq[MT];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              aq[mt] = *reinterpret_cast<const f32x4*>(as + mt * 16 * PA + 8 * c + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int mt = 0; mt < MT; ++mt)
                acc[mt] = mfma4(aq[mt][j], rb[u][h][j], acc[mt]);
          }
        }
      }
      // slot of part p in m tile mt's scratch: p, or p - 1 past the finishing wave mt
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (mt == kp) continue;
        const int slot = kp < mt ? kp : kp - 1;
        *reinterpret_cast<f32x4*>(red + ((us * MT + mt) * (RS_KP - 1) + slot) * 256 + 4 * lane) =
            acc[mt];
      }
      __syncthreads();
      if (kp < MT && live && n < N) {
        f32x4 own = acc[0];
#pragma unroll
        for (int mt = 1; mt < MT; ++mt)
          if (mt == kp) own = acc[mt];
        f32x4 part[RS_KP - 1];
#pragma unroll
        for (int p = 0; p < RS_KP - 1; ++p)
          part[p] = *reinterpret_cast<const f32x4*>(red + ((us * MT + kp) * (RS_KP - 1) + p) * 256 + 4 * lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = 0.0f;
#pragma unroll
          for (int p = 0; p < RS_KP; ++p) v += p == kp ? own[q] : part[p < kp ? p : p - 1][q];
          const int m = 16 * kp + 4 * lq + q;
          if (m < M) {
            v = epilogue(v, n, g);
            if (GATE && !(gt[q] > 0.0f)) v = 0.0f;
            float* cp = g.c + (int64_t)m * g.ldc + n;
            *cp = g.beta ? *cp + v : v;
          }
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// Few-column dense layer (the network heads: N <= 8 Q values / logits / values over K <= 4096
// hidden units): one wave per output row m, lane l accumulates k = l, l + 64, ... for every
// column in registers, then a fixed-order xor butterfly over the wave (deterministic), and
// lane n applies bias / activation / gate / beta to column n. One launch without a K split:
// the tile path's split + reduce took ~10 + ~5 us for these shapes (profiles/r04aa C3
// timeline), latency, not work.
// ---------------------------------------------------------------------------
constexpr int RD_MAXN = 8;

// lane n (< N) returns column n of row m (epilogue applied); other lanes 0
XA_DEV float rowdot_row(const XaGemmArgs& g, int m, int lane) {
  const float* a = static_cast<const float*>(g.a) + (int64_t)m * g.a_rm;
  float acc[RD_MAXN];
#pragma unroll
  for (int n = 0; n < RD_MAXN; ++n) acc[n] = 0.0f;
  // RD_U k steps per pass with every load of the pass issued before the FMAs (one memory
  // round trip per pass instead of one per k step: K = 512 is one pass)
  constexpr int RD_U = 8;
  for (int k0 = lane; k0 < g.K; k0 += 64 * RD_U) {
    float av[RD_U], wv[RD_U][RD_MAXN];
#pragma unroll
    for (int u = 0; u < RD_U; ++u) {
      const int k = k0 + 64 * u;
      const bool in = k < g.K;
      av[u] = in ? a[k] : 0.0f;
      const float* w = g.b + (int64_t)(in ? k : 0) * g.b_ks;
#pragma unroll
      for (int n = 0; n < RD_MAXN; ++n)
        wv[u][n] = (in && n < g.N) ? w[(int64_t)n * g.b_ns] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < RD_U; ++u)
#pragma unroll
      for (int n = 0; n < RD_MAXN; ++n) acc[n] = fmaf(av[u], wv[u][n], acc[n]);
  }
  float v = 0.0f;
#pragma unroll
  for (int n = 0; n < RD_MAXN; ++n) {
    float t = acc[n];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if (lane == n) v = t;
  }
  return lane < g.N ? epilogue(v, lane, g) : 0.0f;
}

__global__ __launch_bounds__(256) void gemm_rowdot_kernel(XaGemmArgs g) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= g.M) return;
  const float v = rowdot_row(g, m, lane);
  if (lane < g.N) store_c(v, m, lane, g);
}

// DQN's per-row heads fused into the Q head's row-dot launch (one launch fewer per use):
// mode 0 (act, dqn/agent.py:107-116): actions[m] = first argmax of the row's Q values;
// mode 1 (TD, dqn/agent.py:118-171): the head is the TARGET network's, row b = sample b:
// exactly xa_dqn_td_grad's arithmetic (offpolicy.hip dqn_td_kernel) with Qt(s') taken from
// the lanes instead of memory; the optimizer step bump rides along
XA_DEV void dqn_row_step(const XaGemmArgs& g, const XaDqnHeadArgs& d, int m, int lane, float v);

__global__ __launch_bounds__(256) void dqn_head_kernel(XaGemmArgs g, XaDqnHeadArgs d) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d.mode == 1 && d.adam_step && blockIdx.x == 0 && threadIdx.x == 0) d.adam_step[0] += 1;
  if (m >= g.M) return;
  const float v = rowdot_row(g, m, lane);
  if (lane < g.N) store_c(v, m, lane, g);
  dqn_row_step(g, d, m, lane, v);
}

// the per-row DQN step after the head's row-dot (lane n < A holds Q[m][n])
XA_DEV void dqn_row_step(const XaGemmArgs& g, const XaDqnHeadArgs& d, int m, int lane, float v) {
  const int A = g.N;
  float qv[RD_MAXN];
#pragma unroll
  for (int n = 0; n < RD_MAXN; ++n) qv[n] = __shfl(v, n);
  if (d.mode == 0) {
    if (lane == 0) {
      int best = 0;
      float bv = qv[0];
#pragma unroll
      for (int a = 1; a < RD_MAXN; ++a)
        if (a < A && qv[a] > bv) {
          bv = qv[a];
          best = a;
        }
      d.actions[m] = best;
    }
    return;
  }
  const int b = m;
  float vn;
  if (d.q_next_online) {
    const float* qo = d.q_next_online + (int64_t)b * A;
    int best = 0;
    float bv = qo[0];
    for (int a = 1; a < A; ++a)
      if (qo[a] > bv) {
        bv = qo[a];
        best = a;
      }
    vn = qv[0];
#pragma unroll
    for (int a = 1; a < RD_MAXN; ++a)
      if (a == best) vn = qv[a];
  } else {
    vn = qv[0];
#pragma unroll
    for (int a = 1; a < RD_MAXN; ++a)
      if (a < A) vn = fmaxf(vn, qv[a]);
  }
  if (d.dones[b] != 0.0f) vn = 0.0f;
  const float y = vn * d.gamma + d.rewards[b];
  const int ab = d.act[b];
  const float diff = y - d.q[(int64_t)b * A + ab];
  float dqa, l;
  if (d.huber > 0.0f) {
    const float ad = fabsf(diff);
    dqa = -fminf(fmaxf(diff, -d.huber), d.huber) / (float)A;
    l = (ad <= d.huber ? 0.5f * (diff * diff) : d.huber * (ad - 0.5f * d.huber)) / (float)A;
  } else {
    dqa = (-2.0f * diff) / (float)A;
    l = (diff * diff) / (float)A;
  }
  if (lane < A) d.dq[(int64_t)b * A + lane] = lane == ab ? dqa : 0.0f;
  if (lane == 0 && d.loss) d.loss[b] = l;
}

// A dense layer's split-K reduce and the row-dot head that reads it (the NatureCNN Q head over
// the 512 hidden units), with DQN's per-row step when asked, in ONE launch instead of two
// (xa_gemm's wide split reduce, then xa_gemm's row-dot / xa_dqn_head): one 1024-thread
// workgroup per row m. Stage 1 sums every output of the row exactly as
// gemm_split_reduce_wide_kernel does (wave w: the contiguous split piece w, in split order;
// the 16 pieces combined in wave order; the dense epilogue), with every load of a row's piece
// in flight at once, and stores the row (the backward's operand); stage 2 runs rowdot_row's
// arithmetic on the row from LDS and dqn_head_kernel's per-row step: bit-identical to the two
// launches.
constexpr int DH_NCH = 8;  // 64-output chunks per row: dense N <= 512

XA_DEV float rowdot_lds(const XaGemmArgs& g, const float* arow, int lane) {
  float acc[RD_MAXN];
#pragma unroll
  for (int n = 0; n < RD_MAXN; ++n) acc[n] = 0.0f;
  constexpr int RD_U = 8;  // (rowdot_row's pass structure and order)
  for (int k0 = lane; k0 < g.K; k0 += 64 * RD_U) {
    float av[RD_U], wv[RD_U][RD_MAXN];
#pragma unroll
    for (int u = 0; u < RD_U; ++u) {
      const int k = k0 + 64 * u;
      const bool in = k < g.K;
      av[u] = in ? arow[k] : 0.0f;
      const float* w = g.b + (int64_t)(in ? k : 0) * g.b_ks;
#pragma unroll
      for (int n = 0; n < RD_MAXN; ++n)
        wv[u][n] = (in && n < g.N) ? w[(int64_t)n * g.b_ns] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < RD_U; ++u)
#pragma unroll
      for (int n = 0; n < RD_MAXN; ++n) acc[n] = fmaf(av[u], wv[u][n], acc[n]);
  }
  float v = 0.0f;
#pragma unroll
  for (int n = 0; n < RD_MAXN; ++n) {
    float t = acc[n];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if (lane == n) v = t;
  }
  return lane < g.N ? epilogue(v, lane, g) : 0.0f;
}

__global__ __launch_bounds__(1024) void dense_head_kernel(XaGemmArgs dn, int splits, XaGemmArgs hd,
                                                          XaDqnHeadArgs q, int mode) {
  __shared__ float part[16][64 * DH_NCH];
  __shared__ float hrow[64 * DH_NCH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m = blockIdx.x;
  const int N = dn.N;
  const int64_t total = (int64_t)dn.M * N;
  const int per = (splits + 15) / 16;
  const int z0 = w * per, z1 = min(splits, z0 + per);
  const float* src = dn.partials + (int64_t)m * N + lane;
  float acc[DH_NCH];
#pragma unroll
  for (int c = 0; c < DH_NCH; ++c) acc[c] = 0.0f;
  for (int z = z0; z < z1; z += 8) {
    float v[DH_NCH][8];
#pragma unroll
    for (int c = 0; c < DH_NCH; ++c)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[c][u] = (z + u < z1 && 64 * c + lane < N) ? src[(int64_t)(z + u) * total + 64 * c] : 0.0f;
#pragma unroll
    for (int c = 0; c < DH_NCH; ++c)
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (z + u < z1) acc[c] = acc[c] + v[c][u];
  }
#pragma unroll
  for (int c = 0; c < DH_NCH; ++c) part[w][64 * c + lane] = acc[c];
  __syncthreads();
  const int t = threadIdx.x;
  if (t < N) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = s + part[i][t];
    const float h = epilogue(s, t, dn);
    store_c(h, m, t, dn);
    hrow[t] = h;
  }
  __syncthreads();
  if (w != 0) return;
  if (mode == 1 && q.adam_step && m == 0 && lane == 0) q.adam_step[0] += 1;
  const float v = rowdot_lds(hd, hrow, lane);
  if (lane < hd.N) store_c(v, m, lane, hd);
  if (mode >= 0) dqn_row_step(hd, q, m, lane, v);
}

constexpr int SK_MAXK_H = 8;  // (the head width bound of xa_head_bwd, as SK_MAXK)

// A row-dot head's backward in one launch (xa_head_bwd): blocks [0, nbx) the input gradient
// (one thread per (m, k): gemm_smallk_kernel's arithmetic), the rest the [W; b] gradient (one
// thread per (k, a) of K + 1 rows, k fastest so a row m of x is read coalesced; m-order fmaf)
struct HeadBwd {
  const float *x, *dz, *W, *gate;
  int M, K, A;
  float* dx;
  int beta;
  float *gw, *gb;
  int accumulate, nbx;
};

__global__ __launch_bounds__(256) void head_bwd_kernel(HeadBwd h) {
  if ((int)blockIdx.x < h.nbx) {
    const int64_t e = blockIdx.x * 256ll + threadIdx.x;
    if (e >= (int64_t)h.M * h.K) return;
    const int m = (int)(e / h.K), k = (int)(e - (int64_t)m * h.K);
    const float* a = h.dz + (int64_t)m * h.A;
    const float* b = h.W + (int64_t)k * h.A;
    float v = 0.0f;
#pragma unroll
    for (int j = 0; j < SK_MAXK_H; ++j)
      if (j < h.A) v = fmaf(a[j], b[j], v);
    if (h.gate && !(h.gate[e] > 0.0f)) v = 0.0f;
    h.dx[e] = h.beta ? h.dx[e] + v : v;
    return;
  }
  const int o = ((int)blockIdx.x - h.nbx) * 256 + (int)threadIdx.x;  // (row r, a), r fastest
  const int rows = h.K + 1;
  if (o >= rows * h.A) return;
  const int a = o / rows, r = o - a * rows;
  // m-order chains; the loads of HB_U rows issued together (one load round trip per HB_U
  // rows, not per row: 28 -> ~3 us at the DQN head's M = 64, profiles/r06l_*)
  constexpr int HB_U = 16;
  float acc = 0.0f;
  const bool wrow = r < h.K;
  for (int m0 = 0; m0 < h.M; m0 += HB_U) {
    float xv[HB_U], dv[HB_U];
#pragma unroll
    for (int u = 0; u < HB_U; ++u) {
      const int m = m0 + u;
      xv[u] = m < h.M && wrow ? h.x[(int64_t)m * h.K + r] : 0.0f;
      dv[u] = m < h.M ? h.dz[(int64_t)m * h.A + a] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < HB_U; ++u)
      if (m0 + u < h.M) acc = wrow ? fmaf(xv[u], dv[u], acc) : acc + dv[u];
  }
  if (wrow) {
    if (h.gw) {
      float* p = h.gw + (int64_t)r * h.A + a;
      *p = h.accumulate ? *p + acc : acc;
    }
  } else if (h.gb) {
    h.gb[a] = h.accumulate ? h.gb[a] + acc : acc;
  }
}

// Few-k GEMM (K <= 8: the network heads' input gradient dZ W^T, K = the head width): one
// thread per output, its K products in k order, the usual epilogue (gate / beta).
constexpr int SK_MAXK = 8;

__global__ __launch_bounds__(256) void gemm_smallk_kernel(XaGemmArgs g) {
  const int64_t e = blockIdx.x * 256ll + threadIdx.x;
  if (e >= (int64_t)g.M * g.N) return;
  const int m = (int)(e / g.N), n = (int)(e - (int64_t)m * g.N);
  const float* a = static_cast<const float*>(g.a) + (int64_t)m * g.a_rm;
  const float* b = g.b + (int64_t)n * g.b_ns;
  float v = 0.0f;
#pragma unroll
  for (int k = 0; k < SK_MAXK; ++k)
    if (k < g.K) v = fmaf(a[k], b[(int64_t)k * g.b_ks], v);
  store_c(epilogue(v, n, g), m, n, g);
}

bool smallk_ok(const XaGemmArgs& g) {
  return !g.force_small && !g.a_ones_row && g.a != nullptr && !g.a_u8 && g.a_pm == 1 &&
         g.a_pk == 1 && g.a_rk == 1 && g.K <= SK_MAXK && (int64_t)g.M * g.N < (1ll << 31);
}

// the row-dot path's contract: f32 A with plain rows (A(m, k) = a[m lda + k]), N <= 8,
// K <= 4096, no split requested by the caller beyond the default
bool rowdot_ok(const XaGemmArgs& g) {
  return !g.force_small && !g.a_ones_row && g.a != nullptr && !g.a_u8 && g.a_pm == 1 &&
         g.a_pk == 1 && g.a_rk == 1 && g.N <= RD_MAXN && g.K <= 4096 && g.M <= (1 << 20);
}


// ---------------------------------------------------------------------------
// Skinny path (weight gradients of the convs: M, N <= 256 / 64, K = rows x positions in
// the millions): one wave per workgroup owns a 32 x 32 output tile and a K range; the
// operands come straight from global memory (A rows / B rows are contiguous along m / n
// for these shapes), 8 K-pairs in flight, one v_mfma_f32_32x32x2_f32 per pair.
// ---------------------------------------------------------------------------
template <bool A_U8>
__global__ __launch_bounds__(64) void gemm_skinny_kernel(XaGemmArgs g) {
  const int lane = threadIdx.x;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int kp = (g.K + 1) / 2;  // K pairs
  const int per = (kp + (int)gridDim.z - 1) / (int)gridDim.z;
  const int p_begin = blockIdx.z * per, p_end = min(kp, p_begin + per);
  const int m = m0 + (lane & 31), n = n0 + (lane & 31), h = lane >> 5;
  const bool m_ok = m < g.M, n_ok = n < g.N;
  const int64_t a_m = m_ok ? grouped(m, (int)g.a_pm, g.a_rm, g.a_sm) : 0;
  const float* af = static_cast<const float*>(g.a);
  const uint8_t* au = static_cast<const uint8_t*>(g.a);
  constexpr int U = 16;
  float av[2][U], bv[2][U];
  auto fetch = [&](int p0, int slot) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = 2 * (p0 + u) + h;
      const bool ok = p0 + u < p_end && k < g.K;
      float a = 0.0f, b = 0.0f;
      if (ok && m_ok) {
        if (g.a == nullptr) {
          a = 1.0f;
        } else {
          const int64_t off = a_m + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk);
          a = A_U8 ? (float)au[off] / 255.0f : af[off];
        }
      }
      if (ok && n_ok) b = g.b[(int64_t)k * g.b_ks + (int64_t)n * g.b_ns];
      av[slot][u] = a;
      bv[slot][u] = b;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  // two register stages (compile-time slots): the next 16 K-pairs are in flight while
  // the current ones feed the MFMAs
  if (p_begin < p_end) fetch(p_begin, 0);
  for (int p0 = p_begin; p0 < p_end; p0 += 2 * U) {
    if (p0 + U < p_end) fetch(p0 + U, 1);
#pragma unroll
    for (int u = 0; u < U; ++u) acc = mfma32(av[0][u], bv[0][u], acc);
    if (p0 + U >= p_end) break;
    if (p0 + 2 * U < p_end) fetch(p0 + 2 * U, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) acc = mfma32(av[1][u], bv[1][u], acc);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const int nn = n0 + (lane & 31);
    if (mm >= g.M || nn >= g.N) continue;
    if (gridDim.z > 1) {
      g.partials[((int64_t)blockIdx.z * g.M + mm) * g.N + nn] = acc[r];
    } else {
      store_c(epilogue(acc[r], nn, g), mm, nn, g);
    }
  }
}

// ---------------------------------------------------------------------------
// Streaming few-row forward (the dense layer over a big flattened input, M <= 64 rows:
// DQN's act / target forwards, 32 / 64 x 512 x 37632): HBM-bound on the weight, which every
// other path reads in short K pieces per 64-column tile. Here workgroup z owns one
// contiguous K range and ALL 512 columns of a column block, so the weight streams in
// whole 2-KB rows, once: lane l loads CW floats of row k + (l >> 5) (lanes 0..31 one
// 32 CW-column slice each wave, 512 columns per workgroup) and feeds them to CW MFMAs whose
// column i is the real column CW i + j (a column permutation the epilogue undoes with one
// 4 CW-byte partial store per row). A's slice sits in LDS (k-major, zero-padded), 16 k-pairs of
// the weight are in flight per lane, and nothing synchronises after the A fill. Partials
// [splits][M][N] go to the usual fixed-order split reduce (bias / activation / gate / beta).
// ---------------------------------------------------------------------------
constexpr int ST_U = 16;       // k-pairs in flight per lane (vmcnt allows 63)
constexpr int ST_NCOL = 512;   // columns per workgroup
constexpr int ST_MAX_LDS = 64 * 1024;
constexpr int kStRsrcWord3 = 0x00020000;  // raw buffer, gfx9-family resource word 3
constexpr int kStAuxNt = 2;               // buffer load aux bits: nontemporal (streamed once)
constexpr int ST_NCH = 6;                 // chunks per workgroup: K ranges <= 2 ST_NCH ST_U

// K per workgroup (a multiple of 4: 16-B A loads) and the LDS rows the loop reads (rounded
// up to its 2 ST_U-k chunk, zero past the range)
__host__ __device__ inline int stream_per(int K, int splits) {
  return ((K + splits - 1) / splits + 3) / 4 * 4;
}
__host__ __device__ inline int stream_rows(int per) {
  return (per + 2 * ST_U - 1) / (2 * ST_U) * (2 * ST_U);
}

template <int CW>
XA_DEV auto stream_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (CW == 4) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kStAuxNt);
  } else {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kStAuxNt));
  }
}

// CW columns per lane: CW = 2 -> 8 waves of 64 columns (8-B loads, the launched form: two
// waves per SIMD interleave their MFMA chains and LDS waits), CW = 4 -> 4 waves of 128
template <int MB, int CW>
__global__ __launch_bounds__(ST_NCOL / CW * 2) void gemm_stream_kernel(XaGemmArgs g) {
  constexpr int MR = 32 * MB, LDA = MR + 1, NTH = ST_NCOL / CW * 2, WCOL = 32 * CW;
  typedef float fv __attribute__((ext_vector_type(CW)));
  extern __shared__ float as[];  // [per][LDA]: A(m, kb + kk) at as[kk LDA + m]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int z = blockIdx.x, n_base = blockIdx.y * ST_NCOL;
  const int per = stream_per(g.K, (int)gridDim.x);
  const int kb = min(g.K, z * per), ke = min(g.K, kb + per);
  const float* a = static_cast<const float*>(g.a);
  const int np = (ke - kb) / 2;  // K ranges are multiples of 4 (K % 4 == 0 is checked)
  const int col = n_base + WCOL * w + CW * (lane & 31);
  f32x16 acc[MB][CW];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int j = 0; j < CW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][j][r] = 0.0f;
  // the weight through a raw buffer resource at this range's first row (lane offset + pair
  // stride in bytes; the host checks the range fits 2^31 bytes). The chunk loop is unrolled
  // whole (ST_NCH chunks, the host bounds the range): with no loop-carried registers the
  // compiler neither merges a prefetch into a load at its use nor waits for every load at
  // a loop head, and the scheduling barrier per pair keeps each prefetch where it is
  // issued, so ST_U pairs stay in flight and each MFMA waits for its own load only.
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(g.b + (int64_t)kb * g.b_ks), 0, 0x7FFFFFF0, kStRsrcWord3);
  const uint32_t lane_off = (uint32_t)(h * g.b_ks + col) * 4u;
  const uint32_t pbytes = (uint32_t)(2 * g.b_ks) * 4u;
  const int last = max(np - 1, 0), nch = (np + ST_U - 1) / ST_U;
  fv wv[ST_U];
  // the first ST_U pairs' loads go out before the A fill (their latency overlaps it)
  if (np > 0) {
#pragma unroll
    for (int u = 0; u < ST_U; ++u)
      wv[u] = stream_load<CW>(wr, lane_off + (uint32_t)min(u, last) * pbytes);
  }
  // A slice -> LDS (16-B loads along k, transposed scalar stores), zeros past ke / M
  const int q_per = stream_rows(per) / 4, total = MR * q_per;
  if (ke > kb) {
    // 8 loads in flight per thread (clamped in-range addresses, masked after the load)
    for (int i0 = 0; i0 < total; i0 += NTH * 8) {
      f32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = min(i0 + NTH * j + tid, total - 1);
        const int m = i / q_per, k = kb + 4 * (i - m * q_per);
        v[j] = *reinterpret_cast<const f32x4*>(a + (int64_t)min(m, g.M - 1) * g.a_rm +
                                               min(k, ke - 4));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + NTH * j + tid;
        if (i >= total) break;
        const int m = i / q_per, kq = i - m * q_per;
        const bool ok = m < g.M && kb + 4 * kq < ke;
#pragma unroll
        for (int e = 0; e < 4; ++e) as[(4 * kq + e) * LDA + m] = ok ? v[j][e] : 0.0f;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < ST_NCH; ++c) {
    if (c < nch) {  // uniform; pairs past np read zero A rows (a padded chunk adds 0)
#pragma unroll
      for (int u = 0; u < ST_U; ++u) {
        const int p = c * ST_U + u;
        const float* ar = as + (2 * p + h) * LDA + (lane & 31);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          const float av = ar[32 * mb];
#pragma unroll
          for (int j = 0; j < CW; ++j) acc[mb][j] = mfma32(av, wv[u][j], acc[mb][j]);
        }
        if (c + 1 < ST_NCH) wv[u] = stream_load<CW>(wr, lane_off + (uint32_t)min(p + ST_U, last) * pbytes);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // D(row (r&3) + 8 (r>>2) + 4 h, col i = l&31) of MFMA j is C(row, CW i + j)
  float* part = g.partials + (int64_t)z * g.M * g.N;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= g.M) continue;
      fv v;
#pragma unroll
      for (int j = 0; j < CW; ++j) v[j] = acc[mb][j][r];
      *reinterpret_cast<fv*>(part + (int64_t)m * g.N + col) = v;
    }
}

// the streaming path's contract: f32 A with plain 16-B aligned rows, n-major 16-B aligned
// B, M <= 64, N a multiple of 512, K % 4 == 0, a K split of >= 64 ranges whose padded A
// slice fits 64 KB of LDS (the caller's split count is the grid)
size_t stream_lds(const XaGemmArgs& g) {
  const int mr = g.M <= 32 ? 32 : 64;
  return sizeof(float) * (size_t)stream_rows(stream_per(g.K, g.splits)) * (mr + 1);
}

// XA_GEMM_STREAM=0 keeps these shapes on the tile kernels (A/B measurements)
bool stream_on() {
  static const bool on = [] {
    const char* e = std::getenv("XA_GEMM_STREAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool stream_ok(const XaGemmArgs& g) {
  return !g.force_small && !g.a_ones_row && g.a != nullptr && !g.a_u8 && g.a_pm == 1 &&
         g.a_pk == 1 && g.a_rk == 1 && g.a_rm % 4 == 0 && ((uintptr_t)g.a & 15) == 0 &&
         g.b_ns == 1 && g.b_ks % 4 == 0 && ((uintptr_t)g.b & 15) == 0 && g.M <= 64 &&
         g.N % ST_NCOL == 0 && g.K % 4 == 0 && g.splits >= 64 && g.partials &&
         ((uintptr_t)g.partials & 15) == 0 && stream_lds(g) <= ST_MAX_LDS &&
         stream_per(g.K, g.splits) <= 2 * ST_NCH * ST_U &&
         ((int64_t)stream_per(g.K, g.splits) + 2) * g.b_ks * 4 < (1ll << 31) && stream_on();
}

// column sums of B (A == NULL, M == 1: bias gradients): rows split over workgroups, each
// workgroup 4 waves x 64 columns, partial rows summed in fixed order by the split reduce
__global__ __launch_bounds__(256) void colsum_kernel(XaGemmArgs g) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.y * 64 + lane;
  const int rows_per = (g.K + (int)gridDim.z - 1) / (int)gridDim.z;
  const int r0 = blockIdx.z * rows_per, r1 = min(g.K, r0 + rows_per);
  __shared__ float red[4][64];
  float acc = 0.0f;
  if (n < g.N) {
    // 8 independent loads in flight per thread, summed in fixed order
    int k = r0 + w;
    for (; k + 28 < r1; k += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = g.b[(int64_t)(k + 4 * u) * g.b_ks + (int64_t)n * g.b_ns];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = acc + v[u];
    }
    for (; k < r1; k += 4) acc = acc + g.b[(int64_t)k * g.b_ks + (int64_t)n * g.b_ns];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && n < g.N) {
    const float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (gridDim.z > 1) g.partials[(int64_t)blockIdx.z * g.N + n] = v;
    else store_c(epilogue(v, n, g), 0, n, g);
  }
}

// fixed-order sum of the split partials + epilogue
__global__ __launch_bounds__(256) void gemm_split_reduce_kernel(XaGemmArgs g, int splits) {
  const int64_t total = (int64_t)g.M * g.N;
  const unsigned N = (unsigned)g.N;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    float s = 0.0f;
    for (int z = 0; z < splits; ++z) s = s + g.partials[(int64_t)z * total + e];
    // M * N < 2^31 is checked on the host
    const unsigned m = (unsigned)e / N, n = (unsigned)e - m * N;
    store_c(epilogue(s, (int)n, g), (int)m, (int)n, g);
  }
}

// fixed-order sum of many split partials over few outputs (bias / conv weight gradients:
// M N <= 64 K, splits in the hundreds or thousands): lane = output (one 256-B row segment
// per split), 16 waves cut the split range into contiguous pieces summed with 8 loads in
// flight, pieces combined in wave order through LDS
XA_DEV void split_reduce_wide(const XaGemmArgs& g, int splits, int bx) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int total = g.M * g.N;
  const int e = bx * 64 + lane;
  const int per = (splits + 15) / 16;
  const int z0 = w * per, z1 = min(splits, z0 + per);
  __shared__ float part[16][64];
  float acc = 0.0f;
  if (e < total) {
    const float* src = g.partials + e;
    int z = z0;
    for (; z + 8 <= z1; z += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(z + u) * total];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = acc + v[u];
    }
    for (; z < z1; ++z) acc = acc + src[(int64_t)z * total];
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w == 0 && e < total) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = s + part[i][lane];
    const int m = e / g.N, n = e - m * g.N;
    store_c(epilogue(s, n, g), m, n, g);
  }
}

__global__ __launch_bounds__(1024) void gemm_split_reduce_wide_kernel(XaGemmArgs g, int splits) {
  split_reduce_wide(g, splits, blockIdx.x);
}

// two split reduces in one launch (the conv weight and bias gradients): blocks [0, nb1) reduce
// g1, the rest g2 -- each output summed exactly as gemm_split_reduce_wide_kernel sums it
__global__ __launch_bounds__(1024) void gemm_split_reduce_wide2_kernel(XaGemmArgs g1,
                                                                       XaGemmArgs g2, int nb1,
                                                                       int splits) {
  if ((int)blockIdx.x < nb1) split_reduce_wide(g1, splits, blockIdx.x);
  else split_reduce_wide(g2, splits, blockIdx.x - nb1);
}

// ---------------------------------------------------------------------------
// Conv1D weight + bias gradient for a narrow im2col (k C <= 8, e.g. NatureCNN's first
// layer on single-channel frames): dW[t][c][f] = sum_{row, p} x[row][p s + t][c] dY[row][p][f]
// and db[f] = sum dY[row][p][f] in ONE pass over dY (the GEMM path reads dY twice, for dW
// and for the bias column sums, and wastes 3/4 of a 32 x 32 MFMA tile on M = 8).
// Block b owns a contiguous range of the rows x positions samples; thread = (filter quad,
// sample lane); fixed-order LDS combine -> per-block partials [G][kC F] and [G][F], summed
// in fixed order by the wide split reduce. Bound: reading dY (HBM).
// ---------------------------------------------------------------------------
constexpr int kWgMaxKC = 8;

struct XaWgradArgs {
  const void* x;
  const float* dy;
  float* ws;
  int rows, W, C, P, k, s, F, kc;
  int vec_x;  // kc % 4 == 0 and every im2col row start 4-element aligned
};

template <bool X_U8>
__global__ __launch_bounds__(256) void conv_wgrad_small_kernel(XaWgradArgs a) {
  const int FQ = a.F >> 2, nsub = 256 / FQ;
  const int q = threadIdx.x % FQ, sub = threadIdx.x / FQ;
  const int R = a.rows * a.P;
  const int per = (R + (int)gridDim.x - 1) / (int)gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(R, r0 + per);
  const float* xf = static_cast<const float*>(a.x);
  const uint8_t* xu = static_cast<const uint8_t*>(a.x);
  float acc[kWgMaxKC][4], bacc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bacc[c] = 0.0f;
#pragma unroll
    for (int j = 0; j < kWgMaxKC; ++j) acc[j][c] = 0.0f;
  }
  // U samples per trip, all their loads issued before the first use
  constexpr int U = 4;
  for (int rb = r0 + sub; rb < r1; rb += U * nsub) {
    f32x4 dz[U];
    float xv[U][kWgMaxKC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rb + u * nsub;
      const bool ok = r < r1;
      const int rr = ok ? r : r0;
      const unsigned row = (unsigned)rr / (unsigned)a.P;
      const int p = rr - (int)row * a.P;
      const int64_t xb = (int64_t)row * a.W * a.C + (int64_t)p * a.s * a.C;
      dz[u] = ok ? *reinterpret_cast<const f32x4*>(a.dy + (int64_t)rr * a.F + 4 * q)
                 : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (!ok) {
#pragma unroll
        for (int j = 0; j < kWgMaxKC; ++j) xv[u][j] = 0.0f;
      } else if (a.vec_x) {
#pragma unroll
        for (int j = 0; j < kWgMaxKC; j += 4) {
          if (j < a.kc) ld4<X_U8>(a.x, xb + j, &xv[u][j]);
          else zero4(&xv[u][j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kWgMaxKC; ++j)
          xv[u][j] = j < a.kc ? (X_U8 ? (float)xu[xb + j] / 255.0f : xf[xb + j]) : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bacc[c] = bacc[c] + dz[u][c];
#pragma unroll
        for (int j = 0; j < kWgMaxKC; ++j) acc[j][c] = fmaf(xv[u][j], dz[u][c], acc[j][c]);
      }
  }
  // combine the nsub sample lanes of every (quad, value) in fixed order
  constexpr int NV = 4 * (kWgMaxKC + 1);
  __shared__ float red[256 * NV];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    red[(sub * FQ + q) * NV + kWgMaxKC * 4 + c] = bacc[c];
#pragma unroll
    for (int j = 0; j < kWgMaxKC; ++j) red[(sub * FQ + q) * NV + j * 4 + c] = acc[j][c];
  }
  __syncthreads();
  const int nval = (a.kc + 1) * a.F;  // dW [kc][F] then db [F]
  const int G = gridDim.x;
  for (int v = threadIdx.x; v < nval; v += 256) {
    const int j = v / a.F, f = v - j * a.F;
    const int qq = f >> 2, c = f & 3;
    const int slot = (j < a.kc ? j : kWgMaxKC) * 4 + c;
    float sum = 0.0f;
    for (int u = 0; u < nsub; ++u) sum = sum + red[(u * FQ + qq) * NV + slot];
    if (j < a.kc) a.ws[(int64_t)blockIdx.x * a.kc * a.F + v] = sum;
    else a.ws[(int64_t)G * a.kc * a.F + (int64_t)blockIdx.x * a.F + f] = sum;
  }
}

constexpr int kWgBlocks = 1024;

// ---------------------------------------------------------------------------
// Keras Conv1D input gradient as one implicit GEMM (a transposed convolution), replacing
// the dY W^T GEMM into an im2col buffer + col2im gather. For phase phi = w mod s
// (blockIdx.z) and output position w = q s + phi:
//   dX[row][w][c] = sum_{j < J_phi} sum_f dY[row][q - j][f] W[phi + j s][c][f]
// with J_phi = ceil((k - phi) / s) taps and terms with q - j outside [0, P) zero, then
// times [gate[row][w][c] > 0]. GEMM view per phase: M = rows Q_phi (m = (row, q)),
// N = C, K = J_phi F (kk = (j, f), f fastest). Tiles as gemm_kernel (16 x 16 x 4 MFMA,
// waves of 32 x 32, K steps of 16 through double-buffered LDS); BNT = 64 channel tiles
// run 64 x 64 blocks, BNT = 32 runs 128 x 32 blocks. Needs F % 4 == 0 (a float4 of
// kk never crosses a tap).
// ---------------------------------------------------------------------------
struct XaDgradArgs {
  const float* dy;
  const float* w;
  const float* gate;
  float* out;
  int rows, P, k, s, C, F, W_in;
};

template <int BNT>
__global__ __launch_bounds__(256) void conv1d_dgrad_kernel(XaDgradArgs d) {
  constexpr int TBM = BNT == 64 ? 64 : 128;
  constexpr int LA = TBM + 4, LB = BNT + 4;
  constexpr int NAM = TBM / 64;  // A rows (m) per thread
  __shared__ __attribute__((aligned(16))) float As[2][BK * LA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = BNT == 64 ? w >> 1 : w, wn = BNT == 64 ? w & 1 : 0;
  const int phi = blockIdx.z;
  const int Q = (d.W_in - phi + d.s - 1) / d.s;
  const int J = phi < d.k ? (d.k - phi + d.s - 1) / d.s : 0;
  const int Mp = d.rows * Q, Kt = J * d.F;
  const int m0 = blockIdx.x * TBM, c0 = blockIdx.y * BNT;
  if (m0 >= Mp) return;

  // A slots: m_local = (tid >> 2) + 64 r, kk quad (tid & 3)
  const int aq = (tid & 3) * 4;
  int a_q[NAM];
  int64_t a_base[NAM];
  bool a_ok[NAM];
#pragma unroll
  for (int r = 0; r < NAM; ++r) {
    const int m = m0 + (tid >> 2) + 64 * r;
    a_ok[r] = m < Mp;
    const unsigned row = a_ok[r] ? (unsigned)m / (unsigned)Q : 0u;
    a_q[r] = a_ok[r] ? m - (int)row * Q : 0;
    a_base[r] = (int64_t)row * d.P * d.F;
  }
  // B slots: channel (tid >> 2), kk quad (tid & 3); threads past the tile stay idle
  const int bc = tid >> 2;
  const bool b_on = bc < BNT && c0 + bc < d.C;

  f32x4 ra[NAM], rb;
  auto load = [&](int kt) {
    const int kk = kt + aq;
    const int j = kk / d.F, f = kk - j * d.F;
#pragma unroll
    for (int r = 0; r < NAM; ++r) {
      const int p = a_q[r] - j;
      f32x4 v = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (a_ok[r] && kk < Kt && p >= 0 && p < d.P)
        v = *reinterpret_cast<const f32x4*>(d.dy + a_base[r] + (int64_t)p * d.F + f);
      ra[r] = v;
    }
    rb = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (b_on && kk < Kt) {
      const int t = phi + j * d.s;
      rb = *reinterpret_cast<const f32x4*>(d.w + ((int64_t)t * d.C + c0 + bc) * d.F + f);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int r = 0; r < NAM; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) As[buf][(aq + i) * LA + (tid >> 2) + 64 * r] = ra[r][i];
    if (bc < BNT)
#pragma unroll
      for (int i = 0; i < 4; ++i) Bs[buf][(aq + i) * LB + bc] = rb[i];
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if (Kt > 0) {
    load(0);
    stash(0);
    __syncthreads();
    int buf = 0;
    for (int kt = 0; kt < Kt; kt += BK) {
      const bool more = kt + BK < Kt;
      if (more) load(kt + BK);
      const float* as = As[buf];
      const float* bs = Bs[buf];
#pragma unroll
      for (int s4 = 0; s4 < BK / 4; ++s4) {
        const int kk = 4 * s4 + (lane >> 4);
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = as[kk * LA + wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = bs[kk * LB + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
      }
      if (more) stash(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
      if (m >= Mp) continue;
      const unsigned row = (unsigned)m / (unsigned)Q;
      const int q = m - (int)row * Q;
      const int64_t o = ((int64_t)row * d.W_in + (int64_t)q * d.s + phi) * d.C;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = c0 + wn * 32 + j * 16 + (lane & 15);
        if (c >= d.C) continue;
        float v = acc[i][j][r];
        if (d.gate && !(d.gate[o + c] > 0.0f)) v = 0.0f;
        d.out[o + c] = v;
      }
    }
}

template <bool AK, bool BNM, bool U8>
void launch(const XaGemmK& g, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm_kernel<AK, BNM, U8>), grid, dim3(256), 0, s, g);
}

template <int WM, int WN, bool AK, bool BNM, bool U8>
void launch_tile(const XaGemmK& g, int splits, hipStream_t s) {
  dim3 grid((g.g.M + 64 * WM - 1) / (64 * WM), (g.g.N + 64 * WN - 1) / (64 * WN), splits);
  hipLaunchKernelGGL((gemm_tile_kernel<WM, WN, AK, BNM, U8>), grid, dim3(256), 0, s, g);
}

template <int WM, int WN>
void dispatch_tile(const XaGemmK& g, bool ak, bool bn, bool u8, hipStream_t s) {
  if (u8) {
    if (ak && bn) launch_tile<WM, WN, true, true, true>(g, g.g.splits, s);
    else if (ak) launch_tile<WM, WN, true, false, true>(g, g.g.splits, s);
    else if (bn) launch_tile<WM, WN, false, true, true>(g, g.g.splits, s);
    else launch_tile<WM, WN, false, false, true>(g, g.g.splits, s);
  } else {
    if (ak && bn) launch_tile<WM, WN, true, true, false>(g, g.g.splits, s);
    else if (ak) launch_tile<WM, WN, true, false, false>(g, g.g.splits, s);
    else if (bn) launch_tile<WM, WN, false, true, false>(g, g.g.splits, s);
    else launch_tile<WM, WN, false, false, false>(g, g.g.splits, s);
  }
}

// kernel for a GEMM: 0 = 64 x 64 small-tile, 22 / 41 / 14 = tile kernel (WM, WN),
// 1 = skinny (one wave per 32 x 32 tile, long K), 2 = column sums (A = ones, M = 1).
// The tile kernel pays off only with >= 8 K steps of 32 per workgroup.
int pick_shape(int M, int N, int K, int k_split, bool ones) {
  if (ones && M == 1) return 2;
  // conv weight gradients (K = rows x positions): the 64 x 64 kernel with many K splits
  // (measured best: many small workgroups per CU hide the operand latency); below 64 rows
  // the one-wave 32 x 32 skinny tile wastes less of the MFMA
  if (N <= 64 && K >= 16384 && M < 64) return 1;
  if (k_split < 256) return 0;
  if (M >= 128 && N >= 128) return 22;
  if (N <= 64 && M >= 256) return 41;
  if (M <= 64 && N >= 256) return 14;
  return 0;
}

void tile_dims(int shape, int& bm, int& bn) {
  bm = bn = 64;
  if (shape == 1) bm = bn = 32;
  else if (shape == 2) bm = 1, bn = 64;
  else if (shape > 2) bm = 64 * (shape / 10), bn = 64 * (shape % 10);
}

template <int MT, int CH, bool GATE>
void launch_res1(const XaGemmArgs& g, int G, int rounds, hipStream_t s) {
  const size_t lds =
      sizeof(float) * ((size_t)MT * 16 * rs_pa<128 * CH>() + (size_t)RS_UPR * MT * (RS_KP - 1) * 256);
  hipLaunchKernelGGL((gemm_smallm_res_kernel<MT, CH, GATE>), dim3(G), dim3(512), lds, s, g, rounds);
}

template <int MT>
void launch_res(const XaGemmArgs& g, int ch, bool gate, int G, int rounds, hipStream_t s) {
  if (ch == 4) gate ? launch_res1<MT, 4, true>(g, G, rounds, s) : launch_res1<MT, 4, false>(g, G, rounds, s);
  else if (ch == 2) gate ? launch_res1<MT, 2, true>(g, G, rounds, s) : launch_res1<MT, 2, false>(g, G, rounds, s);
  else gate ? launch_res1<MT, 1, true>(g, G, rounds, s) : launch_res1<MT, 1, false>(g, G, rounds, s);
}

// the small-M kernel's contract: f32 A(m, k) = a[m lda + k], B(k, n) = b[n ldb + k], both
// 16-B aligned with lda, ldb multiples of 4, M <= 64, K in {128, 256, 512} (all of A in
// LDS), and enough 16-column units (N >= 2048) to cover the chip
bool smallm_res_ok(const XaGemmArgs& g) {
  return (!g.force_small || g.force_small >= 3) && !g.a_ones_row && g.a != nullptr && !g.a_u8 &&
         g.a_pm == 1 &&
         g.a_pk == 1 &&
         g.a_rk == 1 && g.a_rm % 4 == 0 && ((uintptr_t)g.a & 15) == 0 && g.b_ks == 1 &&
         g.b_ns % 4 == 0 && ((uintptr_t)g.b & 15) == 0 && g.M <= 64 &&
         (g.K == 128 || g.K == 256 || g.K == 512) && g.N >= 2048;
}

}  // namespace

extern "C" int xa_gemm_splits(int M, int N, int K) {
  // enough workgroups to cover the chip (>= 1024), each split >= 8 K tiles
  // without knowing A, assume a real A (the column-sum case is picked in xa_gemm)
  const int shape = pick_shape(M, N, K, K, false);
  int bm, bn;
  tile_dims(shape, bm, bn);
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int kt = (K + BK - 1) / BK;
  // skinny workgroups are one wave: 4096 of them keep 4 waves per SIMD streaming
  const int want = shape == 1 ? (M == 1 ? 512 : 4096) : 2048;
  // two or more full-K tiles per CU already fill the chip: a split only adds partial
  // traffic and, below 256 K per split, drops the 32x32-MFMA tile kernel (measured,
  // tools/gemm_split_sweep.py: dense dX 336 x 37632 x 512 167 us unsplit vs 212 us at the
  // former 4 splits; dense dW 37632 x 512 x 336 163 vs 180 us)
  if (shape != 1 && tiles >= 512) return 1;
  if (shape >= 14) {
    // few 32x32-MFMA tiles (the dense forward, K = 37632): split until the shape that is
    // actually launched (it drops to 64x64 below 256 K per split) covers ~1024 workgroups
    // (tools/gemm_split_sweep.py: 336 x 512 x 37632 187 us at 128 splits vs 227 us at 256;
    // 4096 x 512 x 37632 1209 us at 8 vs 1246 us at 16)
    // ... or, on the 128 x 128 kernel, 512 of its 4x-larger workgroups when the next
    // doubling would drop to the 64 x 64 kernel (128 x 512 x 37632, the double-DQN online
    // forward: 62.9 us at 128 splits vs 67.6 us at 256, profiles/r04an_split_sweep.txt)
    int s = 1;
    while (s < 4096 && kt / (s * 2) >= 8) {
      int tm, tn;
      const int sh = pick_shape(M, N, K, (K + s - 1) / s, false);
      tile_dims(sh, tm, tn);
      const int64_t wg = (int64_t)((M + tm - 1) / tm) * ((N + tn - 1) / tn) * s;
      if (wg >= 1024) break;
      if (sh == 22 && wg >= 512 && pick_shape(M, N, K, (K + 2 * s - 1) / (2 * s), false) == 0)
        break;
      s *= 2;
    }
    return s;
  }
  int s = 1;
  while (tiles * s < want && kt / (s * 2) >= 8 && s < 4096) s *= 2;
  return s;
}

extern "C" int xa_gemm_shape(int M, int N, int K, int splits) {
  if (splits < 1) splits = 1;
  return pick_shape(M, N, K, (K + splits - 1) / splits, false);
}

extern "C" size_t xa_gemm_workspace_floats(int M, int N, int K, int splits) {
  return splits > 1 ? (size_t)splits * M * N : 0;
}

// the kernel argument: the public args + the host's vectorisation verdicts (XaGemmK)
static XaGemmK kernel_args(const XaGemmArgs& g) {
  const bool ak = g.a_pk == 1 && g.a_rk == 1, bn = g.b_ns == 1, u8 = g.a_u8 != 0;
  XaGemmK kg{g, 0, 0, g.a_ones_row ? g.M - 1 : -1, XaAdamApply{}, 0};
  const int m_real = g.a_ones_row ? g.M - 1 : g.M;
  if (g.a != nullptr && ((uintptr_t)g.a & (u8 ? 3 : 15)) == 0) {
    const bool rows4 = g.a_rm % 4 == 0 && (g.a_pm == 1 || g.a_sm % 4 == 0);
    const bool cols4 = g.a_rk % 4 == 0 && (g.a_pk == 1 || g.a_sk % 4 == 0);
    kg.vec_a = ak ? (g.K % 4 == 0 && rows4)
                  : (g.a_pm == 1 && g.a_rm == 1 && m_real % 4 == 0 && cols4);
  }
  if (((uintptr_t)g.b & 15) == 0)
    kg.vec_b = bn ? (g.b_ks % 4 == 0 && g.N % 4 == 0)
                  : (g.b_ks == 1 && g.b_ns % 4 == 0 && g.K % 4 == 0);
  return kg;
}

extern "C" int xa_gemm_adam(const XaGemmArgs* p, const XaAdamApply* ad, void* stream) {
  XA_CHECK_ARG(p != nullptr && ad != nullptr, "xa_gemm_adam: null args");
  const XaGemmArgs& g = *p;
  XA_CHECK_ARG(g.M > 0 && g.N > 0 && g.K > 0 && g.a && g.b, "xa_gemm_adam: bad sizes or operands");
  XA_CHECK_ARG(g.a_pm > 0 && g.a_pk > 0 && (int64_t)g.M * g.N < (1ll << 31),
               "xa_gemm_adam: bad groups or M * N >= 2^31");
  const bool ak = g.a_pk == 1 && g.a_rk == 1, bn = g.b_ns == 1;
  XA_CHECK_ARG(g.splits == 1 && !g.bias && g.act == XA_ACT_NONE && !g.gate && !g.beta &&
                   !g.a_u8 && !ak && bn && g.N % 4 == 0 && g.ldc % 4 == 0 &&
                   pick_shape(g.M, g.N, g.K, g.K, false) == 0,
               "xa_gemm_adam: needs one K split, no bias / activation / gate / beta, f32 m-major "
               "A, n-major B, N and ldc multiples of 4 and the 64 x 64 kernel");
  XA_CHECK_ARG(ad->theta && ad->m && ad->v && ad->step &&
                   (((uintptr_t)ad->theta | (uintptr_t)ad->m | (uintptr_t)ad->v |
                     (uintptr_t)g.c) & 15) == 0,
               "xa_gemm_adam: theta / m / v / step missing or not 16-B aligned");
  XaGemmK kg = kernel_args(g);
  kg.ad = *ad;
  const int mt = (g.M + BM - 1) / BM, nt = (g.N + BN - 1) / BN;
  static const bool xmap = [] {
    const char* e = getenv("XA_GEMM_ADAM_XMAP");
    return !(e && e[0] == '0');
  }();
  dim3 grid(mt, nt, 1);
  if (xmap) {  // the XCD-aware 1-D tile order (gemm_kernel)
    kg.xmap_nt = nt;
    grid = dim3(8 * nt * ((mt + 7) / 8), 1, 1);
  }
  hipLaunchKernelGGL((gemm_kernel<false, true, false, true>), grid, dim3(256), 0,
                     (hipStream_t)stream, kg);
  XA_CHECK_LAUNCH("xa_gemm_adam");
  return 0;
}

static bool wide_reduce(const XaGemmArgs& g);
static void launch_main(const XaGemmArgs& g, hipStream_t s);

extern "C" int xa_gemm(const XaGemmArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_gemm: null args");
  const XaGemmArgs& g = *p;
  XA_CHECK_ARG(g.M > 0 && g.N > 0 && g.K > 0, "xa_gemm: M, N, K must be > 0 (got %d, %d, %d)",
               g.M, g.N, g.K);
  XA_CHECK_ARG(g.b && g.c, "xa_gemm: null B or C");
  XA_CHECK_ARG(g.a_pm > 0 && g.a_pk > 0, "xa_gemm: group sizes must be > 0");
  XA_CHECK_ARG(g.splits >= 1 && g.splits <= 4096, "xa_gemm: splits must be in [1, 4096]");
  XA_CHECK_ARG(g.splits == 1 || g.partials, "xa_gemm: splits > 1 needs partials");
  XA_CHECK_ARG(!g.gate || g.ld_gate > 0, "xa_gemm: gate needs ld_gate");
  XA_CHECK_ARG((int64_t)g.M * g.N < (1ll << 31) && g.a_pm < (1ll << 31) && g.a_pk < (1ll << 31),
               "xa_gemm: M * N and group sizes must stay below 2^31");
  hipStream_t s = (hipStream_t)stream;
  if (smallm_res_ok(g)) {
    const int units = (g.N + 15) / 16;
    int cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    const int G = std::min(cus, (units + RS_UPR - 1) / RS_UPR);
    int rounds = (units + RS_UPR * G - 1) / (RS_UPR * G);
    rounds = (rounds + RS_NR - 1) / RS_NR * RS_NR;  // the round loop is unrolled by RS_NR
    const int mt = (g.M + 15) / 16, ch = g.K / 128;
    const bool gate = g.gate != nullptr;
    if (mt <= 1) launch_res<1>(g, ch, gate, G, rounds, s);
    else if (mt <= 2) launch_res<2>(g, ch, gate, G, rounds, s);
    else launch_res<4>(g, ch, gate, G, rounds, s);
    XA_CHECK_LAUNCH("xa_gemm (small M, resident A)");
    return 0;
  }
  if (smallk_ok(g)) {
    const int64_t total = (int64_t)g.M * g.N;
    hipLaunchKernelGGL(gemm_smallk_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, g);
    XA_CHECK_LAUNCH("xa_gemm (few k)");
    return 0;
  }
  if (rowdot_ok(g)) {
    hipLaunchKernelGGL(gemm_rowdot_kernel, dim3((g.M + 3) / 4), dim3(256), 0, s, g);
    XA_CHECK_LAUNCH("xa_gemm (row dot)");
    return 0;
  }
  XA_CHECK_ARG(!g.a_ones_row || ((g.force_small == 1 ||
                                   pick_shape(g.M, g.N, g.K, (g.K + g.splits - 1) / g.splits,
                                              g.a == nullptr) == 0) &&
                                  g.a != nullptr && g.M >= 2),
               "xa_gemm: a_ones_row needs the 64 x 64 kernel (xa_gemm_shape == 0), A and M >= 2");
  launch_main(g, s);
  XA_CHECK_LAUNCH("xa_gemm");
  if (g.splits > 1) {
    const int64_t total = (int64_t)g.M * g.N;
    if (wide_reduce(g)) {
      hipLaunchKernelGGL(gemm_split_reduce_wide_kernel, dim3((int)((total + 63) / 64)),
                         dim3(1024), 0, s, g, g.splits);
    } else {
      const int64_t want = (total + 255) / 256;
      const int blocks = (int)(want < 4096 ? want : 4096);
      hipLaunchKernelGGL(gemm_split_reduce_kernel, dim3(blocks), dim3(256), 0, s, g, g.splits);
    }
    XA_CHECK_LAUNCH("xa_gemm (split reduce)");
  }
  return 0;
}

// the split-reduce form xa_gemm takes: lane-per-output over 16 contiguous split pieces
static bool wide_reduce(const XaGemmArgs& g) {
  return (int64_t)g.M * g.N <= 65536 && g.splits >= 64;
}

// the main GEMM launch of xa_gemm's tile / stream / skinny / colsum paths (the split partials
// when g.splits > 1)
static void launch_main(const XaGemmArgs& g, hipStream_t s) {
  dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN, g.splits);
  const bool use_stream = stream_ok(g);
  const bool ak = g.a_pk == 1 && g.a_rk == 1;
  const bool bn = g.b_ns == 1;
  const bool u8 = g.a_u8 != 0;
  const int per_split = (g.K + g.splits - 1) / g.splits;
  const int shape = g.force_small == 1 ? 0 : pick_shape(g.M, g.N, g.K, per_split, g.a == nullptr);
  const XaGemmK kg = kernel_args(g);
  if (use_stream) {
    const dim3 gs(g.splits, g.N / ST_NCOL);
    // 8 waves of 64 columns (8-B loads): 20.5 / 32.9 us at M = 32 / 64 against 21.0 / 34.2
    // for 4 waves of 128 columns (16-B loads), profiles/r05zs_stream_cw_ab.txt
    if (g.M <= 32)
      hipLaunchKernelGGL((gemm_stream_kernel<1, 2>), gs, dim3(512), stream_lds(g), s, g);
    else
      hipLaunchKernelGGL((gemm_stream_kernel<2, 2>), gs, dim3(512), stream_lds(g), s, g);
  } else if (shape == 2) {
    hipLaunchKernelGGL(colsum_kernel, dim3(1, (g.N + 63) / 64, g.splits), dim3(256), 0, s, g);
  } else if (shape == 1) {
    dim3 gs((g.M + 31) / 32, (g.N + 31) / 32, g.splits);
    if (u8) hipLaunchKernelGGL(gemm_skinny_kernel<true>, gs, dim3(64), 0, s, g);
    else hipLaunchKernelGGL(gemm_skinny_kernel<false>, gs, dim3(64), 0, s, g);
  } else if (shape == 22) dispatch_tile<2, 2>(kg, ak, bn, u8, s);
  else if (shape == 41) dispatch_tile<4, 1>(kg, ak, bn, u8, s);
  else if (shape == 14) dispatch_tile<1, 4>(kg, ak, bn, u8, s);
  else if (u8) {
    if (ak && bn) launch<true, true, true>(kg, grid, s);
    else if (ak) launch<true, false, true>(kg, grid, s);
    else if (bn) launch<false, true, true>(kg, grid, s);
    else launch<false, false, true>(kg, grid, s);
  } else {
    if (ak && bn) launch<true, true, false>(kg, grid, s);
    else if (ak) launch<true, false, false>(kg, grid, s);
    else if (bn) launch<false, true, false>(kg, grid, s);
    else launch<false, false, false>(kg, grid, s);
  }
}


extern "C" int xa_dqn_head(const XaGemmArgs* p, const XaDqnHeadArgs* d, void* stream) {
  XA_CHECK_ARG(p != nullptr && d != nullptr, "xa_dqn_head: null args");
  const XaGemmArgs& g = *p;
  XA_CHECK_ARG(g.M > 0 && g.N > 0 && g.K > 0 && g.b && g.c && rowdot_ok(g) && !g.gate && !g.beta,
               "xa_dqn_head: needs the row-dot head shape (f32 plain rows, N <= %d, K <= 4096, "
               "no gate / beta)", RD_MAXN);
  XA_CHECK_ARG(d->mode == 0 ? d->actions != nullptr
                            : (d->mode == 1 && d->q && d->act && d->rewards && d->dones && d->dq),
               "xa_dqn_head: mode 0 needs actions, mode 1 q / act / rewards / dones / dq");
  hipLaunchKernelGGL(dqn_head_kernel, dim3((g.M + 3) / 4), dim3(256), 0, (hipStream_t)stream, g, *d);
  XA_CHECK_LAUNCH("xa_dqn_head");
  return 0;
}

extern "C" int xa_gemm_head(const XaGemmArgs* dp, const XaGemmArgs* hp, const XaDqnHeadArgs* q,
                            void* stream) {
  XA_CHECK_ARG(dp != nullptr && hp != nullptr, "xa_gemm_head: null args");
  const XaGemmArgs& d = *dp;
  const XaGemmArgs& h = *hp;
  XA_CHECK_ARG(xa_gemm_head_ok(dp, hp) == 1,
               "xa_gemm_head: needs a split-K dense layer on the wide reduce (M N <= 65536, >= 64 "
               "splits, N <= %d, no gate / beta) and a row-dot head on its output rows (M equal, "
               "K = the dense N, A = the dense C, no gate / beta)", 64 * DH_NCH);
  XA_CHECK_ARG(q == nullptr || (q->mode == 0 ? q->actions != nullptr
                                             : (q->mode == 1 && q->q && q->act && q->rewards &&
                                                q->dones && q->dq)),
               "xa_gemm_head: mode 0 needs actions, mode 1 q / act / rewards / dones / dq");
  hipStream_t s = (hipStream_t)stream;
  launch_main(d, s);
  XA_CHECK_LAUNCH("xa_gemm_head (split partials)");
  XaDqnHeadArgs qq{};
  if (q) qq = *q;
  hipLaunchKernelGGL(dense_head_kernel, dim3(d.M), dim3(1024), 0, s, d, d.splits, h, qq,
                     q ? q->mode : -1);
  XA_CHECK_LAUNCH("xa_gemm_head (reduce + head)");
  return 0;
}

extern "C" int xa_gemm_head_ok(const XaGemmArgs* dp, const XaGemmArgs* hp) {
  if (!dp || !hp) return 0;
  const XaGemmArgs& d = *dp;
  const XaGemmArgs& h = *hp;
  const bool dense = d.M > 0 && d.N > 0 && d.K > 0 && d.b && d.c && d.a_pm > 0 && d.a_pk > 0 &&
                     d.splits > 1 && d.splits <= 4096 && d.partials && wide_reduce(d) &&
                     d.N <= 64 * DH_NCH && !d.gate && !d.beta && !d.a_ones_row &&
                     !smallm_res_ok(d) && !smallk_ok(d) && !rowdot_ok(d);
  const bool head = h.M == d.M && h.K == d.N && h.b && h.c && rowdot_ok(h) && !h.gate &&
                    !h.beta && h.a == (const void*)d.c && h.a_rm == d.ldc;
  return dense && head ? 1 : 0;
}

extern "C" int xa_head_bwd(const float* x, const float* dz, const float* W, const float* gate,
                           int M, int K, int A, float* dx, int beta, float* gw, float* gb,
                           int accumulate, void* stream) {
  XA_CHECK_ARG(x && dz && W && dx && M > 0 && K > 0 && A > 0 && A <= SK_MAXK_H && K <= 4096 &&
                   (int64_t)M * K < (1ll << 31),
               "xa_head_bwd: bad operands or sizes (A <= %d, K <= 4096)", SK_MAXK_H);
  HeadBwd h{x, dz, W, gate, M, K, A, dx, beta, gw, gb, accumulate, 0};
  h.nbx = (int)(((int64_t)M * K + 255) / 256);
  const int nbw = ((K + 1) * A + 255) / 256;
  hipLaunchKernelGGL(head_bwd_kernel, dim3(h.nbx + nbw), dim3(256), 0, (hipStream_t)stream, h);
  XA_CHECK_LAUNCH("xa_head_bwd");
  return 0;
}

extern "C" int xa_conv1d_dgrad(const float* dy, const float* kernel, int rows, int positions,
                               int ksize, int stride, int channels, int filters, int width_in,
                               const float* gate, float* dinput, void* stream) {
  XA_CHECK_ARG(dy && kernel && dinput && rows > 0 && positions > 0 && ksize > 0 && stride > 0 &&
                   channels > 0 && filters > 0 &&
                   width_in >= (positions - 1) * stride + ksize,
               "xa_conv1d_dgrad: bad arguments");
  XA_CHECK_ARG(filters % 4 == 0, "xa_conv1d_dgrad: filters must be a multiple of 4 (got %d)",
               filters);
  XA_CHECK_ARG(((uintptr_t)dy & 15) == 0 && ((uintptr_t)kernel & 15) == 0,
               "xa_conv1d_dgrad: dY and the kernel must be 16-byte aligned");
  XA_CHECK_ARG((int64_t)rows * width_in < (1ll << 31) &&
                   (int64_t)rows * width_in * channels < (1ll << 40),
               "xa_conv1d_dgrad: rows * width_in must stay below 2^31");
  XaDgradArgs d{dy, kernel, gate, dinput, rows, positions, ksize, stride, channels, filters,
                width_in};
  const int q0 = (width_in + stride - 1) / stride;  // phase 0 has the most positions
  const int64_t m0 = (int64_t)rows * q0;
  const int nph = stride < width_in ? stride : width_in;
  hipStream_t s = (hipStream_t)stream;
  if (channels <= 32) {
    dim3 grid((unsigned)((m0 + 127) / 128), 1, nph);
    hipLaunchKernelGGL(conv1d_dgrad_kernel<32>, grid, dim3(256), 0, s, d);
  } else {
    dim3 grid((unsigned)((m0 + 63) / 64), (channels + 63) / 64, nph);
    hipLaunchKernelGGL(conv1d_dgrad_kernel<64>, grid, dim3(256), 0, s, d);
  }
  XA_CHECK_LAUNCH("xa_conv1d_dgrad");
  return 0;
}

extern "C" size_t xa_conv1d_wgrad_workspace_floats(int ksize, int channels, int filters) {
  const int kc = ksize * channels;
  const bool ok = kc >= 1 && kc <= kWgMaxKC && filters >= 4 && filters <= 64 &&
                  (filters & (filters - 1)) == 0;
  return ok ? (size_t)kWgBlocks * (kc + 1) * filters : 0;
}

extern "C" int xa_conv1d_wgrad(const void* x, int x_u8, const float* dy, int rows, int width_in,
                               int channels, int positions, int ksize, int stride, int filters,
                               float* dw, float* db, int accumulate, float* workspace,
                               size_t workspace_floats, void* stream) {
  const size_t need = xa_conv1d_wgrad_workspace_floats(ksize, channels, filters);
  XA_CHECK_ARG(need > 0, "xa_conv1d_wgrad: needs ksize * channels <= 8 and filters a power of "
                         "two in [4, 64] (got k %d, C %d, F %d)", ksize, channels, filters);
  XA_CHECK_ARG(x && dy && dw && db && workspace && workspace_floats >= need,
               "xa_conv1d_wgrad: null pointer or workspace below %zu floats", need);
  XA_CHECK_ARG(rows > 0 && positions > 0 && stride > 0 &&
                   width_in >= (positions - 1) * stride + ksize &&
                   (int64_t)rows * positions < (1ll << 31) && ((uintptr_t)dy & 15) == 0,
               "xa_conv1d_wgrad: bad sizes or unaligned dY");
  hipStream_t s = (hipStream_t)stream;
  const int kc = ksize * channels;
  const int align = x_u8 ? 3 : 15;
  const int vec_x = kc % 4 == 0 && (width_in * channels) % 4 == 0 &&
                    (stride * channels) % 4 == 0 && ((uintptr_t)x & align) == 0;
  XaWgradArgs a{x, dy, workspace, rows, width_in, channels, positions, ksize, stride, filters, kc,
                vec_x};
  if (x_u8) hipLaunchKernelGGL(conv_wgrad_small_kernel<true>, dim3(kWgBlocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv_wgrad_small_kernel<false>, dim3(kWgBlocks), dim3(256), 0, s, a);
  XA_CHECK_LAUNCH("xa_conv1d_wgrad");
  // fixed-order sums over the blocks: dW [kc][F], then db [F]
  XaGemmArgs r{};
  r.M = kc;
  r.N = filters;
  r.K = 1;
  r.c = dw;
  r.ldc = filters;
  r.partials = workspace;
  r.beta = accumulate;
  r.act = XA_ACT_NONE;
  XaGemmArgs rb = r;
  rb.M = 1;
  rb.c = db;
  rb.partials = workspace + (size_t)kWgBlocks * kc * filters;
  const int nbw = (kc * filters + 63) / 64, nbb = (filters + 63) / 64;
  hipLaunchKernelGGL(gemm_split_reduce_wide2_kernel, dim3(nbw + nbb), dim3(1024), 0, s, r, rb, nbw,
                     kWgBlocks);
  XA_CHECK_LAUNCH("xa_conv1d_wgrad (reduce)");
  return 0;
}
