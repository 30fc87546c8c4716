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
#include "../../include/xagents_hip.h"
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

// A_KMAJOR: g(k) is unit stride (loader reads along k); otherwise along m.
// B_NMAJOR: b_ns == 1 (loader reads along n); otherwise along k.
template <bool A_KMAJOR, bool B_NMAJOR, bool A_U8>
__global__ __launch_bounds__(256) void gemm_kernel(XaGemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int tiles_k = (g.K + BK - 1) / BK;
  const int per = (tiles_k + (int)gridDim.z - 1) / (int)gridDim.z;
  const int k_begin = blockIdx.z * per * BK;
  const int k_end = min(g.K, k_begin + per * BK);

  // this thread's load slots (4 A elements, 4 B elements per K tile)
  const int a_m = A_KMAJOR ? tid >> 2 : (tid & 15) * 4;
  const int a_k = A_KMAJOR ? (tid & 3) * 4 : tid >> 4;
  const int b_k = B_NMAJOR ? tid >> 4 : (tid & 3) * 4;
  const int b_n = B_NMAJOR ? (tid & 15) * 4 : tid >> 2;
  int64_t a_row[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + a_m + (A_KMAJOR ? 0 : i);
    a_ok[i] = m < g.M;
    a_row[i] = a_ok[i] ? grouped(m, (int)g.a_pm, g.a_rm, g.a_sm) : 0;
  }
  const float* af = static_cast<const float*>(g.a);
  const uint8_t* au = static_cast<const uint8_t*>(g.a);

  float ra[4], rb[4];
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kt + a_k + (A_KMAJOR ? i : 0);
      const int ai = A_KMAJOR ? 0 : i;
      float v = 0.0f;
      if (a_ok[ai] && k < k_end) {
        if (g.a == nullptr) {
          v = 1.0f;
        } else {
          const int64_t off = a_row[ai] + grouped(k, (int)g.a_pk, g.a_rk, g.a_sk);
          v = A_U8 ? (float)au[off] / 255.0f : af[off];
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kt + b_k + (B_NMAJOR ? 0 : i);
      const int n = n0 + b_n + (B_NMAJOR ? i : 0);
      rb[i] = (k < k_end && n < g.N) ? g.b[(int64_t)k * g.b_ks + (int64_t)n * g.b_ns] : 0.0f;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      As[buf][(a_k + (A_KMAJOR ? i : 0)) * LDA + a_m + (A_KMAJOR ? 0 : i)] = ra[i];
      Bs[buf][(b_k + (B_NMAJOR ? 0 : i)) * LDB + b_n + (B_NMAJOR ? i : 0)] = rb[i];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if (k_begin < k_end) {
    load(k_begin);
    stash(0);
    __syncthreads();
    int buf = 0;
    for (int kt = k_begin; kt < k_end; kt += BK) {
      const bool more = kt + BK < k_end;
      if (more) load(kt + BK);
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

template <bool AK, bool BNM, bool U8>
void launch(const XaGemmArgs& g, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm_kernel<AK, BNM, U8>), grid, dim3(256), 0, s, g);
}

}  // namespace

extern "C" int xa_gemm_splits(int M, int N, int K) {
  // enough workgroups to cover the chip (>= 1024), each split >= 8 K tiles
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int kt = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < 1024 && kt / (s * 2) >= 8 && s < 4096) s *= 2;
  return s;
}

extern "C" size_t xa_gemm_workspace_floats(int M, int N, int K, int splits) {
  return splits > 1 ? (size_t)splits * M * N : 0;
}

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
  dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN, g.splits);
  const bool ak = g.a_pk == 1 && g.a_rk == 1;
  const bool bn = g.b_ns == 1;
  const bool u8 = g.a_u8 != 0;
  if (u8) {
    if (ak && bn) launch<true, true, true>(g, grid, s);
    else if (ak) launch<true, false, true>(g, grid, s);
    else if (bn) launch<false, true, true>(g, grid, s);
    else launch<false, false, true>(g, grid, s);
  } else {
    if (ak && bn) launch<true, true, false>(g, grid, s);
    else if (ak) launch<true, false, false>(g, grid, s);
    else if (bn) launch<false, true, false>(g, grid, s);
    else launch<false, false, false>(g, grid, s);
  }
  XA_CHECK_LAUNCH("xa_gemm");
  if (g.splits > 1) {
    const int64_t total = (int64_t)g.M * g.N;
    const int64_t want = (total + 255) / 256;
    const int blocks = (int)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(gemm_split_reduce_kernel, dim3(blocks), dim3(256), 0, s, g, g.splits);
    XA_CHECK_LAUNCH("xa_gemm (split reduce)");
  }
  return 0;
}
