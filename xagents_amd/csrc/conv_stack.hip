// Fused forward of the reference's NatureCNN convolution stack (xagents/*/models/cnn*.cfg:
// Conv1D 32 x 8 / 4, 64 x 4 / 2, 64 x 3 / 1, ReLU each, built by
// xagents/utils/common.py:225-240 over (84, 84, 1) frames). Keras' Conv1D on a 4-D input
// convolves along the width of each of the 84 frame rows independently, so a "sequence" is
// one 84-pixel row: 84 -> [20][32] -> [9][64] -> [7][64] (the 448 floats of the row's
// share of the flattened 37632-float feature vector).
//
// The per-layer path (three xa_gemm launches) writes every activation to HBM and reads it
// back as the next layer's im2col operand, at 1.4-2 TB/s (profiles/r05s_profc3_timeline.txt:
// 19.7 / 25.4 / 27.8 us for a 128-frame batch). Here one workgroup per CU walks groups of
// CR = 16 sequences; a group's three layers run out of LDS:
//   x [16][84] -> h1 [320][32] -> h2 [144][64] -> h3 [112][64] -> HBM
// with v_mfma_f32_16x16x4f32. Wave w owns output columns 16 w .. 16 w + 15 of conv2 and
// conv3 and keeps those columns' weights in registers for the whole launch (conv2: 128 x 16,
// conv3: 192 x 16, i.e. 32 + 48 floats per lane), so only A comes from LDS: within each
// 16-deep K block lane group q = l / 16 takes k = 16 kb + 4 q + j in MFMA j, which makes a
// lane's 4 A values one contiguous 16-B LDS read (the im2col window of a Conv1D row is
// contiguous in k: k = tap * C + channel over positions stride * p + tap). The M extents
// 320 / 144 / 112 of a 16-sequence group are all multiples of 16 (no padded tiles).
// h1 / h2 also go to HBM when the caller keeps them (the backward's ReLU gates and weight-
// gradient operands); h3 always does. Sum order per output: k ascending in 16-blocks, lane
// groups' partial products combined by the MFMA -- the same f32 dot products as the GEMM
// path up to association (tests compare against f64 at the executor's tolerance).
#include <hip/hip_runtime.h>

#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

XA_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int CW0 = 84, CK1 = 8, CS1 = 4, CF1 = 32, CP1 = 20;
constexpr int CK2 = 4, CS2 = 2, CF2 = 64, CP2 = 9;
constexpr int CK3 = 3, CS3 = 1, CF3 = 64, CP3 = 7;
constexpr int CR = 16;                                  // sequences per group
constexpr int M1 = CR * CP1, M2 = CR * CP2, M3 = CR * CP3;  // 320, 144, 112
constexpr int LD1 = CF1 + 4, LD2 = CF2 + 4;             // LDS row pitches (16-B aligned rows)
constexpr int XQ = CR * CW0 / 4;                        // 4-value items of a group's input
static_assert(CP1 == (CW0 - CK1) / CS1 + 1 && CP2 == (CP1 - CK2) / CS2 + 1 &&
                  CP3 == (CP2 - CK3) / CS3 + 1, "NatureCNN Conv1D geometry");
static_assert(M1 % 16 == 0 && M2 % 16 == 0 && M3 % 16 == 0, "whole 16-row tiles");
static_assert(CK1 * 1 == 8 && CF1 == 32 && CF2 == 64 && CF3 == 64, "tile mapping below");

// the 4 input values of item i (row i / 21, pixels 4 (i % 21) ..) of the group at row0;
// rows past the batch read as 0
XA_DEV f32x4 load_x4(const XaConvStackArgs& p, int row0, int i) {
  const int r = i / (CW0 / 4), c = i - r * (CW0 / 4);
  f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
  if (row0 + r < p.rows) {
    const int64_t off = (int64_t)(row0 + r) * CW0 + 4 * c;
    if (p.x_u8) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(p.x) + off);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (float)((u >> (8 * e)) & 0xFFu) / 255.0f;
    } else {
      v = *reinterpret_cast<const f32x4*>(static_cast<const float*>(p.x) + off);
    }
  }
  return v;
}

XA_DEV void store_x4(float* xs, int i, f32x4 v) {
  *reinterpret_cast<f32x4*>(xs + 4 * i) = v;  // item i covers xs[4 i .. 4 i + 3]
}

__global__ __launch_bounds__(256) void conv_stack_fwd_kernel(XaConvStackArgs p) {
  __shared__ __attribute__((aligned(16))) float xs[CR * CW0];
  __shared__ __attribute__((aligned(16))) float h1s[M1 * LD1];
  __shared__ __attribute__((aligned(16))) float h2s[M2 * LD2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, i16 = lane & 15;

  // this wave's weights: conv2 / conv3 columns 16 w + i16, k = 16 kb + 4 q + j
  const int n2 = 16 * w + i16;
  float wr2[CK2 * CF1 / 16][4], wr3[CK3 * CF2 / 16][4];
#pragma unroll
  for (int kb = 0; kb < CK2 * CF1 / 16; ++kb)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr2[kb][j] = p.w2[(16 * kb + 4 * q + j) * CF2 + n2];
#pragma unroll
  for (int kb = 0; kb < CK3 * CF2 / 16; ++kb)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr3[kb][j] = p.w3[(16 * kb + 4 * q + j) * CF3 + n2];
  const float bias2 = p.b2[n2], bias3 = p.b3[n2];
  // conv1 (K = 8, 32 columns): column tile w & 1, M tiles of parity w >> 1; MFMA j takes
  // k = 4 j + q
  const int n1 = 16 * (w & 1) + i16;
  const float w1a = p.w1[q * CF1 + n1], w1b = p.w1[(4 + q) * CF1 + n1], bias1 = p.b1[n1];

  const int G = (p.rows + CR - 1) / CR;
  if ((int)blockIdx.x >= G) return;
  for (int i = tid; i < XQ; i += 256) store_x4(xs, i, load_x4(p, (int)blockIdx.x * CR, i));
  __syncthreads();

  for (int gi = blockIdx.x; gi < G; gi += gridDim.x) {
    const int row0 = gi * CR;
    // ---- conv1: x -> h1 (bias + ReLU) ----
    for (int mt = w >> 1; mt < M1 / 16; mt += 2) {
      const int m = 16 * mt + i16, r = m / CP1, pp = m - r * CP1;
      const float* xr = xs + r * CW0 + CS1 * pp + q;
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      acc = mfma4(xr[0], w1a, acc);
      acc = mfma4(xr[4], w1b, acc);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int mo = 16 * mt + 4 * q + e;
        const float v = fmaxf(acc[e] + bias1, 0.0f);
        h1s[mo * LD1 + n1] = v;
        if (p.h1 && row0 + mo / CP1 < p.rows) p.h1[((int64_t)row0 * CP1 + mo) * CF1 + n1] = v;
      }
    }
    __syncthreads();  // h1s complete; xs free
    // the next group's input, in flight during conv2
    const int gn = gi + (int)gridDim.x;
    f32x4 xn[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u;
      xn[u] = (gn < G && i < XQ) ? load_x4(p, gn * CR, i) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    // ---- conv2: h1 -> h2, two M tiles per pass (independent accumulators) ----
    for (int mt = 0; mt < M2 / 16; mt += 2) {
      const bool two = mt + 1 < M2 / 16;
      int base[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int m = 16 * min(mt + s, M2 / 16 - 1) + i16, r = m / CP2, pp = m - r * CP2;
        base[s] = (r * CP1 + CS2 * pp) * LD1 + 4 * q;
      }
      f32x4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
      // k = 16 kb + 4 q + j: tap kb / 2, channel 16 (kb % 2) + 4 q + j; the next block's A
      // reads are issued before this block's MFMAs (pinning them there with scheduling
      // barriers measured slower: 46.2 vs 42.4 us, profiles/r05y)
      auto off2 = [](int kb) { return (kb >> 1) * LD1 + (kb & 1) * 16; };
      f32x4 nx0 = *reinterpret_cast<const f32x4*>(h1s + base[0] + off2(0));
      f32x4 nx1 = *reinterpret_cast<const f32x4*>(h1s + base[1] + off2(0));
#pragma unroll
      for (int kb = 0; kb < CK2 * CF1 / 16; ++kb) {
        const f32x4 a0 = nx0, a1 = nx1;
        if (kb + 1 < CK2 * CF1 / 16) {
          nx0 = *reinterpret_cast<const f32x4*>(h1s + base[0] + off2(kb + 1));
          nx1 = *reinterpret_cast<const f32x4*>(h1s + base[1] + off2(kb + 1));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[0] = mfma4(a0[j], wr2[kb][j], acc[0]);
          acc[1] = mfma4(a1[j], wr2[kb][j], acc[1]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 1 && !two) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int mo = 16 * (mt + s) + 4 * q + e;
          const float v = fmaxf(acc[s][e] + bias2, 0.0f);
          h2s[mo * LD2 + n2] = v;
          if (p.h2 && row0 + mo / CP2 < p.rows) p.h2[((int64_t)row0 * CP2 + mo) * CF2 + n2] = v;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u;
      if (gn < G && i < XQ) store_x4(xs, i, xn[u]);
    }
    __syncthreads();  // h2s complete; the next group's xs staged
    // ---- conv3: h2 -> h3 (HBM) ----
    for (int mt = 0; mt < M3 / 16; mt += 2) {
      const bool two = mt + 1 < M3 / 16;
      int base[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int m = 16 * min(mt + s, M3 / 16 - 1) + i16, r = m / CP3, pp = m - r * CP3;
        base[s] = (r * CP2 + CS3 * pp) * LD2 + 4 * q;
      }
      f32x4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
      // tap kb / 4, channel 16 (kb % 4) + 4 q + j; reads one block ahead as in conv2
      auto off3 = [](int kb) { return (kb >> 2) * LD2 + (kb & 3) * 16; };
      f32x4 nx0 = *reinterpret_cast<const f32x4*>(h2s + base[0] + off3(0));
      f32x4 nx1 = *reinterpret_cast<const f32x4*>(h2s + base[1] + off3(0));
#pragma unroll
      for (int kb = 0; kb < CK3 * CF2 / 16; ++kb) {
        const f32x4 a0 = nx0, a1 = nx1;
        if (kb + 1 < CK3 * CF2 / 16) {
          nx0 = *reinterpret_cast<const f32x4*>(h2s + base[0] + off3(kb + 1));
          nx1 = *reinterpret_cast<const f32x4*>(h2s + base[1] + off3(kb + 1));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[0] = mfma4(a0[j], wr3[kb][j], acc[0]);
          acc[1] = mfma4(a1[j], wr3[kb][j], acc[1]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 1 && !two) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int mo = 16 * (mt + s) + 4 * q + e;
          if (row0 + mo / CP3 < p.rows)
            p.h3[((int64_t)row0 * CP3 + mo) * CF3 + n2] = fmaxf(acc[s][e] + bias3, 0.0f);
        }
      }
    }
    // no barrier here: the next conv1 writes only h1s (conv3 reads h2s), and the next
    // conv2 writes h2s after the next post-conv1 barrier
  }
}

int cu_count() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

}  // namespace

extern "C" int xa_conv_stack_fwd(const XaConvStackArgs* a, void* stream) {
  XA_CHECK_ARG(a != nullptr, "xa_conv_stack_fwd: null args");
  const XaConvStackArgs& p = *a;
  XA_CHECK_ARG(p.x && p.w1 && p.b1 && p.w2 && p.b2 && p.w3 && p.b3 && p.h3 && p.rows > 0,
               "xa_conv_stack_fwd: null operand or rows <= 0");
  XA_CHECK_ARG(((uintptr_t)p.x & (p.x_u8 ? 3 : 15)) == 0,
               "xa_conv_stack_fwd: x must be %d-B aligned", p.x_u8 ? 4 : 16);
  const int G = (p.rows + CR - 1) / CR;
  const int grid = G < cu_count() ? G : cu_count();
  hipLaunchKernelGGL(conv_stack_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
  XA_CHECK_LAUNCH("xa_conv_stack_fwd");
  return 0;
}
