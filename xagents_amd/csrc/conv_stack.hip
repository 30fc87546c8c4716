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
#include "xa_adam.hpp"
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
XA_DEV f32x4 load_x4(const void* x, int x_u8, int rows, int row0, int i) {
  const int r = i / (CW0 / 4), c = i - r * (CW0 / 4);
  f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
  if (row0 + r < rows) {
    const int64_t off = (int64_t)(row0 + r) * CW0 + 4 * c;
    if (x_u8) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(x) + off);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (float)((u >> (8 * e)) & 0xFFu) / 255.0f;
    } else {
      v = *reinterpret_cast<const f32x4*>(static_cast<const float*>(x) + off);
    }
  }
  return v;
}

// workgroup blockIdx.x's share [s0, s1) of `rows` sequences: even shares over the grid (sizes
// differ by at most one), so a batch that is not a multiple of CR per workgroup leaves no
// workgroup with a whole extra chunk (64 frames = 5376 rows on 256 workgroups: 16 + 5 rows
// each, where one 16-row group per workgroup plus 80 second groups took two group times)
XA_DEV void stack_share(int rows, int& s0, int& s1) {
  const int64_t n = gridDim.x, b = blockIdx.x;
  s0 = (int)((int64_t)rows * b / n);
  s1 = (int)((int64_t)rows * (b + 1) / n);
}

XA_DEV void store_x4(float* xs, int i, f32x4 v) {
  *reinterpret_cast<f32x4*>(xs + 4 * i) = v;  // item i covers xs[4 i .. 4 i + 3]
}

__global__ __launch_bounds__(512) void conv_stack_fwd_kernel(XaConvStackArgs p) {
  __shared__ __attribute__((aligned(16))) float xs[CR * CW0];
  __shared__ __attribute__((aligned(16))) float h1s[M1 * LD1];
  __shared__ __attribute__((aligned(16))) float h2s[M2 * LD2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, i16 = lane & 15;
  // 8 waves: waves w and w + 4 share column tile wc = w & 3 of conv2 / conv3 (and its
  // weights) and split the M tiles by wh = w >> 2, so two waves per SIMD interleave
  const int wc = w & 3, wh = w >> 2;

  // this wave's weights: conv2 / conv3 columns 16 wc + i16, k = 16 kb + 4 q + j
  const int n2 = 16 * wc + i16;
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
  // conv1 (K = 8, 32 columns): column tile w & 1, M tiles w >> 1 (mod 4); MFMA j takes
  // k = 4 j + q
  const int n1 = 16 * (w & 1) + i16;
  const float w1a = p.w1[q * CF1 + n1], w1b = p.w1[(4 + q) * CF1 + n1], bias1 = p.b1[n1];

  // this workgroup's rows [s0, s1): an even share of the batch, walked in chunks of <= CR
  int s0, s1;
  stack_share(p.rows, s0, s1);
  if (s0 >= s1) return;
  for (int i = tid; i < XQ; i += 512)
    store_x4(xs, i, load_x4(p.x, p.x_u8, min(s0 + CR, s1), s0, i));
  __syncthreads();

  for (int row0 = s0; row0 < s1; row0 += CR) {
    const int nrow = min(CR, s1 - row0);
    // M tiles holding any of the chunk's rows (the rest are skipped; a partial tile's rows
    // past the chunk read zero inputs or stale LDS rows and are never stored)
    const int nt1 = (nrow * CP1 + 15) / 16, nt2 = (nrow * CP2 + 15) / 16, nt3 = (nrow * CP3 + 15) / 16;
    // ---- conv1: x -> h1 (bias + ReLU) ----
    for (int mt = w >> 1; mt < nt1; mt += 4) {
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
        if (p.h1 && mo < nrow * CP1) p.h1[((int64_t)row0 * CP1 + mo) * CF1 + n1] = v;
      }
    }
    __syncthreads();  // h1s complete; xs free
    // the next group's input, in flight during conv2
    const int rn = row0 + CR;
    const f32x4 xn = (rn < s1 && tid < XQ) ? load_x4(p.x, p.x_u8, min(rn + CR, s1), rn, tid)
                                            : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // ---- conv2: h1 -> h2, M tiles 0..4 (wh 0) / 5..8 (wh 1) of a full chunk, two per pass ----
    {
      const int h0 = (nt2 + 1) / 2, t0 = wh ? h0 : 0, nt = wh ? nt2 - h0 : h0;
      for (int i = 0; i < nt; i += 2) {
        const bool two = i + 1 < nt;
        int base[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int m = 16 * (t0 + min(i + s, nt - 1)) + i16, r = m / CP2, pp = m - r * CP2;
          base[s] = (r * CP1 + CS2 * pp) * LD1 + 4 * q;
        }
        f32x4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
        // k = 16 kb + 4 q + j: tap kb / 2, channel 16 (kb % 2) + 4 q + j; the next block's A
        // reads are issued before this block's MFMAs (pinning them there with scheduling
        // barriers measured slower on the 4-wave kernel: 46.2 vs 42.4 us, profiles/r05y)
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
            const int mo = 16 * (t0 + i + s) + 4 * q + e;
            const float v = fmaxf(acc[s][e] + bias2, 0.0f);
            h2s[mo * LD2 + n2] = v;
            if (p.h2 && mo < nrow * CP2) p.h2[((int64_t)row0 * CP2 + mo) * CF2 + n2] = v;
          }
        }
      }
    }
    if (rn < s1 && tid < XQ) store_x4(xs, tid, xn);
    __syncthreads();  // h2s complete; the next chunk's xs staged
    // ---- conv3: h2 -> h3 (HBM), M tiles 0..3 (wh 0) / 4..6 (wh 1) of a full chunk ----
    {
      const int h0 = (nt3 + 1) / 2, t0 = wh ? h0 : 0, nt = wh ? nt3 - h0 : h0;
      for (int i = 0; i < nt; i += 2) {
        const bool two = i + 1 < nt;
        int base[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int m = 16 * (t0 + min(i + s, nt - 1)) + i16, r = m / CP3, pp = m - r * CP3;
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
            const int mo = 16 * (t0 + i + s) + 4 * q + e;
            if (mo < nrow * CP3)
              p.h3[((int64_t)row0 * CP3 + mo) * CF3 + n2] = fmaxf(acc[s][e] + bias3, 0.0f);
          }
        }
      }
    }
    // no barrier here: the next conv1 writes only h1s (conv3 reads h2s), and the next
    // conv2 writes h2s after the next post-conv1 barrier
  }
}


// ---------------------------------------------------------------------------
// Fused backward of the same stack. Input: dZ3 = dL/d(conv3 pre-activation) [rows][7][64]
// (the dense layer's input gradient with h3's ReLU gate applied), the forward's h1 / h2 and
// the frames. Per 16-sequence group, out of LDS (x, h1, h2, dZ3: 147 KB with the pads):
//   (a) dW3 += im2col(h2)^T dZ3, db3 += colsum dZ3
//   (b) dZ2 = (dZ3 (*) W3^T, transposed conv) . [h2 > 0]       -> over h2 in place
//   (c) dW2 += im2col(h1)^T dZ2, db2 += colsum dZ2
//   (d) dZ1 = (dZ2 (*) W2^T, stride-2 transposed conv) . [h1 > 0] -> over h1 in place;
//       output position 2 h + par takes taps t = 2 s + par from dZ2 rows h - s (s = 0, 1),
//       so each wave's (par, 16-channel) tile is a K = 2 x 64 GEMM with no zero taps
//   (e) dW1 += im2col(x)^T dZ1, db1 += colsum dZ1
// Weight-gradient tiles stay in registers over all of a workgroup's groups (a wave owns
// filter columns 16 (w & 3) .. of dW3 / dW2 and half of their k tiles); the dgrad phases
// hold their 16-column slice of W3^T / W2^T in registers, loaded per group from L2. Each workgroup writes its partial
// [w1 b1 w2 b2 w3 b3] (20896 floats, theta order) to ws[blockIdx]; a second launch sums
// the partials in workgroup order (deterministic) into the gradient (+= when accumulate).
// ---------------------------------------------------------------------------
constexpr int LD3 = CF3 + 4;
constexpr int NW1 = CK1 * CF1, NB1 = CF1;                // 256, 32
constexpr int NW2 = CK2 * CF1 * CF2, NB2 = CF2;          // 8192, 64
constexpr int NW3 = CK3 * CF2 * CF3, NB3 = CF3;          // 12288, 64
constexpr int OW1 = 0, OB1 = NW1, OW2 = OB1 + NB1, OB2 = OW2 + NW2, OW3 = OB2 + NB2,
              OB3 = OW3 + NW3, NPAR = OB3 + NB3;         // 20896
constexpr int KT3 = CK3 * CF2 / 16, KT2 = CK2 * CF1 / 16;  // 12, 8 weight-gradient k tiles
constexpr int HH = CP1 / 2;                              // 10 output pairs of conv1
// the backward's dZ3 / h2 rows per sequence with zero rows around them, so the transposed
// convolutions read out-of-range taps as zeros instead of selecting (a select waits for its
// LDS read on the spot): dZ3 rows p3 = -2 .. 8 (taps of (b)), h2 rows p2 = -1 .. 9 ((d))
constexpr int D3B = CK3 - 1, D3R = CP3 + 2 * D3B;       // 2 before, 11 per sequence
constexpr int H2B = 1, H2R = CP2 + 2 * H2B;              // 1 before, 11 per sequence
XA_DEV int d3row(int m) { return (m / CP3) * D3R + D3B + m % CP3; }
XA_DEV int h2row(int m) { return (m / CP2) * H2R + H2B + m % CP2; }


// 8 waves (512 threads): two waves per 16-column tile, so every SIMD runs two waves whose
// MFMA chains and LDS waits interleave (a 4-wave version, one wave per SIMD holding ~512
// registers, reached ~56 % of its MFMA issue time: profiles/r05zm_conv_bwd_stamps.txt; this
// one is 1.2-2 % faster end to end, profiles/r05zo_conv_bwd8_ab.txt). Waves w and w + 4
// share column tile wc = w & 3 and split the work by wh = w >> 2: (a) / (c) the weight-
// gradient k tiles (6 / 4 each), (b) / (d) the M tiles (5 + 4 / 6 + 4), (e) m blocks by
// residue w >> 1 (mod 4). Staging: LDS rows [m][LD] <- global rows [m][C] (m < valid, later
// rows 0), every load of a group issued before the first store (a load per loop trip behind
// a branch waited out one memory latency each).
template <int NTT, int C>
XA_DEV void stage_load8(f32x4 (&v)[NTT], const float* src, int valid, int tot) {
  const f32x4* g = reinterpret_cast<const f32x4*>(src);
  const int last = min(valid * (C / 4), tot) - 1;
#pragma unroll
  for (int u = 0; u < NTT; ++u) v[u] = g[min((int)threadIdx.x + 512 * u, last)];
}
template <int NTT, int C, int LD, int P = 1, int PR = 1, int PB = 0>
XA_DEV void stage_store8(float* dst, const f32x4 (&v)[NTT], int valid, int tot) {
  const int last = valid * (C / 4) - 1;
#pragma unroll
  for (int u = 0; u < NTT; ++u) {
    const int i = threadIdx.x + 512 * u;
    if (i >= tot) break;
    const int m = i / (C / 4), c = 4 * (i - m * (C / 4));
    const int row = (m / P) * PR + PB + m % P;
    *reinterpret_cast<f32x4*>(dst + row * LD + c) = i <= last ? v[u] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  }
}
constexpr int TOT1 = M1 * CF1 / 4, TOT2 = M2 * CF2 / 4, TOT3 = M3 * CF3 / 4;
constexpr int N81 = (TOT1 + 511) / 512, N82 = (TOT2 + 511) / 512, N83 = (TOT3 + 511) / 512;
constexpr int KH3 = KT3 / 2, KH2 = KT2 / 2;  // weight-gradient k tiles per wave

__global__ __launch_bounds__(512) void conv_stack_bwd8_kernel(XaConvStackBwdArgs p) {
  __shared__ __attribute__((aligned(16))) float xs[CR * CW0];
  __shared__ __attribute__((aligned(16))) float h1s[M1 * LD1];          // h1, then dZ1
  __shared__ __attribute__((aligned(16))) float h2s[CR * H2R * LD2];    // h2, then dZ2
  __shared__ __attribute__((aligned(16))) float d3s[CR * D3R * LD3];    // dZ3
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, i16 = lane & 15;
  const int wc = w & 3, wh = w >> 2;
  const int cb = 16 * wc + i16, par = wc >> 1, cd = 16 * (wc & 1) + i16;
  XA_STAMP_DECL  // diagnostic build only (-DXA_STAMPS, tools/conv_stack_stamps.py)
  XA_STAMP(7);
  const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
  f32x4 g3[KH3], g2[KH2], g1 = z4;
#pragma unroll
  for (int i = 0; i < KH3; ++i) g3[i] = z4;
#pragma unroll
  for (int i = 0; i < KH2; ++i) g2[i] = z4;
  float bs3 = 0.0f, bs2 = 0.0f, bs1 = 0.0f;
  for (int i = tid; i < CR * H2R * LD2 / 4; i += 512) reinterpret_cast<f32x4*>(h2s)[i] = z4;
  for (int i = tid; i < CR * D3R * LD3 / 4; i += 512) reinterpret_cast<f32x4*>(d3s)[i] = z4;
  __syncthreads();

  // this workgroup's rows [s0, s1) in chunks of <= CR (stack_share); M tiles past a chunk's
  // rows are skipped: their staged rows are zero, so they would add exact zeros
  int s0, s1;
  stack_share(p.rows, s0, s1);
  for (int row0 = s0; row0 < s1; row0 += CR) {
    const int nrow = min(CR, s1 - row0);
    const int nt1 = (nrow * CP1 + 15) / 16, nt2 = (nrow * CP2 + 15) / 16;
    const int nt3 = (nrow * CP3 + 15) / 16, ntp = (nrow * HH + 15) / 16;
    {
      f32x4 v1[N81], v2[N82], v3[N83], vx;
      stage_load8<N81, CF1>(v1, p.h1 + (int64_t)row0 * CP1 * CF1, nrow * CP1, TOT1);
      stage_load8<N82, CF2>(v2, p.h2 + (int64_t)row0 * CP2 * CF2, nrow * CP2, TOT2);
      stage_load8<N83, CF3>(v3, p.dz3 + (int64_t)row0 * CP3 * CF3, nrow * CP3, TOT3);
      vx = load_x4(p.x, p.x_u8, row0 + nrow, row0, min(tid, XQ - 1));
      stage_store8<N81, CF1, LD1>(h1s, v1, nrow * CP1, TOT1);
      stage_store8<N82, CF2, LD2, CP2, H2R, H2B>(h2s, v2, nrow * CP2, TOT2);
      stage_store8<N83, CF3, LD3, CP3, D3R, D3B>(d3s, v3, nrow * CP3, TOT3);
      if (tid < XQ) store_x4(xs, tid, vx);
    }
    __syncthreads();
    XA_STAMP(0);
    // ---- (a) dW3: k tiles 6 wh .. 6 wh + 5, n tile wc ----
    for (int mb = 0; mb < nt3; ++mb) {
      float bq[4];
      int rb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * mb + 4 * q + j, r = m / CP3, pp = m - r * CP3;
        bq[j] = d3s[d3row(m) * LD3 + cb];
        rb[j] = (r * H2R + H2B + pp) * LD2;
        if (wh == 0) bs3 += bq[j];
      }
      float av[2][KH3];
      auto koff3 = [&](int kt) {
        const int k = KH3 * wh + kt;
        return (k >> 2) * LD2 + ((k & 3) << 4) + i16;
      };
#pragma unroll
      for (int kt = 0; kt < KH3; ++kt) av[0][kt] = h2s[rb[0] + koff3(kt)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < 3) {
#pragma unroll
          for (int kt = 0; kt < KH3; ++kt) av[(j + 1) & 1][kt] = h2s[rb[j + 1] + koff3(kt)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kt = 0; kt < KH3; ++kt) g3[kt] = mfma4(av[j & 1][kt], bq[j], g3[kt]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float wb3[KT3][4];
#pragma unroll
    for (int kb = 0; kb < KT3; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wb3[kb][j] = p.w3[((kb >> 2) * CF2 + cb) * CF3 + ((kb & 3) << 4) + 4 * q + j];
    __syncthreads();  // (a) has read h2
    XA_STAMP(1);
    // ---- (b) dZ2 over h2: column tile wc, M tiles 0..4 (wh 0) / 5..8 (wh 1) ----
    {
      const int h0 = (nt2 + 1) / 2, t0 = wh ? h0 : 0, nt = wh ? nt2 - h0 : h0;
      for (int i = 0; i < nt; i += 2) {
        int r[2], p2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int m = 16 * (t0 + min(i + u, nt - 1)) + i16;
          r[u] = m / CP2;
          p2[u] = m - r[u] * CP2;
        }
        f32x4 acc[2] = {z4, z4};
        auto rd3 = [&](int kb, int u) {
          return *reinterpret_cast<const f32x4*>(
              d3s + (r[u] * D3R + D3B + p2[u] - (kb >> 2)) * LD3 + ((kb & 3) << 4) + 4 * q);
        };
        f32x4 an[2] = {rd3(0, 0), rd3(0, 1)};
#pragma unroll
        for (int kb = 0; kb < KT3; ++kb) {
          const f32x4 a0 = an[0], a1 = an[1];
          if (kb + 1 < KT3) {
            an[0] = rd3(kb + 1, 0);
            an[1] = rd3(kb + 1, 1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[0] = mfma4(a0[j], wb3[kb][j], acc[0]);
            acc[1] = mfma4(a1[j], wb3[kb][j], acc[1]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (i + u >= nt) break;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float* hp = h2s + h2row(16 * (t0 + i + u) + 4 * q + e) * LD2 + cb;
            *hp = *hp > 0.0f ? acc[u][e] : 0.0f;
          }
        }
      }
    }
    __syncthreads();  // dZ2 complete
    XA_STAMP(2);
    // ---- (c) dW2: k tiles 4 wh .. 4 wh + 3, n tile wc ----
    for (int mb = 0; mb < nt2; ++mb) {
      float bq[4];
      int rb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 16 * mb + 4 * q + j, r = m / CP2, pp = m - r * CP2;
        bq[j] = h2s[h2row(m) * LD2 + cb];
        rb[j] = (r * CP1 + CS2 * pp) * LD1;
        if (wh == 0) bs2 += bq[j];
      }
      float av[2][KH2];
      auto koff2 = [&](int kt) {
        const int k = KH2 * wh + kt;
        return (k >> 1) * LD1 + ((k & 1) << 4) + i16;
      };
#pragma unroll
      for (int kt = 0; kt < KH2; ++kt) av[0][kt] = h1s[rb[0] + koff2(kt)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < 3) {
#pragma unroll
          for (int kt = 0; kt < KH2; ++kt) av[(j + 1) & 1][kt] = h1s[rb[j + 1] + koff2(kt)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kt = 0; kt < KH2; ++kt) g2[kt] = mfma4(av[j & 1][kt], bq[j], g2[kt]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float wb2[KT2][4];
#pragma unroll
    for (int kb = 0; kb < KT2; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wb2[kb][j] = p.w2[((2 * (kb >> 2) + par) * CF1 + cd) * CF2 + ((kb & 3) << 4) + 4 * q + j];
    __syncthreads();  // (c) has read h1
    XA_STAMP(3);
    // ---- (d) dZ1 over h1: column (par, 16-channel tile) wc, M tiles 0..5 / 6..9 ----
    {
      // 6 + 4 of a full chunk's 10 tiles: whole passes of two
      const int h0 = min(ntp, 2 * ((ntp + 3) / 4)), t0 = wh ? h0 : 0, nt = wh ? ntp - h0 : h0;
      for (int i = 0; i < nt; i += 2) {
        int r[2], hh[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int m = 16 * (t0 + min(i + u, nt - 1)) + i16;
          r[u] = m / HH;
          hh[u] = m - r[u] * HH;
        }
        f32x4 acc[2] = {z4, z4};
        auto rd2 = [&](int kb, int u) {
          return *reinterpret_cast<const f32x4*>(
              h2s + (r[u] * H2R + H2B + hh[u] - (kb >> 2)) * LD2 + ((kb & 3) << 4) + 4 * q);
        };
        f32x4 an[2] = {rd2(0, 0), rd2(0, 1)};
#pragma unroll
        for (int kb = 0; kb < KT2; ++kb) {
          const f32x4 a0 = an[0], a1 = an[1];
          if (kb + 1 < KT2) {
            an[0] = rd2(kb + 1, 0);
            an[1] = rd2(kb + 1, 1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[0] = mfma4(a0[j], wb2[kb][j], acc[0]);
            acc[1] = mfma4(a1[j], wb2[kb][j], acc[1]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (i + u >= nt) break;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int mo = 16 * (t0 + i + u) + 4 * q + e, ro = mo / HH, ho = mo - ro * HH;
            float* hp = h1s + (ro * CP1 + 2 * ho + par) * LD1 + cd;
            *hp = *hp > 0.0f ? acc[u][e] : 0.0f;
          }
        }
      }
    }
    __syncthreads();  // dZ1 complete
    XA_STAMP(4);
    // ---- (e) dW1: n tile w & 1, m blocks w >> 1 (mod 4), all reads of a pass first ----
    {
      const int n1 = 16 * (w & 1) + i16;
      float av[M1 / 64][4], bv[M1 / 64][4];
#pragma unroll
      for (int u = 0; u < M1 / 64; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = 16 * (4 * u + (w >> 1)) + 4 * q + j, r = m / CP1, pp = m - r * CP1;
          const bool in = 4 * u + (w >> 1) < nt1;  // (a skipped tile's rows add zeros)
          bv[u][j] = in ? h1s[m * LD1 + n1] : 0.0f;
          const float a = xs[r * CW0 + CS1 * pp + (i16 & (CK1 - 1))];
          av[u][j] = in && i16 < CK1 ? a : 0.0f;
        }
#pragma unroll
      for (int u = 0; u < M1 / 64; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          g1 = mfma4(av[u][j], bv[u][j], g1);
          bs1 += bv[u][j];
        }
    }
    __syncthreads();  // LDS free for the next group
    XA_STAMP(5);
  }

  // ---- partials -> ws[blockIdx.x][NPAR] ----
  float* out = p.ws + (int64_t)blockIdx.x * NPAR;
#pragma unroll
  for (int kt = 0; kt < KH3; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      out[OW3 + (16 * (KH3 * wh + kt) + 4 * q + e) * CF3 + cb] = g3[kt][e];
#pragma unroll
  for (int kt = 0; kt < KH2; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      out[OW2 + (16 * (KH2 * wh + kt) + 4 * q + e) * CF2 + cb] = g2[kt][e];
  float* red = h1s;
  red[tid] = bs3;
  red[512 + tid] = bs2;
  red[1024 + tid] = bs1;
#pragma unroll
  for (int e = 0; e < 4; ++e) red[1536 + e * 512 + tid] = g1[e];
  __syncthreads();
  if (tid < CF3) {  // db3 / db2: column n = 16 wc + i16 from waves wc (wh = 0), 4 lane groups
    const int wn = tid >> 4, ln = tid & 15;
    float s3 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      s3 += red[wn * 64 + qq * 16 + ln];
      s2 += red[512 + wn * 64 + qq * 16 + ln];
    }
    out[OB3 + tid] = s3;
    out[OB2 + tid] = s2;
  }
  if (tid < CF1) {  // db1: column 16 t + i16 from waves w = 2 rr + t (rr = 0..3), lane groups
    const int wt = tid >> 4, ln = tid & 15;
    float s1 = 0.0f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) s1 += red[1024 + (2 * rr + wt) * 64 + qq * 16 + ln];
    out[OB1 + tid] = s1;
  }
  if (tid < NW1) {  // dW1 [k1][n1]: D rows k1 = 4 q + e (q < 2) of waves 2 rr + (n1 >> 4)
    const int k1 = tid / CF1, n1 = tid - k1 * CF1, wt = n1 >> 4, ln = n1 & 15;
    const int qq = k1 >> 2, e = k1 & 3;
    float s = 0.0f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s += red[1536 + e * 512 + (2 * rr + wt) * 64 + qq * 16 + ln];
    out[OW1 + tid] = s;
  }
  XA_STAMP(6);
}

// grad[e] (+)= sum over workgroups z of ws[z][e]: 4 waves per 64 elements, wave v sums the
// z slice [v nz / 4, (v + 1) nz / 4) in order, the slices combined in order
// (+ optionally Keras Adam on those parameters and on a second range whose gradient is already
// final: blocks past the reduce's take that range, one element per thread -- xa_clip_adam's
// element arithmetic with no clip, so the same values as the separate launches)
__global__ __launch_bounds__(256) void conv_stack_bwd_reduce_kernel(const float* __restrict__ ws,
                                                                    int nz, XaConvStackBwdArgs p) {
  __shared__ float part[4][64];
  __shared__ float s_alpha;
  constexpr int kMain = (NPAR + 63) / 64;
  if (p.adam_on && threadIdx.x == 0) {
    const XaAdamApply& ad = (int)blockIdx.x < kMain ? p.adam : p.rest;
    s_alpha = adam_alpha(ad.lr, ad.beta1, ad.beta2, *ad.step);
  }
  if ((int)blockIdx.x >= kMain) {  // the second Adam range
    __syncthreads();
    const XaAdamApply& ad = p.rest;
    const int i = ((int)blockIdx.x - kMain) * 256 + (int)threadIdx.x;
    if (i < p.n_rest) {
      float th = ad.theta[i], mm = ad.m[i], vv = ad.v[i];
      adam_elem((p.rest_grad[i] * ad.grad_scale) * 1.0f, th, mm, vv, s_alpha, 1.0f - ad.beta1,
                1.0f - ad.beta2, ad.eps);
      ad.theta[i] = th;
      ad.m[i] = mm;
      ad.v[i] = vv;
    }
    return;
  }
  float* __restrict__ grad = p.grad;
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6, e = blockIdx.x * 64 + lane;
  const int z0 = v * nz / 4, z1 = (v + 1) * nz / 4;
  float s = 0.0f;
  if (e < NPAR) {
    int z = z0;
    for (; z + 8 <= z1; z += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = ws[(int64_t)(z + u) * NPAR + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; z < z1; ++z) s += ws[(int64_t)z * NPAR + e];
  }
  part[v][lane] = s;
  __syncthreads();
  if (v == 0 && e < NPAR) {
    const float t = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    if (!p.adam_on) {
      grad[e] = p.accumulate ? grad[e] + t : t;
    } else {
      if (p.write_grad) grad[e] = t;
      const XaAdamApply& ad = p.adam;
      float th = ad.theta[e], mm = ad.m[e], vv = ad.v[e];
      adam_elem((t * ad.grad_scale) * 1.0f, th, mm, vv, s_alpha, 1.0f - ad.beta1,
                1.0f - ad.beta2, ad.eps);
      ad.theta[e] = th;
      ad.m[e] = mm;
      ad.v[e] = vv;
    }
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

// one workgroup per CU, each an even share of the rows (at most one per row)
int stack_grid(int rows) { return rows < cu_count() ? rows : cu_count(); }

}  // namespace

XA_DIAG_READER(xa_diag_read_stamps_conv)

extern "C" int xa_conv_stack_fwd(const XaConvStackArgs* a, void* stream) {
  XA_CHECK_ARG(a != nullptr, "xa_conv_stack_fwd: null args");
  const XaConvStackArgs& p = *a;
  XA_CHECK_ARG(p.x && p.w1 && p.b1 && p.w2 && p.b2 && p.w3 && p.b3 && p.h3 && p.rows > 0,
               "xa_conv_stack_fwd: null operand or rows <= 0");
  XA_CHECK_ARG(((uintptr_t)p.x & (p.x_u8 ? 3 : 15)) == 0,
               "xa_conv_stack_fwd: x must be %d-B aligned", p.x_u8 ? 4 : 16);
  const int grid = stack_grid(p.rows);
  hipLaunchKernelGGL(conv_stack_fwd_kernel, dim3(grid), dim3(512), 0, (hipStream_t)stream, p);
  XA_CHECK_LAUNCH("xa_conv_stack_fwd");
  return 0;
}

extern "C" size_t xa_conv_stack_bwd_workspace_floats(int rows) {
  return (size_t)stack_grid(rows) * NPAR;
}

extern "C" int xa_conv_stack_bwd(const XaConvStackBwdArgs* a, void* stream) {
  XA_CHECK_ARG(a != nullptr, "xa_conv_stack_bwd: null args");
  const XaConvStackBwdArgs& p = *a;
  XA_CHECK_ARG(p.x && p.w2 && p.w3 && p.h1 && p.h2 && p.dz3 && p.ws && p.rows > 0 &&
                   (p.grad || (p.adam_on && !p.write_grad)),
               "xa_conv_stack_bwd: null operand or rows <= 0");
  XA_CHECK_ARG(!p.adam_on || (!p.accumulate && p.adam.theta && p.adam.m && p.adam.v &&
                              p.adam.step && (p.n_rest <= 0 || (p.rest.theta && p.rest.m &&
                                                                p.rest.v && p.rest.step &&
                                                                p.rest_grad))),
               "xa_conv_stack_bwd: adam_on needs accumulate 0 and the Adam pointers (and the "
               "rest range's with n_rest > 0)");
  XA_CHECK_ARG(((uintptr_t)p.x & (p.x_u8 ? 3 : 15)) == 0 &&
                   (((uintptr_t)p.h1 | (uintptr_t)p.h2 | (uintptr_t)p.dz3) & 15) == 0,
               "xa_conv_stack_bwd: x, h1, h2, dz3 misaligned");
  XA_CHECK_ARG(p.ws_floats >= xa_conv_stack_bwd_workspace_floats(p.rows),
               "xa_conv_stack_bwd: workspace of %zu floats needed",
               xa_conv_stack_bwd_workspace_floats(p.rows));
  const int grid = stack_grid(p.rows);
  hipLaunchKernelGGL(conv_stack_bwd8_kernel, dim3(grid), dim3(512), 0, (hipStream_t)stream, p);
  XA_CHECK_LAUNCH("xa_conv_stack_bwd");
  const int rest_blocks = p.adam_on && p.n_rest > 0 ? (p.n_rest + 255) / 256 : 0;
  hipLaunchKernelGGL(conv_stack_bwd_reduce_kernel, dim3((NPAR + 63) / 64 + rest_blocks), dim3(256),
                     0, (hipStream_t)stream, p.ws, grid, p);
  XA_CHECK_LAUNCH("xa_conv_stack_bwd (reduce)");
  return 0;
}
