// Actor-critic update for the MLP: minibatch shuffle/gather, per-minibatch
// advantage statistics, fused forward + PPO/A2C loss + backward, gradient
// reduction, tf.clip_by_global_norm + Keras Adam.
//
// Replaces PPO.get_mini_batches / run_ppo_epochs / update_gradients
// (xagents/ppo/agent.py:96-191) and A2C.train_step (xagents/a2c/agent.py:190-218).
//
// xa_ac_grad schedule: a workgroup of 256 threads walks 64-sample tiles of the
// minibatch. Weights (W2 in both orientations) sit in LDS; every activation and
// back-propagated tile is an LDS-resident [64 x 64] f32 tile, and the three
// 64x64x64 products (H1*W2, H1^T*dA2, dA2*W2^T) run as 16x16 thread grids with
// 4x4 register tiles fed by ds_read_b128 (conflict-free: one operand broadcast
// across 16 lanes, the other one 256 contiguous bytes). Weight gradients stay in
// registers across tiles and each block writes ONE partial-gradient row; the
// rows are summed in f64 in fixed order by xa_grad_reduce (deterministic).
#include <math.h>

#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int H = XA_MLP_HIDDEN;
constexpr int S = 64;  // samples per tile

struct Offs {
  int w1, b1, w2, b2, w3, b3, w4, b4, P;
};
__host__ __device__ inline Offs offs(int obs, int A) {
  Offs o;
  o.w1 = 0;
  o.b1 = obs * H;
  o.w2 = o.b1 + H;
  o.b2 = o.w2 + H * H;
  o.w3 = o.b2 + H;
  o.b3 = o.w3 + H * A;
  o.w4 = o.b3 + A;
  o.b4 = o.w4 + H;
  o.P = o.b4 + 1;
  return o;
}

struct ShuffleKeys {
  uint32_t k[4];
  uint32_t half_bits;
};

XA_DEV ShuffleKeys shuffle_keys(const XaShuffle& sh, int epoch, int batch) {
  ShuffleKeys s;
  const uint64_t ctr = sh.rng_counter ? *sh.rng_counter : 0ull;
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

XA_DEV int shuffle_index(const XaShuffle& sh, const ShuffleKeys& keys, int epoch, int batch,
                         int g) {
  if (sh.perm) return sh.perm[(size_t)epoch * batch + g];
  return (int)xa_permute((uint32_t)g, (uint32_t)batch, keys.half_bits, keys.k[0], keys.k[1],
                         keys.k[2], keys.k[3]);
}

// ---------------------------------------------------------------------------
// advantage statistics: one block per (epoch, minibatch)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adv_stats_kernel(const float* __restrict__ ret,
                                                        const float* __restrict__ val, int batch,
                                                        int mb_size, int n_mb, XaShuffle sh,
                                                        double* stats) {
  __shared__ double red[2][4];
  const int e = blockIdx.x / n_mb, m = blockIdx.x % n_mb;
  const ShuffleKeys keys = shuffle_keys(sh, e, batch);
  const int start = m * mb_size;
  const int cnt = min(mb_size, batch - start);
  double s1 = 0.0, s2 = 0.0;
  for (int q = threadIdx.x; q < cnt; q += blockDim.x) {
    const int idx = shuffle_index(sh, keys, e, batch, start + q);
    const float adv = ret[idx] - val[idx];
    s1 += (double)adv;
    s2 += (double)adv * (double)adv;
  }
  s1 = xa_wave_sum_f64(s1);
  s2 = xa_wave_sum_f64(s2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = s1;
    red[1][wid] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    stats[(size_t)blockIdx.x * 2 + 0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    stats[(size_t)blockIdx.x * 2 + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// ---------------------------------------------------------------------------
// fused gather + forward + loss + backward
// ---------------------------------------------------------------------------
template <int OBS, int A>
__global__ __launch_bounds__(256) void ac_grad_kernel(XaAcGradArgs p) {
  constexpr int AH = A + 1;  // logits + value head
  __shared__ __attribute__((aligned(16))) float sW2[H * H];
  __shared__ __attribute__((aligned(16))) float sW2T[H * H];
  __shared__ __attribute__((aligned(16))) float sH1[S * H];   // [s][i]
  __shared__ __attribute__((aligned(16))) float sH1T[H * S];  // [i][s]
  __shared__ __attribute__((aligned(16))) float sH2[S * H];   // [s][j]
  __shared__ __attribute__((aligned(16))) float sH2T[H * S];  // [j][s]; reused as dA1 [s][i]
  __shared__ __attribute__((aligned(16))) float sdA2[S * H];  // [s][j]
  __shared__ __attribute__((aligned(16))) float sdA2T[H * S]; // [j][s]
  __shared__ float sW1[OBS * H], sb1[H], sb2[H], sW34[H * AH], sb34[AH];
  __shared__ float sX[S * OBS];
  __shared__ float sdZ[S * AH];
  __shared__ int sIdx[S];
  __shared__ float sLoss[4][4];

  const Offs o = offs(OBS, A);
  const int tid = threadIdx.x;
  const int ti = tid >> 4, tj = tid & 15;
  const int r0 = ti * 4, c0 = tj * 4;
  const float* __restrict__ th = p.theta;

  for (int i = tid; i < H * H; i += 256) {
    const float w = th[o.w2 + i];
    sW2[i] = w;
    sW2T[(i & 63) * H + (i >> 6)] = w;
  }
  for (int i = tid; i < OBS * H; i += 256) sW1[i] = th[o.w1 + i];
  if (tid < H) {
    sb1[tid] = th[o.b1 + tid];
    sb2[tid] = th[o.b2 + tid];
  }
  for (int i = tid; i < H * AH; i += 256) {
    const int j = i / AH, a = i - j * AH;
    sW34[i] = a < A ? th[o.w3 + j * A + a] : th[o.w4 + j];
  }
  if (tid < AH) sb34[tid] = tid < A ? th[o.b3 + tid] : th[o.b4];

  const bool is_ppo = p.loss_kind == XA_LOSS_PPO;
  const int start = p.mb_index * p.mb_size;
  const int cnt = min(p.mb_size, p.batch - start);
  const int n_tiles = (cnt + S - 1) / S;
  ShuffleKeys keys;
  if (is_ppo) keys = shuffle_keys(p.shuffle, p.epoch, p.batch);
  float adv_mean = 0.0f, adv_std = 0.0f;
  if (is_ppo && p.adv_in == nullptr) {
    const int sidx = p.epoch * ((p.batch + p.mb_size - 1) / p.mb_size) + p.mb_index;
    const double n = p.adv_count;
    const double mean = p.adv_stats[2 * sidx] / n;
    const double var = fmax(p.adv_stats[2 * sidx + 1] / n - mean * mean, 0.0);
    adv_mean = (float)mean;
    adv_std = (float)sqrt(var);
  }

  // register accumulators
  float gW2[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) gW2[a][b] = 0.0f;
  constexpr int NW34 = (H * AH + 255) / 256;
  constexpr int NW1 = (OBS * H + 255) / 256;
  float gW34[NW34], gW1[NW1];
#pragma unroll
  for (int q = 0; q < NW34; ++q) gW34[q] = 0.0f;
#pragma unroll
  for (int q = 0; q < NW1; ++q) gW1[q] = 0.0f;
  float gb1 = 0.0f, gb2 = 0.0f, gb34 = 0.0f;
  float l_pg = 0.0f, l_v = 0.0f, l_ent = 0.0f, l_cnt = 0.0f;

  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    __syncthreads();
    // ---- P1: gather ----
    if (tid < S) {
      const int q = tile * S + tid;
      int idx = -1;
      if (q < cnt) idx = is_ppo ? shuffle_index(p.shuffle, keys, p.epoch, p.batch, start + q)
                                : start + q;
      sIdx[tid] = idx;
    }
    __syncthreads();
    for (int e = tid; e < S * OBS; e += 256) {
      const int s = e / OBS, k = e - s * OBS;
      const int idx = sIdx[s];
      sX[e] = idx >= 0 ? p.obs[(size_t)idx * OBS + k] : 0.0f;
    }
    __syncthreads();
    // ---- P2: H1 = tanh(X W1 + b1) ----
    {
      float h[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float z = 0.0f;
#pragma unroll
          for (int k = 0; k < OBS; ++k) z = fmaf(sX[(r0 + ii) * OBS + k], sW1[k * H + c0 + jj], z);
          h[ii][jj] = xa_tanhf(z + sb1[c0 + jj]);
        }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
        *reinterpret_cast<float4*>(&sH1[(r0 + ii) * H + c0]) =
            make_float4(h[ii][0], h[ii][1], h[ii][2], h[ii][3]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        *reinterpret_cast<float4*>(&sH1T[(c0 + jj) * S + r0]) =
            make_float4(h[0][jj], h[1][jj], h[2][jj], h[3][jj]);
    }
    __syncthreads();
    // ---- P3: H2 = tanh(H1 W2 + b2) ----
    {
      float acc[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = 0.0f;
#pragma unroll 8
      for (int k = 0; k < H; ++k) {
        const float4 a4 = *reinterpret_cast<const float4*>(&sH1T[k * S + r0]);
        const float4 b4 = *reinterpret_cast<const float4*>(&sW2[k * H + c0]);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = fmaf(av[ii], bv[jj], acc[ii][jj]);
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = xa_tanhf(acc[ii][jj] + sb2[c0 + jj]);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
        *reinterpret_cast<float4*>(&sH2[(r0 + ii) * H + c0]) =
            make_float4(acc[ii][0], acc[ii][1], acc[ii][2], acc[ii][3]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        *reinterpret_cast<float4*>(&sH2T[(c0 + jj) * S + r0]) =
            make_float4(acc[0][jj], acc[1][jj], acc[2][jj], acc[3][jj]);
    }
    __syncthreads();
    // ---- P4: heads + loss + dL/dz (one thread per sample) ----
    if (tid < S) {
      const int s = tid;
      const int idx = sIdx[s];
      float z[AH];
#pragma unroll
      for (int a = 0; a < AH; ++a) z[a] = 0.0f;
      for (int j = 0; j < H; ++j) {
        const float hj = sH2T[j * S + s];
#pragma unroll
        for (int a = 0; a < AH; ++a) z[a] = fmaf(hj, sW34[j * AH + a], z[a]);
      }
#pragma unroll
      for (int a = 0; a < AH; ++a) z[a] = z[a] + sb34[a];
      float dz[AH];
#pragma unroll
      for (int a = 0; a < AH; ++a) dz[a] = 0.0f;
      if (idx >= 0) {
        const int act = p.actions[idx];
        float m = z[0];
#pragma unroll
        for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
        float e[A], ssum = 0.0f;
#pragma unroll
        for (int a = 0; a < A; ++a) {
          e[a] = xa_expf(z[a] - m);
          ssum = ssum + e[a];
        }
        const float ls = xa_logf(ssum);
        float lp[A], pr[A], ent = 0.0f, logp = 0.0f;
#pragma unroll
        for (int a = 0; a < A; ++a) {
          lp[a] = (z[a] - m) - ls;
          pr[a] = e[a] / ssum;
          ent = ent - pr[a] * lp[a];
          if (a == act) logp = lp[a];
        }
        const float v = z[A];
        const float R = p.returns[idx];
        const float oldv = p.old_values[idx];
        const float adv_raw = R - oldv;
        const float sc = p.loss_scale;
        float dlogp, dv, pg, vl;
        if (is_ppo) {
          const float adv =
              p.adv_in ? p.adv_in[idx] : (adv_raw - adv_mean) / (adv_std + p.adv_eps);
          const float ratio = xa_expf(logp - p.old_logp[idx]);
          const float c = p.clip_norm;
          const float pg1 = -adv * ratio;
          const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
          pg = fmaxf(pg1, pg2);
          dlogp = (pg1 >= pg2) ? (sc * -adv) * ratio : 0.0f;
          const float vclip = oldv + fminf(fmaxf(v - oldv, -c), c);
          const float vl1 = (v - R) * (v - R);
          const float vl2 = (vclip - R) * (vclip - R);
          vl = fmaxf(vl1, vl2);
          dv = (vl1 >= vl2) ? sc * p.value_coef * 0.5f * 2.0f * (v - R) : 0.0f;
        } else {
          pg = -(adv_raw * logp);
          dlogp = -sc * adv_raw;
          vl = (v - R) * (v - R);
          dv = sc * p.value_coef * 2.0f * (v - R);
        }
        const float ec = sc * p.entropy_coef;
#pragma unroll
        for (int a = 0; a < A; ++a)
          dz[a] = dlogp * ((a == act ? 1.0f : 0.0f) - pr[a]) + ec * pr[a] * (lp[a] + ent);
        dz[A] = dv;
        l_pg += pg;
        l_v += vl;
        l_ent += ent;
        l_cnt += 1.0f;
      }
#pragma unroll
      for (int a = 0; a < AH; ++a) sdZ[s * AH + a] = dz[a];
    }
    __syncthreads();
    // ---- P5: head grads, dA2 = (dZ W34^T) * (1 - H2^2) ----
#pragma unroll
    for (int q = 0; q < NW34; ++q) {
      const int oo = tid + q * 256;
      if (oo < H * AH) {
        const int j = oo & 63, a = oo >> 6;
        float acc = gW34[q];
        for (int s = 0; s < S; ++s) acc = fmaf(sH2[s * H + j], sdZ[s * AH + a], acc);
        gW34[q] = acc;
      }
    }
    if (tid < AH) {
      float acc = gb34;
      for (int s = 0; s < S; ++s) acc = acc + sdZ[s * AH + tid];
      gb34 = acc;
    }
    {
      float d[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float dh = 0.0f;
#pragma unroll
          for (int a = 0; a < AH; ++a)
            dh = fmaf(sdZ[(r0 + ii) * AH + a], sW34[(c0 + jj) * AH + a], dh);
          const float hv = sH2[(r0 + ii) * H + c0 + jj];
          d[ii][jj] = dh * (1.0f - hv * hv);
        }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
        *reinterpret_cast<float4*>(&sdA2[(r0 + ii) * H + c0]) =
            make_float4(d[ii][0], d[ii][1], d[ii][2], d[ii][3]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        *reinterpret_cast<float4*>(&sdA2T[(c0 + jj) * S + r0]) =
            make_float4(d[0][jj], d[1][jj], d[2][jj], d[3][jj]);
    }
    __syncthreads();
    // ---- P6: dW2 += H1^T dA2 ; db2 ; dA1 = (dA2 W2^T) * (1 - H1^2) -> sH2T ----
#pragma unroll 8
    for (int s = 0; s < S; ++s) {
      const float4 a4 = *reinterpret_cast<const float4*>(&sH1[s * H + r0]);
      const float4 b4 = *reinterpret_cast<const float4*>(&sdA2[s * H + c0]);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
      const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) gW2[ii][jj] = fmaf(av[ii], bv[jj], gW2[ii][jj]);
    }
    if (tid < H) {
      float acc = gb2;
      for (int s = 0; s < S; ++s) acc = acc + sdA2[s * H + tid];
      gb2 = acc;
    }
    {
      float acc[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = 0.0f;
#pragma unroll 8
      for (int j = 0; j < H; ++j) {
        const float4 a4 = *reinterpret_cast<const float4*>(&sdA2T[j * S + r0]);
        const float4 b4 = *reinterpret_cast<const float4*>(&sW2T[j * H + c0]);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[ii][jj] = fmaf(av[ii], bv[jj], acc[ii][jj]);
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const float4 h4 = *reinterpret_cast<const float4*>(&sH1[(r0 + ii) * H + c0]);
        const float hv[4] = {h4.x, h4.y, h4.z, h4.w};
        float dd[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) dd[jj] = acc[ii][jj] * (1.0f - hv[jj] * hv[jj]);
        *reinterpret_cast<float4*>(&sH2T[(r0 + ii) * H + c0]) =
            make_float4(dd[0], dd[1], dd[2], dd[3]);
      }
    }
    __syncthreads();
    // ---- P7: dW1 += X^T dA1 ; db1 ----
    const float* sdA1 = sH2T;
#pragma unroll
    for (int q = 0; q < NW1; ++q) {
      const int oo = tid + q * 256;
      if (oo < OBS * H) {
        const int k = oo >> 6, i = oo & 63;
        float acc = gW1[q];
        for (int s = 0; s < S; ++s) acc = fmaf(sX[s * OBS + k], sdA1[s * H + i], acc);
        gW1[q] = acc;
      }
    }
    if (tid < H) {
      float acc = gb1;
      for (int s = 0; s < S; ++s) acc = acc + sdA1[s * H + tid];
      gb1 = acc;
    }
  }

  // ---- write this block's partial-gradient row ----
  float* part = p.partials + (size_t)blockIdx.x * o.P;
#pragma unroll
  for (int ii = 0; ii < 4; ++ii)
    *reinterpret_cast<float4*>(&part[o.w2 + (r0 + ii) * H + c0]) =
        make_float4(gW2[ii][0], gW2[ii][1], gW2[ii][2], gW2[ii][3]);
#pragma unroll
  for (int q = 0; q < NW34; ++q) {
    const int oo = tid + q * 256;
    if (oo < H * AH) {
      const int j = oo & 63, a = oo >> 6;
      if (a < A) part[o.w3 + j * A + a] = gW34[q];
      else part[o.w4 + j] = gW34[q];
    }
  }
  if (tid < AH) {
    if (tid < A) part[o.b3 + tid] = gb34;
    else part[o.b4] = gb34;
  }
#pragma unroll
  for (int q = 0; q < NW1; ++q) {
    const int oo = tid + q * 256;
    if (oo < OBS * H) part[o.w1 + oo] = gW1[q];
  }
  if (tid < H) {
    part[o.b1 + tid] = gb1;
    part[o.b2 + tid] = gb2;
  }
  if (p.loss_partials) {
    if (tid < 64) {  // wave 0 holds every per-sample loss accumulator
      l_pg = xa_wave_sum(l_pg);
      l_v = xa_wave_sum(l_v);
      l_ent = xa_wave_sum(l_ent);
      l_cnt = xa_wave_sum(l_cnt);
      if (tid == 0) {
        float* lp = p.loss_partials + (size_t)blockIdx.x * 4;
        lp[0] = l_pg;
        lp[1] = l_v;
        lp[2] = l_ent;
        lp[3] = l_cnt;
      }
    }
  }
  (void)sLoss;
}

// ---------------------------------------------------------------------------
// gradient reduction over partial rows
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void grad_reduce_kernel(const float* __restrict__ part, int nb,
                                                          int P, float* __restrict__ g,
                                                          int* adam_step) {
  const int pi = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0 && adam_step) adam_step[0] += 1;
  if (pi >= P) return;
  double acc = 0.0;
  int b = 0;
  for (; b + 4 <= nb; b += 4) {
    const float a0 = part[(size_t)b * P + pi];
    const float a1 = part[(size_t)(b + 1) * P + pi];
    const float a2 = part[(size_t)(b + 2) * P + pi];
    const float a3 = part[(size_t)(b + 3) * P + pi];
    acc += ((double)a0 + (double)a1) + ((double)a2 + (double)a3);
  }
  for (; b < nb; ++b) acc += (double)part[(size_t)b * P + pi];
  g[pi] = (float)acc;
}

// ---------------------------------------------------------------------------
// global norm + clip + Keras Adam
// ---------------------------------------------------------------------------
constexpr int kSmallP = 65536;

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ g, int P,
                                                            float grad_scale, double* ws) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
    const float x = g[i] * grad_scale;
    acc += (double)x * (double)x;
  }
  acc = xa_wave_sum_f64(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void clip_adam_kernel(float* __restrict__ theta,
                                                        float* __restrict__ m,
                                                        float* __restrict__ v,
                                                        const float* __restrict__ g, int P,
                                                        float grad_scale, float clip, float lr,
                                                        float b1, float b2, float eps,
                                                        const int* step, const double* ws,
                                                        int n_ws, float* gnorm_out) {
  __shared__ double red[4];
  __shared__ float s_scale;
  double total = 0.0;
  if (ws == nullptr) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
      const float x = g[i] * grad_scale;
      acc += (double)x * (double)x;
    }
    acc = xa_wave_sum_f64(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    total = (red[0] + red[1]) + (red[2] + red[3]);
  } else {
    for (int i = 0; i < n_ws; ++i) total += ws[i];
  }
  if (threadIdx.x == 0) {
    const float gn = (float)sqrt(total);
    float sc = 1.0f;
    if (clip > 0.0f) sc = clip * fminf(1.0f / gn, 1.0f / clip);
    s_scale = sc;
    if (blockIdx.x == 0 && gnorm_out) gnorm_out[0] = gn;
  }
  __syncthreads();
  const float sc = s_scale;
  const int t = step ? *step : 1;
  const float b1p = (float)pow((double)b1, (double)t);
  const float b2p = (float)pow((double)b2, (double)t);
  const float alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  const float omb1 = 1.0f - b1, omb2 = 1.0f - b2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const float gg = (g[i] * grad_scale) * sc;
  float mm = m[i], vv = v[i];
  mm = mm + (gg - mm) * omb1;
  vv = vv + (gg * gg - vv) * omb2;
  m[i] = mm;
  v[i] = vv;
  theta[i] = theta[i] - (mm * alpha) / (sqrtf(vv) + eps);
}

template <int OBS, int A>
int launch_grad(const XaAcGradArgs* p, hipStream_t s) {
  hipLaunchKernelGGL((ac_grad_kernel<OBS, A>), dim3(p->n_blocks), dim3(256), 0, s, *p);
  XA_CHECK_LAUNCH("xa_ac_grad");
  return 0;
}

}  // namespace

extern "C" int xa_ac_grad_blocks(int mb_size) {
  const int tiles = (mb_size + S - 1) / S;
  // one tile per block up to 128 blocks; more samples per block beyond that keeps
  // the partial-gradient rows (the update's dominant HBM traffic) bounded
  return tiles < 128 ? tiles : 128;
}

extern "C" int xa_ppo_adv_stats(const float* returns, const float* values, int batch, int mb_size,
                                int epochs, const XaShuffle* shuffle, double* stats,
                                void* stream) {
  XA_CHECK_ARG(returns && values && stats && shuffle, "xa_ppo_adv_stats: null pointer");
  XA_CHECK_ARG(batch > 0 && mb_size > 0 && epochs > 0, "xa_ppo_adv_stats: bad sizes");
  const int n_mb = (batch + mb_size - 1) / mb_size;
  hipLaunchKernelGGL(adv_stats_kernel, dim3(epochs * n_mb), dim3(256), 0, (hipStream_t)stream,
                     returns, values, batch, mb_size, n_mb, *shuffle, stats);
  XA_CHECK_LAUNCH("xa_ppo_adv_stats");
  return 0;
}

extern "C" int xa_ac_grad(const XaAcGradArgs* p, void* stream) {
  XA_CHECK_ARG(p && p->theta && p->obs && p->actions && p->old_values && p->returns &&
                   p->partials,
               "xa_ac_grad: null pointer");
  XA_CHECK_ARG(p->batch > 0 && p->mb_size > 0 && p->n_blocks > 0, "xa_ac_grad: bad sizes");
  XA_CHECK_ARG(p->mb_index * p->mb_size < p->batch, "xa_ac_grad: minibatch index out of range");
  if (p->loss_kind == XA_LOSS_PPO)
    XA_CHECK_ARG(p->old_logp && (p->adv_in || (p->adv_stats && p->adv_count > 0)),
                 "xa_ac_grad: PPO needs old_logp and adv_stats (or adv_in)");
  const int obs_dim = p->obs_dim, n_actions = p->n_actions;
  hipStream_t s = (hipStream_t)stream;
  if (obs_dim == 4 && n_actions == 2) return launch_grad<4, 2>(p, s);
  if (obs_dim == 6 && n_actions == 3) return launch_grad<6, 3>(p, s);
  if (obs_dim == 8 && n_actions == 4) return launch_grad<8, 4>(p, s);
  if (obs_dim == 2 && n_actions == 3) return launch_grad<2, 3>(p, s);
  xa_set_error("xa_ac_grad: unsupported (obs_dim, n_actions) = (%d, %d)", obs_dim, n_actions);
  return -3;
}

extern "C" int xa_grad_reduce(const float* partials, int n_parts, int n_params, float* grad,
                              int* adam_step, void* stream) {
  XA_CHECK_ARG(partials && grad && n_parts > 0 && n_params > 0, "xa_grad_reduce: bad arguments");
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((n_params + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, partials, n_parts, n_params, grad, adam_step);
  XA_CHECK_LAUNCH("xa_grad_reduce");
  return 0;
}

extern "C" int xa_clip_adam(float* theta, float* adam_m, float* adam_v, const float* grad,
                            int n_params, float grad_scale, float clip_norm, float lr,
                            float beta1, float beta2, float eps, const int* adam_step,
                            double* workspace, float* gnorm_out, void* stream) {
  XA_CHECK_ARG(theta && adam_m && adam_v && grad && n_params > 0, "xa_clip_adam: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const double* ws = nullptr;
  int n_ws = 0;
  if (n_params > kSmallP) {
    XA_CHECK_ARG(workspace != nullptr, "xa_clip_adam: n_params > %d needs a workspace", kSmallP);
    n_ws = min(1024, (n_params + 4095) / 4096);
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(n_ws), dim3(256), 0, s, grad, n_params,
                       grad_scale, workspace);
    XA_CHECK_LAUNCH("xa_clip_adam(sumsq)");
    ws = workspace;
  }
  hipLaunchKernelGGL(clip_adam_kernel, dim3((n_params + 255) / 256), dim3(256), 0, s, theta,
                     adam_m, adam_v, grad, n_params, grad_scale, clip_norm, lr, beta1, beta2, eps,
                     adam_step, ws, n_ws, gnorm_out);
  XA_CHECK_LAUNCH("xa_clip_adam");
  return 0;
}
