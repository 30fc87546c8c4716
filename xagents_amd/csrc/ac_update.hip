// Actor-critic update for the MLP: minibatch shuffle + gather + advantage
// statistics, fused forward + PPO/A2C loss + backward, deterministic gradient
// reduction, tf.clip_by_global_norm + Keras Adam.
//
// Replaces PPO.get_mini_batches / run_ppo_epochs / update_gradients
// (xagents/ppo/agent.py:96-191) and A2C.train_step (xagents/a2c/agent.py:190-218).
//
// Per PPO train step (E epochs x M minibatches, k = 0 .. E*M-1):
//   xa_ppo_minibatches      shuffle (host perm or Feistel), gather every minibatch into
//                           contiguous rows, f64 advantage sums per 1024-sample chunk
//   xa_ac_grad(k)           [prologue: clip + Keras Adam of minibatch k-1's gradient,
//                           recomputed identically by every block from the reduced
//                           gradient; block 0 writes the new theta/m/v (ping-pong)]
//                           forward, loss, backward of 32-sample tiles -> partial rows
//   xa_grad_reduce(k)       partial rows -> gradient (f64, fixed order), Adam step += 1
//   [all-reduce of the gradient when data-parallel]
//   xa_clip_adam            the last minibatch's optimizer step
// so the optimizer costs no launch of its own inside the minibatch chain. A single
// optimizer step (A2C) uses xa_grad_reduce_adam instead: the reduce's last block runs
// clip + Adam (measured: for PPO's 16 chained steps the redundant per-block prologue is
// faster than a one-block tail, whose loads all miss the freshly invalidated L2).
//
// xa_ac_grad tile schedule (256 threads = 4 waves, 32 samples):
//   H1 = tanh(X W1 + b1)                (VALU, K = obs)
//   Z2 = H1 W2                          (MFMA f32 16x16x4, K = 64)
//   heads + loss + dL/dz                (8 lanes per sample, xor shuffles)
//   dA2 = (dZ W34^T) * (1 - H2^2)       (VALU, K = A + 1)
//   dW2 += H1^T dA2 ; dH1 = dA2 W2^T    (MFMA f32 16x16x4, K = 32 / 64)
//   dW1 += X^T dA1                      (VALU, K = 32)
// MFMA operands are read from LDS as contiguous 16-byte rows: the K index lane
// group q feeds is remapped to a contiguous block (k = 16q + kk), which only
// reorders the f32 accumulation (tolerance-checked against float64).
#include <math.h>

#include "../../include/xagents_hip.h"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

constexpr int H = XA_MLP_HIDDEN;
constexpr int S = 32;    // samples per tile
constexpr int LDW = 68;  // LDS row stride of [*][64] tiles (16-B aligned, conflict-spreading)
constexpr int LDT = 36;  // LDS row stride of transposed [64][32] tiles
constexpr int kStatsChunk = 1024;
constexpr int kRedThreads = 1024, kRedBatch = 16, kRedPB = 32;  // reduce: 32 row streams, one batch for <= 512 rows

typedef float f32x4 __attribute__((ext_vector_type(4)));

// D = A B + C on a 16x16 tile, K = 4: lane l feeds A[l&15][k=l>>4], B[k=l>>4][l&15];
// D[row = 4*(l>>4) + r][col = l&15] lands in register r (exact f32 fma chain).
XA_DEV f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

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

__host__ __device__ inline int stats_chunks(int mb_size) {
  return (mb_size + kStatsChunk - 1) / kStatsChunk;
}

// ---------------------------------------------------------------------------
// minibatch preparation: one block per (epoch, minibatch, 1024-sample chunk), one thread
// per sample (the shuffle index -> scattered loads -> stores chain runs once per thread)
// ---------------------------------------------------------------------------
constexpr int kMbThreads = kStatsChunk;

__global__ __launch_bounds__(kMbThreads) void minibatch_kernel(XaMinibatchArgs a, int n_mb,
                                                               int n_chunks) {
  constexpr int NW = kMbThreads / 64;
  __shared__ double red[2][NW];
  const int sidx = blockIdx.x / n_chunks, chunk = blockIdx.x % n_chunks;
  const int e = sidx / n_mb, m = sidx % n_mb;
  const ShuffleKeys keys = shuffle_keys(a.shuffle, e, a.batch);
  const int start = m * a.mb_size;
  const int cnt = min(a.mb_size, a.batch - start);
  const int q0 = chunk * kStatsChunk, q1 = min(cnt, q0 + kStatsChunk);
  const bool gather = a.mb_obs != nullptr;
  double s1 = 0.0, s2 = 0.0;
  for (int q = q0 + (int)threadIdx.x; q < q1; q += blockDim.x) {
    const int idx = shuffle_index(a.shuffle, keys, e, a.batch, start + q);
    const float r = a.returns[idx], v = a.values[idx];
    const float adv = r - v;
    s1 += (double)adv;
    s2 += (double)adv * (double)adv;
    if (gather) {
      const size_t row = (size_t)e * a.batch + start + q;
      for (int k = 0; k < a.obs_dim; ++k)
        a.mb_obs[row * a.obs_dim + k] = a.obs[(size_t)idx * a.obs_dim + k];
      a.mb_actions[row] = a.actions[idx];
      a.mb_old_logp[row] = a.old_logp[idx];
      a.mb_values[row] = v;
      a.mb_returns[row] = r;
    }
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
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      t1 += red[0][w];
      t2 += red[1][w];
    }
    a.stats[(size_t)blockIdx.x * 2 + 0] = t1;
    a.stats[(size_t)blockIdx.x * 2 + 1] = t2;
  }
}

// ---------------------------------------------------------------------------
// fused [pending optimizer step] + forward + loss + backward
// ---------------------------------------------------------------------------
template <int OBS, int A>
__global__ __launch_bounds__(256) void ac_grad_kernel(XaAcGradArgs p) {
  constexpr int AH = A + 1;            // logits + value head
  constexpr int NSLOT = AH + 2 + OBS;  // per-feature partial sums combined at the end
  constexpr int NREST = OBS * H + H + H + H * A + A + H + 1;  // parameters outside W2
  constexpr int RPT = (NREST + 255) / 256;                    // of them per thread
  __shared__ __attribute__((aligned(16))) float sW2[H * LDW];   // [i][j]
  __shared__ __attribute__((aligned(16))) float sW2T[H * LDW];  // [j][k] = W2[k][j]
  __shared__ __attribute__((aligned(16))) float sH1[S * LDW];   // [s][i]
  __shared__ __attribute__((aligned(16))) float sH1T[H * LDT];  // [i][s]
  __shared__ __attribute__((aligned(16))) float sH2[S * LDW];   // [s][j]; then dA1 [s][i]
  __shared__ __attribute__((aligned(16))) float sdA2[S * LDW];  // [s][j]
  __shared__ __attribute__((aligned(16))) float sdA2T[H * LDT]; // [j][s]
  __shared__ float sW1[OBS * H], sb1[H], sb2[H], sW34[H * AH], sb34[AH];
  __shared__ float sX[S * OBS], sdZ[S * AH];
  __shared__ float sAct[S], sOldLp[S], sOldV[S], sRet[S], sAdvIn[S];
  __shared__ int sValid[S];
  __shared__ float sRed[4 * H * NSLOT];
  __shared__ float sLoss[4][4];
  __shared__ double sNorm[4];

  const Offs o = offs(OBS, A);
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;     // MFMA lane coordinates
  const int f = tid & 63, c8 = (tid >> 6) * 8;  // element-wise phases: feature, 8-sample chunk
  XA_STAMP_DECL
  XA_STAMP(10);

  const bool is_ppo = p.loss_kind == XA_LOSS_PPO;
  const int start = p.mb_index * p.mb_size;
  const int cnt = min(p.mb_size, p.batch - start);
  const int n_tiles = (cnt + S - 1) / S;
  const size_t row0 = p.gathered ? (size_t)p.epoch * p.batch + start : 0;
  ShuffleKeys keys;
  if (is_ppo && !p.gathered) keys = shuffle_keys(p.shuffle, p.epoch, p.batch);
  // per-sample inputs of the next tile, fetched one tile ahead by threads < S
  float nx[OBS], n_act = 0.0f, n_ret = 0.0f, n_oldv = 0.0f, n_oldlp = 0.0f, n_adv = 0.0f;
  int n_valid = 0;
  auto fetch_tile = [&](int tile) {
    if (tid >= S) return;
    const int q = tile * S + tid;
    long idx = -1;
    if (tile < n_tiles && q < cnt) {
      if (p.gathered) idx = (long)(row0 + q);
      else idx = is_ppo ? shuffle_index(p.shuffle, keys, p.epoch, p.batch, start + q) : start + q;
    }
    n_valid = idx >= 0;
    const size_t ix = idx >= 0 ? (size_t)idx : 0;
#pragma unroll
    for (int k = 0; k < OBS; ++k) nx[k] = idx >= 0 ? p.obs[ix * OBS + k] : 0.0f;
    n_act = idx >= 0 ? (float)p.actions[ix] : 0.0f;
    n_ret = idx >= 0 ? p.returns[ix] : 0.0f;
    n_oldv = idx >= 0 ? p.old_values[ix] : 0.0f;
    n_oldlp = (idx >= 0 && is_ppo) ? p.old_logp[ix] : 0.0f;
    n_adv = (idx >= 0 && p.adv_in) ? p.adv_in[ix] : 0.0f;
  };
  fetch_tile(blockIdx.x);  // in flight while the parameters are prepared

  // advantage statistics of this minibatch and the Adam step: loaded up front so
  // their round trip overlaps the parameter loads
  double st1 = 0.0, st2 = 0.0;
  if (is_ppo && p.adv_in == nullptr) {
    const int n_mb = (p.batch + p.mb_size - 1) / p.mb_size;
    const int sidx = p.epoch * n_mb + p.mb_index;
    const int nc = stats_chunks(p.mb_size);
    for (int c = 0; c < nc; ++c) {
      st1 += p.adv_stats[2 * ((size_t)sidx * nc + c)];
      st2 += p.adv_stats[2 * ((size_t)sidx * nc + c) + 1];
    }
  }
  const int pend_t = p.pend_grad ? *p.adam_step : 0;

  // ---- parameters (optionally after the pending clip + Keras Adam step) ----
  {
    const int k0 = 4 * (tid >> 4), j0 = 4 * (tid & 15);  // this thread's 4x4 block of W2
    float wv[16], rv[RPT];
    int ri[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int r = tid + 256 * q;
      ri[q] = r < NREST ? (r < o.w2 ? r : r + H * H) : -1;
    }
    auto w2_at = [&](const float* base, int rr) {
      return *reinterpret_cast<const float4*>(&base[o.w2 + (k0 + rr) * H + j0]);
    };
    if (p.pend_grad == nullptr) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 t4 = w2_at(p.theta, rr);
        wv[4 * rr] = t4.x; wv[4 * rr + 1] = t4.y; wv[4 * rr + 2] = t4.z; wv[4 * rr + 3] = t4.w;
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) rv[q] = ri[q] >= 0 ? p.theta[ri[q]] : 0.0f;
    } else {
      float gw[16], gr[RPT];
      // every load of the step (g, theta, m, v) is issued before the first use
      float4 tw4[4], mw4[4], vw4[4];
      float tr[RPT], mr[RPT], vr[RPT];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        tw4[rr] = w2_at(p.theta, rr);
        mw4[rr] = w2_at(p.pend_m, rr);
        vw4[rr] = w2_at(p.pend_v, rr);
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        const int e = ri[q] >= 0 ? ri[q] : 0;
        tr[q] = p.theta[e];
        mr[q] = p.pend_m[e];
        vr[q] = p.pend_v[e];
      }
      double sq = 0.0;
      const float gs = p.adam.grad_scale;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 t4 = w2_at(p.pend_grad, rr);
        gw[4 * rr] = t4.x * gs; gw[4 * rr + 1] = t4.y * gs;
        gw[4 * rr + 2] = t4.z * gs; gw[4 * rr + 3] = t4.w * gs;
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) gr[q] = ri[q] >= 0 ? p.pend_grad[ri[q]] * gs : 0.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sq += (double)gw[i] * (double)gw[i];
#pragma unroll
      for (int q = 0; q < RPT; ++q) sq += (double)gr[q] * (double)gr[q];
      XA_STAMP(20);
      sq = xa_wave_sum_f64(sq);
      if (lane == 0) sNorm[w] = sq;
      const float alpha = adam_alpha(p.adam.lr, p.adam.beta1, p.adam.beta2, pend_t);
      __syncthreads();
      XA_STAMP(21);
      // every block forms the identical norm and step (fixed assignment and order)
      const double tot = (sNorm[0] + sNorm[1]) + (sNorm[2] + sNorm[3]);
      const float sc = clip_scale(tot, p.adam.clip_norm);
      const float omb1 = 1.0f - p.adam.beta1, omb2 = 1.0f - p.adam.beta2, eps = p.adam.eps;
      const bool writer = blockIdx.x == 0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float4 t4 = tw4[rr], m4 = mw4[rr], v4 = vw4[rr];
        float th[4] = {t4.x, t4.y, t4.z, t4.w}, mm[4] = {m4.x, m4.y, m4.z, m4.w},
              vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          adam_elem(gw[4 * rr + c] * sc, th[c], mm[c], vv[c], alpha, omb1, omb2, eps);
          wv[4 * rr + c] = th[c];
        }
        if (writer) {
          const size_t off = o.w2 + (k0 + rr) * H + j0;
          *reinterpret_cast<float4*>(&p.theta_out[off]) = make_float4(th[0], th[1], th[2], th[3]);
          *reinterpret_cast<float4*>(&p.m_out[off]) = make_float4(mm[0], mm[1], mm[2], mm[3]);
          *reinterpret_cast<float4*>(&p.v_out[off]) = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        if (ri[q] < 0) continue;
        float th = tr[q], mm = mr[q], vv = vr[q];
        adam_elem(gr[q] * sc, th, mm, vv, alpha, omb1, omb2, eps);
        rv[q] = th;
        if (writer) {
          p.theta_out[ri[q]] = th;
          p.m_out[ri[q]] = mm;
          p.v_out[ri[q]] = vv;
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      *reinterpret_cast<float4*>(&sW2[(k0 + rr) * LDW + j0]) =
          make_float4(wv[4 * rr], wv[4 * rr + 1], wv[4 * rr + 2], wv[4 * rr + 3]);
      *reinterpret_cast<float4*>(&sW2T[(j0 + rr) * LDW + k0]) =
          make_float4(wv[rr], wv[4 + rr], wv[8 + rr], wv[12 + rr]);
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int e = ri[q];
      if (e < 0) continue;
      const float x = rv[q];
      if (e < o.b1) sW1[e] = x;
      else if (e < o.w2) sb1[e - o.b1] = x;
      else if (e < o.w3) sb2[e - o.b2] = x;
      else if (e < o.b3) {
        const int jj = (e - o.w3) / A, a = (e - o.w3) - jj * A;
        sW34[jj * AH + a] = x;
      } else if (e < o.w4) sb34[e - o.b3] = x;
      else if (e < o.b4) sW34[(e - o.w4) * AH + A] = x;
      else sb34[A] = x;
    }
  }

  XA_STAMP(22);
  float adv_mean = 0.0f, adv_std = 0.0f;
  if (is_ppo && p.adv_in == nullptr) {
    const double n = p.adv_count;
    const double mean = st1 / n;
    const double var = fmax(st2 / n - mean * mean, 0.0);
    adv_mean = (float)mean;
    adv_std = (float)sqrt(var);
  }

  // register accumulators
  f32x4 gW2[4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) gW2[jt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float gW34[AH], gW1[OBS];
#pragma unroll
  for (int a = 0; a < AH; ++a) gW34[a] = 0.0f;
#pragma unroll
  for (int k = 0; k < OBS; ++k) gW1[k] = 0.0f;
  float gb1 = 0.0f, gb2 = 0.0f, gb34 = 0.0f;
  float l_pg = 0.0f, l_v = 0.0f, l_ent = 0.0f, l_cnt = 0.0f;

  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    __syncthreads();
    XA_STAMP(11);
    // ---- gather: the prefetched samples into LDS, next tile's loads issued ----
    if (tid < S) {
      sValid[tid] = n_valid;
#pragma unroll
      for (int k = 0; k < OBS; ++k) sX[tid * OBS + k] = nx[k];
      sAct[tid] = n_act;
      sRet[tid] = n_ret;
      sOldV[tid] = n_oldv;
      sOldLp[tid] = n_oldlp;
      sAdvIn[tid] = n_adv;
    }
    if (tile + (int)gridDim.x < n_tiles) fetch_tile(tile + gridDim.x);
    __syncthreads();
    XA_STAMP(12);
    // ---- H1 = tanh(X W1 + b1): feature f, samples c8..c8+7 ----
    {
      float hv[8];
#pragma unroll
      for (int ss = 0; ss < 8; ++ss) {
        const int s = c8 + ss;
        float z = 0.0f;
#pragma unroll
        for (int k = 0; k < OBS; ++k) z = fmaf(sX[s * OBS + k], sW1[k * H + f], z);
        hv[ss] = xa_tanhf(z + sb1[f]);
        sH1[s * LDW + f] = hv[ss];
      }
      *reinterpret_cast<float4*>(&sH1T[f * LDT + c8]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
      *reinterpret_cast<float4*>(&sH1T[f * LDT + c8 + 4]) = make_float4(hv[4], hv[5], hv[6], hv[7]);
    }
    __syncthreads();
    XA_STAMP(13);
    // ---- Z2 = H1 W2 (MFMA): wave w owns hidden columns 16w..16w+15 ----
    {
      float bv[16];
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const float4 t4 = *reinterpret_cast<const float4*>(&sW2T[(16 * w + li) * LDW + 16 * lq + 4 * v4]);
        bv[4 * v4] = t4.x; bv[4 * v4 + 1] = t4.y; bv[4 * v4 + 2] = t4.z; bv[4 * v4 + 3] = t4.w;
      }
      const float bias = sb2[16 * w + li];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float av[16];
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) {
          const float4 t4 = *reinterpret_cast<const float4*>(&sH1[(16 * st + li) * LDW + 16 * lq + 4 * v4]);
          av[4 * v4] = t4.x; av[4 * v4 + 1] = t4.y; av[4 * v4 + 2] = t4.z; av[4 * v4 + 3] = t4.w;
        }
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) acc = mfma4(av[kk], bv[kk], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sH2[(16 * st + 4 * lq + r) * LDW + 16 * w + li] = xa_tanhf(acc[r] + bias);
      }
    }
    __syncthreads();
    XA_STAMP(14);
    // ---- heads + loss + dL/dz: 8 lanes per sample ----
    {
      const int s = tid >> 3, pp = tid & 7;
      float z[AH];
#pragma unroll
      for (int a = 0; a < AH; ++a) z[a] = 0.0f;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = 8 * pp + jj;
        const float hj = sH2[s * LDW + j];
#pragma unroll
        for (int a = 0; a < AH; ++a) z[a] = fmaf(hj, sW34[j * AH + a], z[a]);
      }
#pragma unroll
      for (int a = 0; a < AH; ++a) z[a] = xa_sum8(z[a]) + sb34[a];
      if (pp == 0) {
        float dz[AH];
#pragma unroll
        for (int a = 0; a < AH; ++a) dz[a] = 0.0f;
        if (sValid[s]) {
          const int act = (int)sAct[s];
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
          const float R = sRet[s];
          const float oldv = sOldV[s];
          const float adv_raw = R - oldv;
          const float sc = p.loss_scale;
          float dlogp, dv, pg, vl;
          if (is_ppo) {
            const float adv =
                p.adv_in ? sAdvIn[s] : (adv_raw - adv_mean) / (adv_std + p.adv_eps);
            const float ratio = xa_expf(logp - sOldLp[s]);
            const float c = p.clip_norm;
            const float pg1 = -adv * ratio;
            const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
            pg = fmaxf(pg1, pg2);
            // tf.maximum routes the gradient to its first input when x >= y; the
            // second input's gradient passes tf.clip_by_value only inside [lo, hi]
            const bool r_in = ratio >= 1.0f - c && ratio <= 1.0f + c;
            dlogp = (pg1 >= pg2 || r_in) ? (sc * -adv) * ratio : 0.0f;
            const float dvo = v - oldv;
            const float vclip = oldv + fminf(fmaxf(dvo, -c), c);
            const float vl1 = (v - R) * (v - R);
            const float vl2 = (vclip - R) * (vclip - R);
            vl = fmaxf(vl1, vl2);
            // rounding can make oldv + (v - oldv) != v inside the clip range: the
            // clipped branch then still carries the gradient 2 (v_clip - R)
            const float kv = sc * p.value_coef * 0.5f * 2.0f;
            if (vl1 >= vl2) dv = kv * (v - R);
            else dv = (dvo >= -c && dvo <= c) ? kv * (vclip - R) : 0.0f;
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
    }
    __syncthreads();
    XA_STAMP(15);
    // ---- dA2 = (dZ W34^T) * (1 - H2^2); head / b2 partial grads ----
    {
      float dv8[8];
#pragma unroll
      for (int ss = 0; ss < 8; ++ss) {
        const int s = c8 + ss;
        float dh = 0.0f;
#pragma unroll
        for (int a = 0; a < AH; ++a) dh = fmaf(sdZ[s * AH + a], sW34[f * AH + a], dh);
        const float hv = sH2[s * LDW + f];
#pragma unroll
        for (int a = 0; a < AH; ++a) gW34[a] = fmaf(hv, sdZ[s * AH + a], gW34[a]);
        const float d = dh * (1.0f - hv * hv);
        gb2 = gb2 + d;
        sdA2[s * LDW + f] = d;
        dv8[ss] = d;
      }
      *reinterpret_cast<float4*>(&sdA2T[f * LDT + c8]) = make_float4(dv8[0], dv8[1], dv8[2], dv8[3]);
      *reinterpret_cast<float4*>(&sdA2T[f * LDT + c8 + 4]) = make_float4(dv8[4], dv8[5], dv8[6], dv8[7]);
      if (tid < AH) {
        float acc = gb34;
        for (int s = 0; s < S; ++s) acc = acc + sdZ[s * AH + tid];
        gb34 = acc;
      }
    }
    __syncthreads();
    XA_STAMP(16);
    // ---- dW2 += H1^T dA2 (rows 16w.., K = samples 8q+kk) and dH1 = dA2 W2^T ----
    {
      float av[8];
      {
        const float4 t0 = *reinterpret_cast<const float4*>(&sH1T[(16 * w + li) * LDT + 8 * lq]);
        const float4 t1 = *reinterpret_cast<const float4*>(&sH1T[(16 * w + li) * LDT + 8 * lq + 4]);
        av[0] = t0.x; av[1] = t0.y; av[2] = t0.z; av[3] = t0.w;
        av[4] = t1.x; av[5] = t1.y; av[6] = t1.z; av[7] = t1.w;
      }
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const float4 t0 = *reinterpret_cast<const float4*>(&sdA2T[(16 * jt + li) * LDT + 8 * lq]);
        const float4 t1 = *reinterpret_cast<const float4*>(&sdA2T[(16 * jt + li) * LDT + 8 * lq + 4]);
        const float bv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) gW2[jt] = mfma4(av[kk], bv[kk], gW2[jt]);
      }
      float wv[16];
#pragma unroll
      for (int v4 = 0; v4 < 4; ++v4) {
        const float4 t4 = *reinterpret_cast<const float4*>(&sW2[(16 * w + li) * LDW + 16 * lq + 4 * v4]);
        wv[4 * v4] = t4.x; wv[4 * v4 + 1] = t4.y; wv[4 * v4 + 2] = t4.z; wv[4 * v4 + 3] = t4.w;
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float dv16[16];
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) {
          const float4 t4 = *reinterpret_cast<const float4*>(&sdA2[(16 * st + li) * LDW + 16 * lq + 4 * v4]);
          dv16[4 * v4] = t4.x; dv16[4 * v4 + 1] = t4.y; dv16[4 * v4 + 2] = t4.z; dv16[4 * v4 + 3] = t4.w;
        }
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) acc = mfma4(dv16[kk], wv[kk], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int s = 16 * st + 4 * lq + r;
          const float h1 = sH1[s * LDW + 16 * w + li];
          sH2[s * LDW + 16 * w + li] = acc[r] * (1.0f - h1 * h1);  // dA1
        }
      }
    }
    __syncthreads();
    XA_STAMP(17);
    // ---- dW1 += X^T dA1 ; db1 ----
#pragma unroll
    for (int ss = 0; ss < 8; ++ss) {
      const int s = c8 + ss;
      const float d = sH2[s * LDW + f];
      gb1 = gb1 + d;
#pragma unroll
      for (int k = 0; k < OBS; ++k) gW1[k] = fmaf(sX[s * OBS + k], d, gW1[k]);
    }
  }

  XA_STAMP(18);
  // ---- combine the 4 sample-chunk partials per feature, write the partial row ----
  float* part = p.partials + (size_t)blockIdx.x * o.P;
  {
    float* r = sRed + ((tid >> 6) * H + f) * NSLOT;
#pragma unroll
    for (int a = 0; a < AH; ++a) r[a] = gW34[a];
    r[AH] = gb2;
    r[AH + 1] = gb1;
#pragma unroll
    for (int k = 0; k < OBS; ++k) r[AH + 2 + k] = gW1[k];
  }
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[o.w2 + (16 * w + 4 * lq + r) * H + 16 * jt + li] = gW2[jt][r];
  if (tid < AH) {
    if (tid < A) part[o.b3 + tid] = gb34;
    else part[o.b4] = gb34;
  }
  __syncthreads();
  for (int e = tid; e < H * NSLOT; e += 256) {
    const int ff = e / NSLOT, slot = e - ff * NSLOT;
    const float v = ((sRed[(0 * H + ff) * NSLOT + slot] + sRed[(1 * H + ff) * NSLOT + slot]) +
                     (sRed[(2 * H + ff) * NSLOT + slot] + sRed[(3 * H + ff) * NSLOT + slot]));
    if (slot < A) part[o.w3 + ff * A + slot] = v;
    else if (slot == A) part[o.w4 + ff] = v;
    else if (slot == AH) part[o.b2 + ff] = v;
    else if (slot == AH + 1) part[o.b1 + ff] = v;
    else part[o.w1 + (slot - AH - 2) * H + ff] = v;
  }
  if (p.loss_partials) {
    l_pg = xa_wave_sum(l_pg);
    l_v = xa_wave_sum(l_v);
    l_ent = xa_wave_sum(l_ent);
    l_cnt = xa_wave_sum(l_cnt);
    if (lane == 0) {
      sLoss[w][0] = l_pg;
      sLoss[w][1] = l_v;
      sLoss[w][2] = l_ent;
      sLoss[w][3] = l_cnt;
    }
    __syncthreads();
    if (tid < 4)
      p.loss_partials[(size_t)blockIdx.x * 4 + tid] =
          (sLoss[0][tid] + sLoss[1][tid]) + (sLoss[2][tid] + sLoss[3][tid]);
  }
  XA_STAMP(19);
}

// ---------------------------------------------------------------------------
// gradient reduction: a block owns PB consecutive parameters (lane % PB = parameter,
// so every row load of a wave is 64 / PB contiguous 4 PB-byte segments); its 16 x 64 / PB
// row streams take rows st, st + 16 (64 / PB), ...; each thread issues its row loads
// before the first use.
// With a tail, the last block to finish applies clip + Keras Adam to the whole
// gradient (xa_clip_adam's arithmetic and norm order, so bit-identical to it).
// ---------------------------------------------------------------------------
// PB parameters per block: a wave's lanes are (row stream rg = lane / PB, parameter
// lane % PB), so PB < 64 spreads the same rows over more blocks (more CUs pulling the
// partial rows) at 4 PB-byte segments per row load.
template <int PB>
__global__ __launch_bounds__(kRedThreads) void grad_reduce_kernel(const float* __restrict__ part,
                                                                  int nb, int P,
                                                                  float* __restrict__ g,
                                                                  int* adam_step, XaAdamTail tail,
                                                                  int has_tail) {
  constexpr int W = kRedThreads / 64, G = 64 / PB, NS = W * G;
  __shared__ double red[W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pl = lane % PB, rg = lane / PB;
  const int st = w * G + rg;  // this thread's row stream
  const int pidx = blockIdx.x * PB + pl;
  const int pc = min(pidx, P - 1);  // clamped: loads stay unconditional
  double acc = 0.0;
  for (int b0 = st; b0 < nb; b0 += NS * kRedBatch) {
    float x[kRedBatch];
#pragma unroll
    for (int r = 0; r < kRedBatch; ++r) {
      const int b = b0 + r * NS;
      x[r] = b < nb ? part[(size_t)b * P + pc] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < kRedBatch; r += 4)
      acc += ((double)x[r] + (double)x[r + 1]) + ((double)x[r + 2] + (double)x[r + 3]);
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && lane < PB && pidx < P) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < W; ++r)
#pragma unroll
      for (int q = 0; q < G; ++q) s += red[r][q * PB + lane];
    g[pidx] = (float)s;
  }
  if (!has_tail) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && adam_step) adam_step[0] += 1;
    return;
  }
  if (last_block_arrived(tail.arrivals)) adam_tail_apply(tail, g, P);
}

// ---------------------------------------------------------------------------
// standalone global norm + clip + Keras Adam (out of place allowed)
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

// fixed-order sum of the sumsq partials into ws[n] (one workgroup)
__global__ __launch_bounds__(256) void sumsq_finalize_kernel(double* ws, int n) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += ws[i];
  acc = xa_wave_sum_f64(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) ws[n] = (red[0] + red[1]) + (red[2] + red[3]);
}

// need_norm == 0: no clipping and no norm output (DQN / DDPG / TD3 minimize). Otherwise
// the global norm comes from `total` (large P: sumsq partials + finalize) or, for small P,
// from a full sum in every workgroup. Grid-stride over the parameters.
__global__ __launch_bounds__(256) void clip_adam_kernel(
    const float* theta, const float* m, const float* v, const float* __restrict__ g, int P,
    float grad_scale, float clip, float lr, float b1, float b2, float eps, const int* step,
    int need_norm, const double* total_p, float* gnorm_out, float* theta_o, float* m_o,
    float* v_o) {
  __shared__ double red[4];
  __shared__ float s_alpha;
  double total = 0.0;
  if (threadIdx.x == 0) s_alpha = adam_alpha(lr, b1, b2, step ? *step : 1);
  if (need_norm && total_p == nullptr) total = clip_norm_sumsq(g, P, grad_scale, red);
  else __syncthreads();
  if (need_norm && total_p != nullptr) total = *total_p;
  if (blockIdx.x == 0 && threadIdx.x == 0 && gnorm_out) gnorm_out[0] = (float)sqrt(total);
  const float sc = need_norm ? clip_scale(total, clip) : 1.0f;
  const float alpha = s_alpha, omb1 = 1.0f - b1, omb2 = 1.0f - b2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
    float th = theta[i], mm = m[i], vv = v[i];
    adam_elem((g[i] * grad_scale) * sc, th, mm, vv, alpha, omb1, omb2, eps);
    theta_o[i] = th;
    m_o[i] = mm;
    v_o[i] = vv;
  }
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
  // one 32-sample tile per block up to one block per CU; beyond that blocks walk
  // several tiles, which keeps the partial-gradient rows at <= 256 x P floats
  return tiles < 256 ? tiles : 256;
}

extern "C" int xa_ppo_adv_stats_size(int batch, int mb_size, int epochs) {
  if (batch <= 0 || mb_size <= 0 || epochs <= 0) return 0;
  const int n_mb = (batch + mb_size - 1) / mb_size;
  return 2 * epochs * n_mb * stats_chunks(mb_size);
}

extern "C" int xa_ppo_minibatches(const XaMinibatchArgs* a, void* stream) {
  XA_CHECK_ARG(a && a->returns && a->values && a->stats, "xa_ppo_minibatches: null pointer");
  XA_CHECK_ARG(a->batch > 0 && a->mb_size > 0 && a->epochs > 0, "xa_ppo_minibatches: bad sizes");
  XA_CHECK_ARG(a->mb_obs == nullptr ||
                   (a->obs && a->actions && a->old_logp && a->mb_actions && a->mb_old_logp &&
                    a->mb_values && a->mb_returns && a->obs_dim > 0),
               "xa_ppo_minibatches: gather needs obs/actions/old_logp and every mb_* output");
  const int n_mb = (a->batch + a->mb_size - 1) / a->mb_size;
  const int nc = stats_chunks(a->mb_size);
  hipLaunchKernelGGL(minibatch_kernel, dim3(a->epochs * n_mb * nc), dim3(kMbThreads), 0,
                     (hipStream_t)stream, *a, n_mb, nc);
  XA_CHECK_LAUNCH("xa_ppo_minibatches");
  return 0;
}

extern "C" int xa_ac_grad(const XaAcGradArgs* p, void* stream) {
  XA_CHECK_ARG(p && p->theta && p->obs && p->actions && p->old_values && p->returns &&
                   p->partials,
               "xa_ac_grad: null pointer");
  XA_CHECK_ARG(p->batch > 0 && p->mb_size > 0 && p->n_blocks > 0, "xa_ac_grad: bad sizes");
  XA_CHECK_ARG(p->mb_index * p->mb_size < p->batch, "xa_ac_grad: minibatch index out of range");
  XA_CHECK_ARG(((uintptr_t)p->theta & 15) == 0, "xa_ac_grad: theta must be 16-byte aligned");
  XA_CHECK_ARG(p->pend_grad == nullptr ||
                   (p->pend_m && p->pend_v && p->theta_out && p->m_out && p->v_out &&
                    p->adam_step && ((uintptr_t)p->pend_grad & 15) == 0 &&
                    ((uintptr_t)p->pend_m & 15) == 0 && ((uintptr_t)p->pend_v & 15) == 0 &&
                    ((uintptr_t)p->theta_out & 15) == 0 && ((uintptr_t)p->m_out & 15) == 0 &&
                    ((uintptr_t)p->v_out & 15) == 0 && p->theta_out != p->theta),
               "xa_ac_grad: a pending optimizer step needs 16-byte aligned grad/m/v and "
               "separate (ping-pong) theta/m/v outputs and adam_step");
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
  XaAdamTail none = {};
  // 32 parameters per block (147 blocks for the 4,675-parameter MLP): measured fastest
  // in the PPO minibatch chain (64: 0.549, 32: 0.522, 16: 0.554 ms per C2 train step)
  hipLaunchKernelGGL(grad_reduce_kernel<kRedPB>, dim3((n_params + kRedPB - 1) / kRedPB),
                     dim3(kRedThreads), 0, (hipStream_t)stream, partials, n_parts, n_params, grad,
                     adam_step, none, 0);
  XA_CHECK_LAUNCH("xa_grad_reduce");
  return 0;
}

extern "C" int xa_grad_reduce_adam(const float* partials, int n_parts, int n_params, float* grad,
                                   const XaAdamTail* tail, void* stream) {
  XA_CHECK_ARG(partials && grad && n_parts > 0 && n_params > 0 && tail,
               "xa_grad_reduce_adam: bad arguments");
  XA_CHECK_ARG(n_params <= XA_ADAM_TAIL_MAX_PARAMS,
               "xa_grad_reduce_adam: n_params %d > %d (use xa_grad_reduce + xa_clip_adam)",
               n_params, XA_ADAM_TAIL_MAX_PARAMS);
  XA_CHECK_ARG(tail->theta && tail->m && tail->v && tail->adam_step && tail->arrivals,
               "xa_grad_reduce_adam: the tail needs theta, m, v, adam_step and arrivals");
  hipLaunchKernelGGL(grad_reduce_kernel<kRedPB>, dim3((n_params + kRedPB - 1) / kRedPB),
                     dim3(kRedThreads), 0, (hipStream_t)stream, partials, n_parts, n_params, grad,
                     nullptr, *tail, 1);
  XA_CHECK_LAUNCH("xa_grad_reduce_adam");
  return 0;
}

extern "C" int xa_clip_adam(float* theta, float* adam_m, float* adam_v, const float* grad,
                            int n_params, float grad_scale, float clip_norm, float lr,
                            float beta1, float beta2, float eps, const int* adam_step,
                            double* workspace, float* gnorm_out, float* theta_out, float* m_out,
                            float* v_out, void* stream) {
  XA_CHECK_ARG(theta && adam_m && adam_v && grad && n_params > 0, "xa_clip_adam: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int need_norm = clip_norm > 0.0f || gnorm_out != nullptr;
  const double* total = nullptr;
  if (need_norm && n_params > kSmallP) {
    XA_CHECK_ARG(workspace != nullptr, "xa_clip_adam: n_params > %d needs a workspace", kSmallP);
    const int n_ws = min(1023, (n_params + 4095) / 4096);
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(n_ws), dim3(256), 0, s, grad, n_params,
                       grad_scale, workspace);
    XA_CHECK_LAUNCH("xa_clip_adam(sumsq)");
    hipLaunchKernelGGL(sumsq_finalize_kernel, dim3(1), dim3(256), 0, s, workspace, n_ws);
    XA_CHECK_LAUNCH("xa_clip_adam(sumsq finalize)");
    total = workspace + n_ws;
  }
  const int blocks = min((n_params + 255) / 256, 8192);
  hipLaunchKernelGGL(clip_adam_kernel, dim3(blocks), dim3(256), 0, s, theta, adam_m, adam_v, grad,
                     n_params, grad_scale, clip_norm, lr, beta1, beta2, eps, adam_step, need_norm,
                     total, gnorm_out, theta_out ? theta_out : theta, m_out ? m_out : adam_m,
                     v_out ? v_out : adam_v);
  XA_CHECK_LAUNCH("xa_clip_adam");
  return 0;
}
XA_DIAG_READER(xa_diag_read_stamps_update)
