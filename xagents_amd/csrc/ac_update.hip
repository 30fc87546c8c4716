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
// The tile arithmetic (forward, loss, backward of 32 samples) lives in ac_tile.hpp, shared
// with the persistent whole-train-step update (ppo_update.hip).
#include <math.h>

#include "../../include/xagents_hip.h"
#include "ac_tile.hpp"
#include "xa_adam.hpp"
#include "xa_common.hpp"

namespace {

using xa_ac::H;
using xa_ac::S;
using xa_ac::Offs;
using xa_ac::offs;
constexpr int kStatsChunk = 1024;
constexpr int kRedThreads = 1024, kRedBatch = 16, kRedPB = 32;  // reduce: 32 row streams, one batch for <= 512 rows

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
  using namespace xa_ac;
  constexpr int RPT = Dims<OBS, A>::RPT;
  __shared__ __attribute__((aligned(16))) TileLds<OBS, A> L;

  const Offs o = offs(OBS, A);
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
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
    ParamSlice<OBS, A> ps;
    ps.init(tid);
    float wv[16], rv[RPT];
    if (p.pend_grad == nullptr) {
      ps.load(p.theta, wv, rv);
    } else {
      // every load of the step (theta, m, v, g) is issued before the first use
      float mw[16], vw[16], gw[16], mr[RPT], vr[RPT], gr[RPT];
      ps.load(p.theta, wv, rv);
      ps.load(p.pend_m, mw, mr);
      ps.load(p.pend_v, vw, vr);
      ps.load(p.pend_grad, gw, gr);
      double sq = 0.0;
      const float gs = p.adam.grad_scale;
#pragma unroll
      for (int i = 0; i < 16; ++i) gw[i] = gw[i] * gs;
#pragma unroll
      for (int q = 0; q < RPT; ++q) gr[q] = ps.ri[q] >= 0 ? gr[q] * gs : 0.0f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sq += (double)gw[i] * (double)gw[i];
#pragma unroll
      for (int q = 0; q < RPT; ++q) sq += (double)gr[q] * (double)gr[q];
      XA_STAMP(20);
      sq = xa_wave_sum_f64(sq);
      if (lane == 0) L.sNorm[w] = sq;
      const float alpha = adam_alpha(p.adam.lr, p.adam.beta1, p.adam.beta2, pend_t);
      __syncthreads();
      XA_STAMP(21);
      // every block forms the identical norm and step (fixed assignment and order)
      const double tot = (L.sNorm[0] + L.sNorm[1]) + (L.sNorm[2] + L.sNorm[3]);
      const float sc = clip_scale(tot, p.adam.clip_norm);
      const float omb1 = 1.0f - p.adam.beta1, omb2 = 1.0f - p.adam.beta2, eps = p.adam.eps;
#pragma unroll
      for (int i = 0; i < 16; ++i) adam_elem(gw[i] * sc, wv[i], mw[i], vw[i], alpha, omb1, omb2, eps);
#pragma unroll
      for (int q = 0; q < RPT; ++q) adam_elem(gr[q] * sc, rv[q], mr[q], vr[q], alpha, omb1, omb2, eps);
      if (blockIdx.x == 0) {
        ps.store(p.theta_out, wv, rv);
        ps.store(p.m_out, mw, mr);
        ps.store(p.v_out, vw, vr);
      }
    }
    ps.to_lds(L, wv, rv);
  }

  XA_STAMP(22);
  LossCfg cfg;
  cfg.is_ppo = is_ppo;
  cfg.has_adv_in = p.adv_in != nullptr;
  cfg.loss_scale = p.loss_scale;
  cfg.clip_norm = p.clip_norm;
  cfg.value_coef = p.value_coef;
  cfg.entropy_coef = p.entropy_coef;
  cfg.adv_eps = p.adv_eps;
  cfg.adv_mean = cfg.adv_std = 0.0f;
  if (is_ppo && p.adv_in == nullptr) {
    const double n = p.adv_count;
    const double mean = st1 / n;
    const double var = fmax(st2 / n - mean * mean, 0.0);
    cfg.adv_mean = (float)mean;
    cfg.adv_std = (float)sqrt(var);
  }
  cfg.adv_rstd = 1.0f / (cfg.adv_std + cfg.adv_eps);

  TileAcc<OBS, A> acc;
  acc.zero();
  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    __syncthreads();
    XA_STAMP(11);
    // ---- gather: the prefetched samples into LDS, next tile's loads issued ----
    if (tid < S) {
      L.sValid[tid] = n_valid;
#pragma unroll
      for (int k = 0; k < OBS; ++k) L.sX[tid * OBS + k] = nx[k];
      L.sAct[tid] = n_act;
      L.sRet[tid] = n_ret;
      L.sOldV[tid] = n_oldv;
      L.sOldLp[tid] = n_oldlp;
      L.sAdvIn[tid] = n_adv;
    }
    if (tile + (int)gridDim.x < n_tiles) fetch_tile(tile + gridDim.x);
    __syncthreads();
    XA_STAMP(12);
    tile_compute<OBS, A>(L, acc, cfg);
  }

  XA_STAMP(18);
  float* part = p.partials + (size_t)blockIdx.x * o.P;
  tile_write_row<OBS, A>(L, acc, [&](int i, float v) { part[i] = v; });
  if (p.loss_partials) {
    const float ls = tile_loss_sums<OBS, A>(L, acc);
    if (tid < 4) p.loss_partials[(size_t)blockIdx.x * 4 + tid] = ls;
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
