// Actor-critic heads for models run through the layer executor (the CNN actor-critic
// cfgs, xagents/{a2c,ppo}/models/cnn-actor-critic.cfg):
//   * xa_categorical: TFP Categorical(logits) sample / log-prob / entropy over a batch of
//     logit rows (A2C.get_model_outputs, xagents/a2c/agent.py:65-94), same arithmetic
//     and inverse-CDF sampling as the fused MLP rollout (mlp_rollout.hip);
//   * xa_diag_gaussian: MultivariateNormalDiag(loc) sample / log-prob / entropy for Box
//     action spaces (a2c/agent.py:59-60);
//   * xa_ac_head_grad: the PPO / A2C loss of a minibatch and its gradient w.r.t. the
//     logits (or the Gaussian mean) and the value head (PPO.update_gradients ppo/agent.py:96-137 with the
//     per-minibatch advantage normalisation of run_ppo_epochs 180-183; A2C.train_step
//     a2c/agent.py:190-218), TF tie semantics as in ac_update.hip.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int kMaxA = 64;
constexpr float kLog2Pi = 1.83787706640934548f;  // log(2 pi)

// MultivariateNormalDiag(loc = mu) with unit scale (a2c/agent.py:59-60, 86-92): sample
// a = mu + N(0, I) (Philox4x32-10 Box-Muller at counter (i, step, *rng_counter), or given
// noise / actions), log-prob and entropy. One thread per row.
__global__ void diag_gaussian_kernel(const float* __restrict__ mu, int64_t ld_mu, int n, int d,
                                     const float* __restrict__ noise,
                                     const uint64_t* __restrict__ ctr, uint64_t seed, int step,
                                     const float* __restrict__ actions_in, int64_t ld_act,
                                     float* __restrict__ act_out, float* __restrict__ logp,
                                     float* __restrict__ ent, int64_t ld_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* m = mu + (int64_t)i * ld_mu;
  const uint64_t c = ctr ? *ctr : 0ull;
  float ss = 0.0f;
  xa_u4 r = {0u, 0u, 0u, 0u};
  for (int j = 0; j < d; ++j) {
    float a;
    if (actions_in) {
      a = actions_in[(int64_t)i * ld_act + j];
    } else {
      float e;
      if (noise) {
        e = noise[(int64_t)i * d + j];
      } else {
        // one Philox draw per 4 dimensions (two Box-Muller pairs: r.x r.y, r.z r.w); the
        // counter is (row, step, *rng_counter) whole, the draw index j / 4 goes into the
        // key (Weyl step), so no (counter, dimension) pair repeats another's draw
        if ((j & 3) == 0)
          r = xa_philox((uint32_t)i, (uint32_t)step, (uint32_t)c, (uint32_t)(c >> 32),
                        (uint32_t)seed + (uint32_t)(j >> 2) * 0x9E3779B9u, (uint32_t)(seed >> 32));
        const uint32_t w1 = (j & 2) ? r.z : r.x, w2 = (j & 2) ? r.w : r.y;
        const float u1 = fmaxf(xa_u01(w1), 1.0e-7f), u2 = xa_u01(w2);
        const float rad = sqrtf(-2.0f * xa_logf(u1));
        e = rad * ((j & 1) ? sinf(6.283185307179586f * u2) : cosf(6.283185307179586f * u2));
      }
      a = m[j] + e;
      if (act_out) act_out[(int64_t)i * ld_act + j] = a;
    }
    const float dj = a - m[j];
    ss = fmaf(dj, dj, ss);
  }
  const int64_t o = (int64_t)i * ld_out;
  if (logp) logp[o] = -0.5f * ss - 0.5f * (float)d * kLog2Pi;
  if (ent) ent[o] = 0.5f * (float)d * (1.0f + kLog2Pi);
}

__global__ void categorical_kernel(const float* __restrict__ logits, int64_t ld, int n, int A,
                                   const float* __restrict__ uniforms,
                                   const uint64_t* __restrict__ ctr, uint64_t seed, int step,
                                   const int* __restrict__ actions_in, int* __restrict__ act_out,
                                   float* __restrict__ logp, float* __restrict__ ent,
                                   int64_t ld_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* l = logits + (int64_t)i * ld;
  float m = l[0];
  for (int a = 1; a < A; ++a) m = fmaxf(m, l[a]);
  float e[kMaxA];
  float s = 0.0f;
  for (int a = 0; a < A; ++a) {
    e[a] = xa_expf(l[a] - m);
    s = s + e[a];
  }
  const float ls = xa_logf(s);
  int act;
  if (actions_in) {
    act = actions_in[i];
  } else {
    float u;
    if (uniforms) {
      u = uniforms[i];
    } else {
      const uint64_t c = ctr ? *ctr : 0ull;
      const xa_u4 r = xa_philox((uint32_t)i, (uint32_t)step, (uint32_t)c, (uint32_t)(c >> 32),
                                (uint32_t)seed, (uint32_t)(seed >> 32));
      u = xa_u01(r.x);
    }
    const float target = u * s;
    act = A - 1;
    float c = 0.0f;
    for (int a = 0; a < A; ++a) {
      c = c + e[a];
      if (target < c) {
        act = a;
        break;
      }
    }
  }
  const float inv_s = 1.0f / s;
  float en = 0.0f, lp = 0.0f;
  for (int a = 0; a < A; ++a) {
    const float la = (l[a] - m) - ls;
    const float p = e[a] * inv_s;
    en = en - p * la;
    if (a == act) lp = la;
  }
  const int64_t o = (int64_t)i * ld_out;
  if (act_out) act_out[o] = act;
  if (logp) logp[o] = lp;
  if (ent) ent[o] = en;
}

// one workgroup: f64 advantage statistics of the minibatch, then per-sample gradients
// d loss / d logits [n, A] and d loss / d value [n] for loss = mean over the minibatch
__global__ __launch_bounds__(1024) void ac_head_grad_kernel(XaHeadGradArgs p) {
  __shared__ double red[2][16];
  __shared__ float sred[4][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = p.n, A = p.n_actions;
  const bool ppo = p.loss_kind == XA_LOSS_PPO;
  double t1 = 0.0, t2 = 0.0, cnt = (double)n;
  if (p.stats_mode == 2) {
    // statistics of the union minibatch, all-reduced over the data-parallel ranks
    t1 = p.adv_stats[0];
    t2 = p.adv_stats[1];
    cnt = p.adv_stats[2];
  } else {
    double s1 = 0.0, s2 = 0.0;
    for (int i = tid; i < n; i += blockDim.x) {
      const double adv = (double)(p.returns[i] - p.old_values[i]);
      s1 += adv;
      s2 += adv * adv;
    }
    s1 = xa_wave_sum_f64(s1);
    s2 = xa_wave_sum_f64(s2);
    if (lane == 0) {
      red[0][w] = s1;
      red[1][w] = s2;
    }
    __syncthreads();
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      t1 += red[0][k];
      t2 += red[1][k];
    }
    if (p.stats_mode == 1) {
      if (tid == 0) {
        p.adv_stats[0] = t1;
        p.adv_stats[1] = t2;
        p.adv_stats[2] = cnt;
      }
      return;
    }
  }
  const double mean = t1 / cnt;
  const float adv_mean = (float)mean;
  const float adv_std = (float)sqrt(fmax(t2 / cnt - mean * mean, 0.0));
  const float sc = 1.0f / (float)n;
  float l_pg = 0.0f, l_v = 0.0f, l_ent = 0.0f;
  const bool gauss = p.dist_kind == XA_DIST_DIAG_GAUSSIAN;
  for (int i = tid; i < n && gauss; i += blockDim.x) {
    // MultivariateNormalDiag(loc = z) with unit scale (a2c/agent.py:59-60):
    // log p(a) = -0.5 |a - z|^2 - 0.5 d log(2 pi), entropy 0.5 d (1 + log(2 pi)) is
    // constant (no gradient), d log p / d z = a - z
    const float* z = p.logits + (int64_t)i * p.ld_logits;
    const float* a = p.actions_f + (int64_t)i * p.ld_actions;
    float ss = 0.0f;
    for (int j = 0; j < A; ++j) {
      const float dj = a[j] - z[j];
      ss = fmaf(dj, dj, ss);
    }
    const float logp = -0.5f * ss - 0.5f * (float)A * kLog2Pi;
    const float ent = 0.5f * (float)A * (1.0f + kLog2Pi);
    const float v = p.values[(int64_t)i * p.ld_values];
    const float R = p.returns[i], oldv = p.old_values[i];
    const float adv_raw = R - oldv;
    float dlogp, dv, pg, vl;
    if (ppo) {
      const float adv = (adv_raw - adv_mean) / (adv_std + p.adv_eps);
      const float ratio = xa_expf(logp - p.old_logp[i]);
      const float c = p.clip_norm;
      const float pg1 = -adv * ratio;
      const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      pg = fmaxf(pg1, pg2);
      const bool r_in = ratio >= 1.0f - c && ratio <= 1.0f + c;
      dlogp = (pg1 >= pg2 || r_in) ? (sc * -adv) * ratio : 0.0f;
      const float dvo = v - oldv;
      const float vclip = oldv + fminf(fmaxf(dvo, -c), c);
      const float vl1 = (v - R) * (v - R), vl2 = (vclip - R) * (vclip - R);
      vl = fmaxf(vl1, vl2);
      const float kv = sc * p.value_coef * 0.5f * 2.0f;
      if (vl1 >= vl2) dv = kv * (v - R);
      else dv = (dvo >= -c && dvo <= c) ? kv * (vclip - R) : 0.0f;
    } else {
      pg = -(adv_raw * logp);
      dlogp = -sc * adv_raw;
      vl = (v - R) * (v - R);
      dv = sc * p.value_coef * 2.0f * (v - R);
    }
    float* dz = p.dlogits + (int64_t)i * A;
    for (int j = 0; j < A; ++j) dz[j] = dlogp * (a[j] - z[j]);
    p.dvalues[i] = dv;
    l_pg += pg;
    l_v += vl;
    l_ent += ent;
  }
  for (int i = tid; i < n && !gauss; i += blockDim.x) {
    const float* z = p.logits + (int64_t)i * p.ld_logits;
    const int act = p.actions[i];
    float m = z[0];
    for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
    float e[kMaxA];
    float ssum = 0.0f;
    for (int a = 0; a < A; ++a) {
      e[a] = xa_expf(z[a] - m);
      ssum = ssum + e[a];
    }
    const float ls = xa_logf(ssum);
    float ent = 0.0f, logp = 0.0f;
    float lp[kMaxA], pr[kMaxA];
    for (int a = 0; a < A; ++a) {
      lp[a] = (z[a] - m) - ls;
      pr[a] = e[a] / ssum;
      ent = ent - pr[a] * lp[a];
      if (a == act) logp = lp[a];
    }
    const float v = p.values[(int64_t)i * p.ld_values];
    const float R = p.returns[i], oldv = p.old_values[i];
    const float adv_raw = R - oldv;
    float dlogp, dv, pg, vl;
    if (ppo) {
      const float adv = (adv_raw - adv_mean) / (adv_std + p.adv_eps);
      const float ratio = xa_expf(logp - p.old_logp[i]);
      const float c = p.clip_norm;
      const float pg1 = -adv * ratio;
      const float pg2 = -adv * fminf(fmaxf(ratio, 1.0f - c), 1.0f + c);
      pg = fmaxf(pg1, pg2);
      const bool r_in = ratio >= 1.0f - c && ratio <= 1.0f + c;
      dlogp = (pg1 >= pg2 || r_in) ? (sc * -adv) * ratio : 0.0f;
      const float dvo = v - oldv;
      const float vclip = oldv + fminf(fmaxf(dvo, -c), c);
      const float vl1 = (v - R) * (v - R), vl2 = (vclip - R) * (vclip - R);
      vl = fmaxf(vl1, vl2);
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
    float* dz = p.dlogits + (int64_t)i * A;
    for (int a = 0; a < A; ++a)
      dz[a] = dlogp * ((a == act ? 1.0f : 0.0f) - pr[a]) + ec * pr[a] * (lp[a] + ent);
    p.dvalues[i] = dv;
    l_pg += pg;
    l_v += vl;
    l_ent += ent;
  }
  if (p.loss) {
    l_pg = xa_wave_sum(l_pg);
    l_v = xa_wave_sum(l_v);
    l_ent = xa_wave_sum(l_ent);
    if (lane == 0) {
      sred[0][w] = l_pg;
      sred[1][w] = l_v;
      sred[2][w] = l_ent;
    }
    __syncthreads();
    if (tid < 3) {
      float s = 0.0f;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += sred[tid][k];
      p.loss[tid] = s / (float)n;
    }
  }
}

}  // namespace

extern "C" int xa_categorical(const float* logits, int64_t ld_logits, int n, int n_actions,
                              const float* uniforms, const uint64_t* rng_counter, uint64_t seed,
                              int step, const int* actions_in, int* actions_out, float* logp,
                              float* entropy, int64_t ld_out, void* stream) {
  XA_CHECK_ARG(logits && n > 0 && n_actions > 0 && n_actions <= kMaxA && ld_logits >= n_actions,
               "xa_categorical: bad arguments (n_actions must be in [1, %d])", kMaxA);
  XA_CHECK_ARG(actions_in || uniforms || rng_counter || !actions_out,
               "xa_categorical: sampling needs uniforms or rng_counter");
  hipLaunchKernelGGL(categorical_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     logits, ld_logits, n, n_actions, uniforms, rng_counter, seed, step,
                     actions_in, actions_out, logp, entropy, ld_out > 0 ? ld_out : 1);
  XA_CHECK_LAUNCH("xa_categorical");
  return 0;
}

extern "C" int xa_diag_gaussian(const float* mu, int64_t ld_mu, int n, int d, const float* noise,
                                const uint64_t* rng_counter, uint64_t seed, int step,
                                const float* actions_in, int64_t ld_act, float* actions_out,
                                float* logp, float* entropy, int64_t ld_out, void* stream) {
  XA_CHECK_ARG(mu && n > 0 && d > 0 && ld_mu >= d && (actions_in || actions_out) &&
                   ld_act >= d,
               "xa_diag_gaussian: bad arguments");
  XA_CHECK_ARG(actions_in || noise || rng_counter,
               "xa_diag_gaussian: sampling needs noise or rng_counter");
  hipLaunchKernelGGL(diag_gaussian_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     mu, ld_mu, n, d, noise, rng_counter, seed, step, actions_in, ld_act,
                     actions_out, logp, entropy, ld_out > 0 ? ld_out : 1);
  XA_CHECK_LAUNCH("xa_diag_gaussian");
  return 0;
}

// One workgroup per (epoch, minibatch): f64 [sum adv, sum adv^2, count] of adv = returns -
// values over the minibatch's flat sample indices (run_ppo_epochs' per-minibatch
// normalisation, ppo/agent.py:180-183), summed in a fixed order (lane-strided partials,
// wave butterfly, waves in index order) so every call gives the same bits.
namespace {

__global__ __launch_bounds__(256) void minibatch_adv_sums_kernel(
    const float* __restrict__ returns, const float* __restrict__ values,
    const int64_t* __restrict__ idx, int batch, int mb_size, int n_mb,
    double* __restrict__ out) {
  __shared__ double red[2][4];
  const int set = blockIdx.x, e = set / n_mb, m = set - e * n_mb;
  const int64_t base = (int64_t)e * batch + (int64_t)m * mb_size;
  const int cnt = min(mb_size, batch - m * mb_size);
  double s1 = 0.0, s2 = 0.0;
  for (int q = threadIdx.x; q < cnt; q += blockDim.x) {
    const int64_t i = idx[base + q];
    const double adv = (double)(returns[i] - values[i]);
    s1 += adv;
    s2 += adv * adv;
  }
  s1 = xa_wave_sum_f64(s1);
  s2 = xa_wave_sum_f64(s2);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < 4; ++k) {
      t1 += red[0][k];
      t2 += red[1][k];
    }
    out[set * 3 + 0] = t1;
    out[set * 3 + 1] = t2;
    out[set * 3 + 2] = (double)cnt;
  }
}

}  // namespace

extern "C" int xa_minibatch_adv_sums(const float* returns, const float* values,
                                     const int64_t* idx, int batch, int mb_size, int epochs,
                                     double* out, void* stream) {
  XA_CHECK_ARG(returns && values && idx && out && batch > 0 && mb_size > 0 &&
                   mb_size <= batch && epochs > 0,
               "xa_minibatch_adv_sums: bad arguments");
  const int n_mb = (batch + mb_size - 1) / mb_size;
  hipLaunchKernelGGL(minibatch_adv_sums_kernel, dim3(epochs * n_mb), dim3(256), 0,
                     (hipStream_t)stream, returns, values, idx, batch, mb_size, n_mb, out);
  XA_CHECK_LAUNCH("xa_minibatch_adv_sums");
  return 0;
}

extern "C" int xa_ac_head_grad(const XaHeadGradArgs* p, void* stream) {
  XA_CHECK_ARG(p && (p->dist_kind != XA_DIST_DIAG_GAUSSIAN || (p->actions_f && p->ld_actions >= p->n_actions)),
               "xa_ac_head_grad: a Gaussian head needs actions_f [n, >= n_actions]");
  XA_CHECK_ARG(p && p->n > 0 && p->n_actions > 0 && p->n_actions <= kMaxA && p->logits &&
                   p->values && (p->actions || p->dist_kind == XA_DIST_DIAG_GAUSSIAN) &&
                   p->returns && p->old_values && p->dlogits &&
                   p->dvalues && (p->loss_kind != XA_LOSS_PPO || p->old_logp) &&
                   (p->stats_mode == 0 || p->adv_stats),
               "xa_ac_head_grad: bad arguments");
  hipLaunchKernelGGL(ac_head_grad_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *p);
  XA_CHECK_LAUNCH("xa_ac_head_grad");
  return 0;
}
