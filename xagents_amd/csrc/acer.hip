// ACER (xagents/acer/agent.py:8-387) on gfx950: the per-trajectory part of
// ACER.update_gradients that is not a layer GEMM.
//
//   * xa_acer_grad: one wave per env trajectory (T + 1 rows of the env-major batch
//     [n_envs, n_steps + 1], the order of ACER.get_batch's reshape, acer/agent.py:164-169):
//       p = softmax(actor logits), V_t = sum_a p_a Q_a (update_gradients 319-323);
//       rho_t = p_a / (mu_a + eps) with mu = softmax(behaviour logits) (329-330);
//       Retrace returns, reverse scan over t (calculate_returns 195-208);
//       the actor gradient w.r.t. the probabilities, trust-region adjusted against the
//       average model (calculate_losses 232-260, calculate_grads 262-293), pushed through
//       the softmax to the logits; the critic gradient of the selected Q.
//     The bootstrap row t = T gets zero gradients (clip_last_step, 84-94). Per-env loss
//     partials [sum gain, sum entropy, sum 0.5 (R - Q_a)^2, sum adj > 0] are written in a
//     fixed order (no atomics); the host sums them.
//   * xa_ema: tf.train.ExponentialMovingAverage.apply without zero-debias:
//     shadow -= (shadow - var) (1 - decay) (update_avg_weights 114-125, apply 346).
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int kMaxA = 64;

XA_DEV void softmax_row(const float* z, int A, float* p) {
  float m = z[0];
  for (int a = 1; a < A; ++a) m = fmaxf(m, z[a]);
  float s = 0.0f;
  for (int a = 0; a < A; ++a) {
    p[a] = xa_expf(z[a] - m);
    s += p[a];
  }
  for (int a = 0; a < A; ++a) p[a] = p[a] / s;
}

// LDS per env: V[T + 1], rho_bar[T], Q_a[T], R[T]
__global__ void __launch_bounds__(64) acer_grad_kernel(XaAcerArgs h) {
  extern __shared__ float lds[];
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  const int T = h.n_steps, A = h.n_actions;
  float* sV = lds;
  float* sRho = sV + (T + 1);
  float* sQa = sRho + T;
  float* sR = sQa + T;
  const int64_t row0 = (int64_t)env * (T + 1);
  float p[kMaxA];
  // phase 1: state values of all T + 1 rows, truncated importance of the taken actions
  for (int t = lane; t <= T; t += 64) {
    const int64_t r = row0 + t;
    softmax_row(h.logits + r * h.ld_logits, A, p);
    const float* q = h.q + r * h.ld_q;
    float v = 0.0f;
    for (int a = 0; a < A; ++a) v += p[a] * q[a];
    sV[t] = v;
    if (t < T) {
      const int64_t s = (int64_t)env * T + t;
      const int act = h.actions[s];
      float mu[kMaxA];
      softmax_row(h.mu_logits + s * A, A, mu);
      sRho[t] = p[act] / (mu[act] + h.epsilon);
      sQa[t] = q[act];
    }
  }
  __syncthreads();
  // phase 2: Retrace (acer/agent.py:200-207), sequential in t
  if (lane == 0) {
    float ret = sV[T];
    for (int t = T - 1; t >= 0; --t) {
      const int64_t s = (int64_t)env * T + t;
      ret = h.rewards[s] + h.gamma * ret * (1.0f - h.dones[s]);
      sR[t] = ret;
      ret = fminf(1.0f, sRho[t]) * (ret - sQa[t]) + sV[t];
    }
  }
  __syncthreads();
  // phase 3: gradients
  const float inv_n = 1.0f / (float)h.n_total;
  const float vcoef = h.trust_region ? h.value_coef : h.value_coef * h.value_coef;
  float l_gain = 0.0f, l_ent = 0.0f, l_val = 0.0f, l_adj = 0.0f;
  for (int t = lane; t <= T; t += 64) {
    const int64_t r = row0 + t;
    float* dz = h.dlogits + r * h.ld_dlogits;
    float* dq = h.dq + r * h.ld_dq;
    if (t == T) {
      for (int a = 0; a < A; ++a) dz[a] = 0.0f, dq[a] = 0.0f;
      continue;
    }
    const int64_t s = (int64_t)env * T + t;
    const int act = h.actions[s];
    softmax_row(h.logits + r * h.ld_logits, A, p);
    const float R = sR[t];
    if (h.returns) h.returns[s] = R;
    const float w = (R - sV[t]) * fminf(h.importance_c, sRho[t]);
    float g[kMaxA];
    float ent = 0.0f;
    for (int a = 0; a < A; ++a) {
      const float lp = xa_logf(p[a] + h.epsilon);
      ent -= p[a] * lp;
      g[a] = -h.entropy_coef * (lp + p[a] / (p[a] + h.epsilon));
    }
    const float lpa = xa_logf(p[act] + h.epsilon);
    g[act] += w / (p[act] + h.epsilon);
    l_gain += lpa * w;
    l_ent += ent;
    if (h.trust_region) {
      float avg[kMaxA];
      softmax_row(h.avg_logits + r * h.ld_avg, A, avg);
      float kg = 0.0f, kk = 0.0f;
      for (int a = 0; a < A; ++a) {
        const float k = -avg[a] / (p[a] + h.epsilon);
        avg[a] = k;
        kg += k * g[a];
        kk += k * k;
      }
      const float adj = fmaxf(0.0f, (kg - h.delta) / (kk + h.epsilon));
      if (adj > 0.0f) l_adj += 1.0f;
      for (int a = 0; a < A; ++a) g[a] -= adj * avg[a];
    }
    // output gradient -g / n through the softmax: dz = p (G - sum_b p_b G_b)
    float pg = 0.0f;
    for (int a = 0; a < A; ++a) {
      g[a] = -g[a] * inv_n;
      pg += p[a] * g[a];
    }
    for (int a = 0; a < A; ++a) dz[a] = p[a] * (g[a] - pg);
    const float qa = h.q[r * h.ld_q + act];
    for (int a = 0; a < A; ++a) dq[a] = 0.0f;
    dq[act] = -(R - qa) * vcoef * inv_n;
    l_val += 0.5f * (R - qa) * (R - qa);
  }
  if (h.env_loss) {
    l_gain = xa_wave_sum(l_gain);
    l_ent = xa_wave_sum(l_ent);
    l_val = xa_wave_sum(l_val);
    l_adj = xa_wave_sum(l_adj);
    if (lane == 0) {
      float* o = h.env_loss + 4 * (int64_t)env;
      o[0] = l_gain, o[1] = l_ent, o[2] = l_val, o[3] = l_adj;
    }
  }
}

__global__ void ema_kernel(float* __restrict__ shadow, const float* __restrict__ var, int64_t n,
                           float one_minus_decay) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float s = shadow[i];
    shadow[i] = s - (s - var[i]) * one_minus_decay;
  }
}

}  // namespace

extern "C" int xa_acer_grad(const XaAcerArgs* p, void* stream) {
  // LDS: (4 n_steps + 1) floats within the 64 KB dynamic default
  XA_CHECK_ARG(p && p->n_envs > 0 && p->n_steps > 0 && p->n_steps <= 4000 &&
                   p->n_actions > 0 && p->n_actions <= kMaxA && p->n_total > 0 && p->logits &&
                   p->q && p->mu_logits && p->actions && p->rewards && p->dones &&
                   p->dlogits && p->dq && (!p->trust_region || p->avg_logits),
               "xa_acer_grad: bad arguments");
  const size_t lds = sizeof(float) * (4 * (size_t)p->n_steps + 1);
  hipLaunchKernelGGL(acer_grad_kernel, dim3(p->n_envs), dim3(64), lds, (hipStream_t)stream, *p);
  XA_CHECK_LAUNCH("xa_acer_grad");
  return 0;
}

extern "C" int xa_ema(float* shadow, const float* var, int64_t n, float decay, void* stream) {
  XA_CHECK_ARG(shadow && var && n > 0, "xa_ema: bad arguments");
  const float omd = 1.0f - decay;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ema_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     shadow, var, n, omd);
  XA_CHECK_LAUNCH("xa_ema");
  return 0;
}
