/*
 * xa_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the xagents hot
 * path used as the parity checker for libxagents_hip.so. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path never does.
 *
 * It restates, in the exact f32 operation order the HIP kernels use (compiled
 * with -ffp-contract=off, explicit fmaf), the reference algorithms:
 *   - GAE            xagents/ppo/agent.py:48-94   (pinned by tests/golden/gae_*.npz,
 *                    produced from the reference's own numpy code)
 *   - n-step returns xagents/a2c/agent.py:141-171 (pinned by tests/golden/nstep_*.npz)
 *   - actor-critic forward + Categorical sample/log_prob/entropy
 *                    xagents/a2c/agent.py:50-94, xagents/base.py:492-511 (TF/TFP math,
 *                    parity unpinned at the TF boundary: no TF in this image)
 *   - rollout + step_envs bookkeeping
 *                    xagents/a2c/agent.py:96-139, xagents/base.py:388-426
 *   - tf.clip_by_global_norm + Keras Adam
 *                    xagents/ppo/agent.py:135-137, xagents/utils/common.py:476
 * and the deterministic f32 math helpers the kernels define
 * (xagents_amd/csrc/xa_common.hpp), restated independently here.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define H 64

static inline float as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline uint32_t as_uint(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

/* ---------------- deterministic f32 math (same op sequence as the kernels) ---------------- */
float xo_expf(float x) {
  if (x != x) return x;
  if (x > 88.72283935546875f) return INFINITY;
  if (x < -103.97208404541015625f) return 0.0f;
  float n = rintf(x * 1.44269502162933349609375f);
  float r = fmaf(n, -0.693145751953125f, x);
  r = fmaf(n, -1.428606765330187045e-06f, r);
  float p = 1.98412698e-4f;
  p = fmaf(p, r, 1.38888889e-3f);
  p = fmaf(p, r, 8.33333333e-3f);
  p = fmaf(p, r, 4.16666667e-2f);
  p = fmaf(p, r, 1.66666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  int ni = (int)n;
  int n1 = ni / 2;
  int n2 = ni - n1;
  float s1 = as_float((uint32_t)(n1 + 127) << 23);
  float s2 = as_float((uint32_t)(n2 + 127) << 23);
  return (p * s1) * s2;
}

float xo_logf(float x) {
  if (x != x) return x;
  if (x < 0.0f) return NAN;
  if (x == 0.0f) return -INFINITY;
  if (x == INFINITY) return x;
  int k = 0;
  uint32_t hx = as_uint(x);
  if (hx < 0x00800000u) {
    x = x * 33554432.0f;
    hx = as_uint(x);
    k = -25;
  }
  k += (int)((hx >> 23) & 0xffu) - 127;
  hx &= 0x007fffffu;
  uint32_t i = (hx + (0x95f64u << 3)) & 0x800000u;
  float m = as_float(hx | (i ^ 0x3f800000u));
  k += (int)(i >> 23);
  float f = m - 1.0f;
  float s = f / (2.0f + f);
  float z = s * s;
  float w = z * z;
  float t1 = w * (4.0000972152e-01f + w * 2.4279078841e-01f);
  float t2 = z * (6.6666662693e-01f + w * 2.8498786688e-01f);
  float R = t2 + t1;
  float hfsq = (0.5f * f) * f;
  float dk = (float)k;
  return dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
}

/* odd rational minimax tanh on the input clamped to +-7.905311 */
float xo_tanhf(float x) {
  const float c = 7.90531110763549805f;
  float xc = fminf(fmaxf(x, -c), c);
  float x2 = xc * xc;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  p = xc * p;
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  /* the quotient as the kernels form it: bit-trick seed, two Newton steps, one residual
     correction (xa_common.hpp xa_tanhf) */
  int32_t qi;
  memcpy(&qi, &q, 4);
  qi = 0x7EF311C3 - qi;
  float r;
  memcpy(&r, &qi, 4);
  r = fmaf(r, fmaf(-q, r, 1.0f), r);
  r = fmaf(r, fmaf(-q, r, 1.0f), r);
  float t = p * r;
  return fmaf(r, fmaf(-q, t, p), t);
}

/* b^t by binary exponentiation in f64 (the kernels' xa_powi) */
static double powi(double b, int t) {
  double r = 1.0;
  while (t > 0) {
    if (t & 1) r *= b;
    b *= b;
    t >>= 1;
  }
  return r;
}

void xo_expf_arr(const float* x, float* y, int n) {
  for (int i = 0; i < n; ++i) y[i] = xo_expf(x[i]);
}
void xo_logf_arr(const float* x, float* y, int n) {
  for (int i = 0; i < n; ++i) y[i] = xo_logf(x[i]);
}
void xo_tanhf_arr(const float* x, float* y, int n) {
  for (int i = 0; i < n; ++i) y[i] = xo_tanhf(x[i]);
}

/* ---------------- Philox4x32-10 + Feistel permutation ---------------- */
static inline uint32_t mulhi(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

void xo_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
               uint32_t* out) {
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = mulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

static inline float u01(uint32_t v) { return (float)(v >> 8) * 5.9604644775390625e-08f; }

static uint32_t feistel_round(uint32_t v, uint32_t key, uint32_t mask) {
  uint32_t h = v * 0x9E3779B1u ^ key;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & mask;
}

/* device shuffle: Feistel permutation of [0, n) keyed per epoch (replaces
 * tf.random.shuffle, xagents/ppo/agent.py:149-154) */
void xo_shuffle_perm(int n, int epoch, uint64_t seed, uint64_t ctr, int* out) {
  uint32_t k[4];
  xo_philox((uint32_t)epoch, 0x5u, (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)seed,
            (uint32_t)(seed >> 32), k);
  uint32_t bits = 1;
  if (n > 1) {
    bits = 0;
    uint32_t v = (uint32_t)(n - 1);
    while (v) {
      bits++;
      v >>= 1;
    }
  }
  uint32_t hb = (bits + 1) / 2;
  if (hb == 0) hb = 1;
  uint32_t mask = (1u << hb) - 1u;
  for (int i = 0; i < n; ++i) {
    uint32_t v = (uint32_t)i;
    do {
      uint32_t l = v >> hb, r = v & mask, t;
      for (int q = 0; q < 4; ++q) {
        l ^= feistel_round(r, k[q], mask);
        t = l;
        l = r;
        r = t;
      }
      v = (l << hb) | r;
    } while (v >= (uint32_t)n);
    out[i] = (int)v;
  }
}

/* ---------------- actor-critic MLP forward (a2c/agent.py:65-94) ---------------- */
typedef struct {
  int w1, b1, w2, b2, w3, b3, w4, b4, P;
} offs_t;

static offs_t offsets(int obs, int A) {
  offs_t o;
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

/* wave64 butterfly sum: x_j <- x_j + x_{j^m}, m = 1..32 */
static float butterfly(float* v) {
  float t[H];
  for (int m = 1; m < H; m <<= 1) {
    for (int j = 0; j < H; ++j) t[j] = v[j] + v[j ^ m];
    memcpy(v, t, sizeof(t));
  }
  return v[0];
}

static void mlp_forward1(const float* th, int obs, int A, const float* x, float* logits,
                         float* value) {
  offs_t o = offsets(obs, A);
  float h1[H], h2[H], prod[H];
  for (int j = 0; j < H; ++j) {
    float z = 0.0f;
    for (int k = 0; k < obs; ++k) z = fmaf(x[k], th[o.w1 + k * H + j], z);
    h1[j] = xo_tanhf(z + th[o.b1 + j]);
  }
  for (int j = 0; j < H; ++j) {
    /* 8 chains, chain r over k = r (mod 8) (mlp_rollout.hip LaneMlp::layer2) */
    float c[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < H; i += 8)
      for (int r = 0; r < 8; ++r) c[r] = fmaf(h1[i + r], th[o.w2 + (i + r) * H + j], c[r]);
    h2[j] = xo_tanhf((((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]))) +
                     th[o.b2 + j]);
  }
  for (int a = 0; a < A; ++a) {
    for (int j = 0; j < H; ++j) prod[j] = h2[j] * th[o.w3 + j * A + a];
    logits[a] = butterfly(prod) + th[o.b3 + a];
  }
  for (int j = 0; j < H; ++j) prod[j] = h2[j] * th[o.w4 + j];
  *value = butterfly(prod) + th[o.b4];
}

/* TFP Categorical(logits): log_prob, entropy; inverse-CDF sample on u */
static void categorical(const float* l, int A, float u, int given, int* act_out, float* logp_out,
                        float* ent_out) {
  float m = l[0];
  for (int a = 1; a < A; ++a) m = fmaxf(m, l[a]);
  float e[16], s = 0.0f;
  for (int a = 0; a < A; ++a) {
    e[a] = xo_expf(l[a] - m);
    s = s + e[a];
  }
  float ls = xo_logf(s);
  int act = given;
  if (act < 0) {
    float target = u * s, c = 0.0f;
    act = A - 1;
    for (int a = 0; a < A; ++a) {
      c = c + e[a];
      if (target < c) {
        act = a;
        break;
      }
    }
  }
  float ent = 0.0f, logp = 0.0f;
  float inv_s = 1.0f / s;
  for (int a = 0; a < A; ++a) {
    float lp = (l[a] - m) - ls;
    float p = e[a] * inv_s;
    ent = ent - p * lp;
    if (a == act) logp = lp;
  }
  *act_out = act;
  *logp_out = logp;
  *ent_out = ent;
}

int xo_mlp_param_count(int obs, int A) { return offsets(obs, A).P; }

void xo_mlp_forward(const float* th, const float* obs, int B, int obs_dim, int A,
                    const int* actions_in, const float* uniforms, int* actions_out, float* logp,
                    float* value, float* entropy, float* logits) {
  for (int b = 0; b < B; ++b) {
    float l[16], v, lp, ent;
    int act;
    mlp_forward1(th, obs_dim, A, obs + (size_t)b * obs_dim, l, &v);
    categorical(l, A, uniforms ? uniforms[b] : 0.0f, actions_in ? actions_in[b] : -1, &act, &lp,
                &ent);
    if (actions_out) actions_out[b] = act;
    if (logp) logp[b] = lp;
    if (value) value[b] = v;
    if (entropy) entropy[b] = ent;
    if (logits)
      for (int a = 0; a < A; ++a) logits[(size_t)b * A + a] = l[a];
  }
}

/* ---------------- returns (ppo/agent.py:84-94, a2c/agent.py:165-171) ---------------- */
void xo_gae(const float* rew, const float* val, const float* done, const float* nv, float* ret,
            int N, int T, float gamma, float gamma_lam) {
  for (int n = 0; n < N; ++n) {
    float carry = 0.0f, vn = nv[n];
    for (int t = T - 1; t >= 0; --t) {
      float nnt = 1.0f - done[(size_t)n * (T + 1) + t + 1];
      float vt = val[(size_t)n * T + t];
      float delta = (rew[(size_t)n * T + t] + (gamma * vn) * nnt) - vt;
      carry = delta + ((gamma_lam * nnt) * carry);
      ret[(size_t)n * T + t] = carry + vt;
      vn = vt;
    }
  }
}

void xo_nstep(const float* rew, const float* done, const float* nv, float* ret, int N, int T,
              float gamma) {
  for (int n = 0; n < N; ++n) {
    float carry = nv[n];
    for (int t = T - 1; t >= 0; --t) {
      float nnt = 1.0f - done[(size_t)n * (T + 1) + t + 1];
      carry = rew[(size_t)n * T + t] + (gamma * carry) * nnt;
      ret[(size_t)n * T + t] = carry;
    }
  }
}

/* ---------------- rollout (a2c/agent.py:96-139 + base.py:388-426) ---------------- */
static int cartpole_step(double* s, int action) {
  const double gravity = 9.8, masspole = 0.1, total_mass = 1.1, length = 0.5;
  const double polemass_length = 0.05, force_mag = 10.0, tau = 0.02;
  double force = action == 1 ? force_mag : -force_mag;
  double costheta = cos(s[2]), sintheta = sin(s[2]);
  double temp = (force + polemass_length * s[3] * s[3] * sintheta) / total_mass;
  double thetaacc = (gravity * sintheta - costheta * temp) /
                    (length * (4.0 / 3.0 - masspole * costheta * costheta / total_mass));
  double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
  s[0] = s[0] + tau * s[1];
  s[1] = s[1] + tau * xacc;
  s[2] = s[2] + tau * s[3];
  s[3] = s[3] + tau * thetaacc;
  double thr = 12.0 * 2.0 * 3.141592653589793 / 360.0;
  return s[0] < -2.4 || s[0] > 2.4 || s[2] < -thr || s[2] > thr;
}

/* Mirrors XaRolloutArgs field-for-field (plain arguments here). env_kind 0 = replay,
 * 1 = cartpole; return_kind 0 none / 1 GAE / 2 n-step. */
void xo_mlp_rollout(int N, int T, int obs, int A, const float* th, int env_kind, float* env_state,
                    double* env_state64, float* env_done, int* env_cursor, float* ep_return,
                    const float* rep_obs, const float* rep_state, const float* rep_rew,
                    const float* rep_done, int t_rec, int max_ep, const float* uniforms,
                    uint64_t seed, uint64_t ctr, float* obs_out, int* act_out, float* logp_out,
                    float* val_out, float* ent_out, float* rew_out, float* done_out,
                    float* epret_out, float* next_val, float* ret_out, int return_kind,
                    float gamma, float gamma_lam) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int n = 0; n < N; ++n) {
    float x[16], st[16];
    double cp[4] = {0, 0, 0, 0};
    for (int k = 0; k < obs; ++k) st[k] = x[k] = env_state[(size_t)n * obs + k];
    if (env_kind == 1)
      for (int k = 0; k < 4; ++k) cp[k] = env_state64[(size_t)n * 4 + k];
    int cur = env_cursor[n];
    float ep = ep_return[n];
    float d_last = env_done[n];
    done_out[(size_t)n * (T + 1)] = d_last;
    for (int t = 0; t < T; ++t) {
      size_t it = (size_t)n * T + t;
      float l[16], v, lp, ent, u;
      int act;
      mlp_forward1(th, obs, A, x, l, &v);
      if (uniforms) {
        u = uniforms[it];
      } else {
        uint32_t r4[4];
        xo_philox((uint32_t)n, (uint32_t)t, (uint32_t)ctr, (uint32_t)(ctr >> 32), k0, k1, r4);
        u = u01(r4[0]);
      }
      categorical(l, A, u, -1, &act, &lp, &ent);
      for (int k = 0; k < obs; ++k) obs_out[it * obs + k] = x[k];
      float r, d, o_obs[16];
      if (env_kind == 0) {
        size_t base = (size_t)n * t_rec + cur;
        r = rep_rew[base];
        d = rep_done[base];
        for (int k = 0; k < obs; ++k) {
          o_obs[k] = rep_obs[base * obs + k];
          st[k] = rep_state[base * obs + k];
        }
        cur = cur + 1;
        if (cur >= t_rec) cur = 0;
      } else {
        int done = cartpole_step(cp, act);
        cur = cur + 1;
        if (cur >= max_ep) done = 1;
        r = 1.0f;
        d = done ? 1.0f : 0.0f;
        for (int k = 0; k < 4; ++k) o_obs[k] = (float)cp[k];
        if (done) {
          uint32_t rr[4];
          xo_philox((uint32_t)n, (uint32_t)t, (uint32_t)ctr, (uint32_t)(ctr >> 32) ^ 0x5eed5eedu,
                    k0, k1, rr);
          for (int k = 0; k < 4; ++k) cp[k] = -0.05 + 0.1 * ((double)rr[k] * 2.3283064365386963e-10);
          cur = 0;
        }
        for (int k = 0; k < 4; ++k) st[k] = (float)cp[k];
      }
      ep = ep + r;
      act_out[it] = act;
      logp_out[it] = lp;
      val_out[it] = v;
      if (ent_out) ent_out[it] = ent;
      rew_out[it] = r;
      done_out[(size_t)n * (T + 1) + t + 1] = d;
      if (epret_out) epret_out[it] = ep;
      if (d != 0.0f) ep = 0.0f;
      d_last = d;
      for (int k = 0; k < obs; ++k) x[k] = o_obs[k];
    }
    float l[16], vnext;
    mlp_forward1(th, obs, A, st, l, &vnext);
    for (int k = 0; k < obs; ++k) env_state[(size_t)n * obs + k] = st[k];
    if (env_kind == 1)
      for (int k = 0; k < 4; ++k) env_state64[(size_t)n * 4 + k] = cp[k];
    env_cursor[n] = cur;
    ep_return[n] = ep;
    env_done[n] = d_last;
    next_val[n] = vnext;
  }
  if (ret_out && return_kind == 1) xo_gae(rew_out, val_out, done_out, next_val, ret_out, N, T, gamma, gamma_lam);
  if (ret_out && return_kind == 2) xo_nstep(rew_out, done_out, next_val, ret_out, N, T, gamma);
}

/* ---------------- clip_by_global_norm + Keras Adam (training_ops ApplyAdam) ---------------- */
void xo_clip_adam(float* theta, float* m, float* v, const float* g, int P, float grad_scale,
                  float clip, float lr, float b1, float b2, float eps, int t, float* gnorm_out) {
  double total = 0.0;
  for (int i = 0; i < P; ++i) {
    float x = g[i] * grad_scale;
    total += (double)x * (double)x;
  }
  float gn = (float)sqrt(total);
  float sc = 1.0f;
  if (clip > 0.0f) sc = clip * fminf(1.0f / gn, 1.0f / clip);
  if (gnorm_out) *gnorm_out = gn;
  float b1p = (float)powi((double)b1, t);
  float b2p = (float)powi((double)b2, t);
  float alpha = lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
  float omb1 = 1.0f - b1, omb2 = 1.0f - b2;
  for (int i = 0; i < P; ++i) {
    float gg = (g[i] * grad_scale) * sc;
    float mm = m[i] + (gg - m[i]) * omb1;
    float vv = v[i] + (gg * gg - v[i]) * omb2;
    m[i] = mm;
    v[i] = vv;
    theta[i] = theta[i] - (mm * alpha) / (sqrtf(vv) + eps);
  }
}

/* ---- BipedalWalker-v3 device stand-in (xagents_amd/csrc/walker.hip) ----------------
 * The f32 restatement of walker_step_kernel, operation for operation (explicit fmaf, the
 * same sin / cos polynomials, the same Philox reset draw). The stand-in replaces gym's
 * BipedalWalker inside BaseAgent.step_envs (xagents/base.py:388-426); gym / Box2D are
 * absent, so its dynamics are parity-unpinned -- this pins the device kernel to its own
 * CPU statement. */
#define WK_STATE 18
#define WK_OBS 24
enum { WS_X, WS_Y, WS_TH, WS_VX, WS_VY, WS_W, WS_Q, WS_DQ = WS_Q + 4, WS_SHAPE = WS_DQ + 4,
       WS_STEPS, WS_FX0, WS_FX1 };
static const float wk_scale = 30.0f, wk_fps = 50.0f, wk_dt = 1.0f / 50.0f;
static const float wk_torque = 80.0f, wk_speed_hip = 4.0f, wk_speed_knee = 6.0f;
static const float wk_leg_h = 34.0f / 30.0f, wk_hip_dy = 0.2f, wk_hull_half_h = 0.25f;
static const float wk_lidar_range = 160.0f / 30.0f;
static const float wk_gravity = 10.0f, wk_gain = 40.0f, wk_jdamp = 2.0f;
static const float wk_react = 2.0f, wk_restore = 3.0f, wk_pdamp = 1.0f, wk_drag = 0.5f;
static const float wk_terrain_end = (200.0f - 10.0f) * (14.0f / 30.0f);
static const float wk_start_x = 20.0f * (14.0f / 30.0f) * 0.5f;
static const float wk_lidar_cos[10] = {1.0f,        0.98877108f, 0.95533649f, 0.90044710f,
                                       0.82533561f, 0.73168887f, 0.62160997f, 0.49757105f,
                                       0.36235775f, 0.21901920f};
static const float wk_hip_lo = -0.8f, wk_hip_hi = 1.1f, wk_knee_lo = -1.6f, wk_knee_hi = -0.1f;

static float wk_reduce(float x) {
  const float k = rintf(x * 0.159154943f);
  return fmaf(-k, 6.28318548f, x);
}
static float wk_sin(float x) {
  const float r = wk_reduce(x), r2 = r * r;
  float p = fmaf(r2, -7.6471637e-13f, 1.6059044e-10f);
  p = fmaf(r2, p, -2.5052108e-08f);
  p = fmaf(r2, p, 2.7557319e-06f);
  p = fmaf(r2, p, -1.9841270e-04f);
  p = fmaf(r2, p, 8.3333333e-03f);
  p = fmaf(r2, p, -1.6666667e-01f);
  p = fmaf(r2, p, 1.0f);
  return r * p;
}
static float wk_cos(float x) {
  const float r = wk_reduce(x), r2 = r * r;
  float p = fmaf(r2, 4.7794773e-14f, -1.1470746e-11f);
  p = fmaf(r2, p, 2.0876757e-09f);
  p = fmaf(r2, p, -2.7557319e-07f);
  p = fmaf(r2, p, 2.4801587e-05f);
  p = fmaf(r2, p, -1.3888889e-03f);
  p = fmaf(r2, p, 4.1666667e-02f);
  p = fmaf(r2, p, -0.5f);
  return fmaf(r2, p, 1.0f);
}
static float wk_clip(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

static void wk_feet(const float* s, float* fx, float* fy) {
  for (int j = 0; j < 2; ++j) {
    const float a1 = s[WS_TH] + s[WS_Q + 2 * j];
    const float a2 = a1 + s[WS_Q + 2 * j + 1];
    fx[j] = fmaf(wk_leg_h, wk_sin(a1), wk_leg_h * wk_sin(a2));
    fy[j] = (-wk_hip_dy - wk_leg_h * wk_cos(a1)) - wk_leg_h * wk_cos(a2);
  }
}

static void wk_observe(const float* s, const float* contact, float* o) {
  o[0] = s[WS_TH];
  o[1] = 2.0f * s[WS_W] / wk_fps;
  o[2] = 0.3f * s[WS_VX] * (600.0f / wk_scale) / wk_fps;
  o[3] = 0.3f * s[WS_VY] * (400.0f / wk_scale) / wk_fps;
  for (int j = 0; j < 2; ++j) {
    o[4 + 5 * j] = s[WS_Q + 2 * j];
    o[5 + 5 * j] = s[WS_DQ + 2 * j] / wk_speed_hip;
    o[6 + 5 * j] = s[WS_Q + 2 * j + 1] + 1.0f;
    o[7 + 5 * j] = s[WS_DQ + 2 * j + 1] / wk_speed_knee;
    o[8 + 5 * j] = contact[j];
  }
  for (int i = 0; i < 10; ++i)
    o[14 + i] = fminf(1.0f, s[WS_Y] / (wk_lidar_range * wk_lidar_cos[i]));
}

static void wk_reset(float* s, int env, int episode, uint64_t seed, float* contact) {
  uint32_t r[4];
  xo_philox((uint32_t)env, (uint32_t)episode, 0x3a1cu, 0u, (uint32_t)seed,
            (uint32_t)(seed >> 32), r);
  for (int k = 0; k < WK_STATE; ++k) s[k] = 0.0f;
  s[WS_X] = wk_start_x;
  s[WS_VX] = (u01(r[0]) * 2.0f - 1.0f) * 0.2f;
  s[WS_Q + 1] = wk_knee_hi;
  s[WS_Q + 3] = wk_knee_hi;
  float fx[2], fy[2];
  wk_feet(s, fx, fy);
  s[WS_Y] = -fminf(fy[0], fy[1]);
  s[WS_FX0] = fx[0];
  s[WS_FX1] = fx[1];
  s[WS_SHAPE] = 130.0f * s[WS_X] / wk_scale;
  contact[0] = contact[1] = 1.0f;
}

void xo_walker_step(int n_envs, float* state, int* episode, const float* actions, long act_ld,
                    uint64_t seed, int reset_only, float* out_obs, float* out_post,
                    float* out_rew, float* out_done) {
  for (int e = 0; e < n_envs; ++e) {
    float* s = state + (size_t)e * WK_STATE;
    float contact[2];
    if (reset_only) {
      wk_reset(s, e, episode[e], seed, contact);
      wk_observe(s, contact, out_post + (size_t)e * WK_OBS);
      continue;
    }
    const float* act = actions + (size_t)e * act_ld;
    float u[4], cost = 0.0f;
    for (int i = 0; i < 4; ++i) {
      u[i] = wk_clip(act[i], -1.0f, 1.0f);
      cost = cost + fabsf(u[i]);
    }
    for (int i = 0; i < 4; ++i) {
      const int hip = (i & 1) == 0;
      const float vmax = hip ? wk_speed_hip : wk_speed_knee;
      float dq = s[WS_DQ + i];
      dq = dq + wk_dt * fmaf(wk_gain, u[i], -wk_jdamp * dq);
      dq = wk_clip(dq, -vmax, vmax);
      float q = fmaf(wk_dt, dq, s[WS_Q + i]);
      const float lo = hip ? wk_hip_lo : wk_knee_lo, hi = hip ? wk_hip_hi : wk_knee_hi;
      if (q < lo || q > hi) dq = 0.0f;
      s[WS_Q + i] = wk_clip(q, lo, hi);
      s[WS_DQ + i] = dq;
    }
    s[WS_W] = s[WS_W] +
              wk_dt * ((-wk_react * (u[0] + u[2]) - wk_restore * s[WS_TH]) - wk_pdamp * s[WS_W]);
    s[WS_TH] = fmaf(wk_dt, s[WS_W], s[WS_TH]);
    float fx[2], fy[2];
    wk_feet(s, fx, fy);
    const float support = -fminf(fy[0], fy[1]);
    s[WS_VY] = s[WS_VY] - wk_gravity * wk_dt;
    float y = fmaf(wk_dt, s[WS_VY], s[WS_Y]);
    int grounded = 0;
    if (y <= support) {
      y = support;
      s[WS_VY] = fmaxf(s[WS_VY], 0.0f);
      grounded = 1;
    }
    s[WS_Y] = y;
    float push = 0.0f, n_st = 0.0f;
    for (int j = 0; j < 2; ++j) {
      contact[j] = grounded && fy[j] <= fminf(fy[0], fy[1]) + 0.02f ? 1.0f : 0.0f;
      if (contact[j] > 0.0f) {
        push = push - (fx[j] - s[WS_FX0 + j]);
        n_st = n_st + 1.0f;
      }
    }
    s[WS_VX] = n_st > 0.0f ? push / (n_st * wk_dt) : s[WS_VX] * (1.0f - wk_drag * wk_dt);
    s[WS_X] = fmaf(wk_dt, s[WS_VX], s[WS_X]);
    s[WS_FX0] = fx[0];
    s[WS_FX1] = fx[1];
    s[WS_STEPS] = s[WS_STEPS] + 1.0f;
    const float shaping = 130.0f * s[WS_X] / wk_scale - 5.0f * fabsf(s[WS_TH]);
    float reward = shaping - s[WS_SHAPE];
    s[WS_SHAPE] = shaping;
    reward = reward - 0.00035f * wk_torque * cost;
    const int game_over = s[WS_Y] - wk_hull_half_h < 0.0f || fabsf(s[WS_TH]) > 1.0f;
    int done = 0;
    if (game_over || s[WS_X] < 0.0f) {
      reward = -100.0f;
      done = 1;
    }
    if (s[WS_X] > wk_terrain_end || s[WS_STEPS] >= 1600.0f) done = 1;
    wk_observe(s, contact, out_obs + (size_t)e * WK_OBS);
    out_rew[e] = reward;
    out_done[e] = done ? 1.0f : 0.0f;
    if (done) {
      episode[e] = episode[e] + 1;
      wk_reset(s, e, episode[e], seed, contact);
    }
    wk_observe(s, contact, out_post + (size_t)e * WK_OBS);
  }
}
