// Fused vectorized rollout for the actor-critic MLP (obs -> 64 tanh -> 64 tanh ->
// {A logits, 1 value}) -- replaces A2C.get_batch (xagents/a2c/agent.py:96-139),
// A2C.get_model_outputs (a2c/agent.py:65-94), BaseAgent.step_envs
// (xagents/base.py:388-426) and the return computation (ppo/agent.py:48-94,
// a2c/agent.py:141-171).
//
// Two schedules. The replay env (records that ignore the actions) runs every step's
// forward as an independent row of one batched forward (replay_rollout_kernel, below).
// The CartPole-dynamics env, whose next input depends on the sampled action, runs the
// step loop (mlp_rollout_kernel): ONE wave64 per env, lane j = hidden unit j. Each lane
// keeps the weights it needs for the whole rollout in VGPRs (column j of W1 and W2, row j
// of the heads: ~75 registers). Per step:
//   h1_j = tanh(sum_k x_k W1[k][j] + b1_j)              (fma chain over k)
//   h1 -> LDS (wave-private row), 16 x ds_read_b128 broadcast back
//   h2_j = tanh(sum of 8 interleaved 8-long fma chains + b2_j)
//   h2 -> the wave's LDS row of this step (a [64 steps][64 units] chunk buffer)
//   logit_a = butterfly_sum_j(h2_j * W3[j][a]) + b3_a (the sample needs them)
//   inverse-CDF sample, then the f64 CartPole dynamics
// and once per 64-step chunk, lane j on step t0 + j: the value head from the step's h2
// row, summed in the pairwise order of the wave butterfly (bitwise the same sums as
// in-step); softmax, log-prob and entropy. Envs are independent, so no inter-wave
// synchronisation exists anywhere.
// The arithmetic order above is restated exactly by oracle/xa_oracle.c.
#include "../../include/xagents_hip.h"
#include "xa_common.hpp"

namespace {

constexpr int H = XA_MLP_HIDDEN;
constexpr int kWaves = 4;       // xa_mlp_forward: waves (samples in flight) per workgroup
// xa_mlp_rollout: env waves per workgroup. The waves never synchronise; one per workgroup
// puts every env's wave on a CU of its own, measured fastest (16-env rollout 57.8 us at 4
// waves, 54.9 at 2, 52.3 at 1: profiles/r03y_variants.txt)
#ifndef XA_ROLLOUT_WAVES
#define XA_ROLLOUT_WAVES 1
#endif
constexpr int kRollWaves = XA_ROLLOUT_WAVES;
constexpr int kFusedMaxT = 1024;
constexpr int kChunk = 64;     // steps per chunk (one per lane in the chunk pass)
constexpr int kHS = H + 4;     // h2 chunk-buffer row stride (floats): conflict-free row reads

XA_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct ParamOffsets {
  int w1, b1, w2, b2, w3, b3, w4, b4;
};

__host__ __device__ inline ParamOffsets param_offsets(int obs, int A) {
  ParamOffsets o;
  o.w1 = 0;
  o.b1 = o.w1 + obs * H;
  o.w2 = o.b1 + H;
  o.b2 = o.w2 + H * H;
  o.w3 = o.b2 + H;
  o.b3 = o.w3 + H * A;
  o.w4 = o.b3 + A;
  o.b4 = o.w4 + H;
  return o;
}

template <int OBS, int A>
struct LaneMlp {
  float w1[OBS];
  float b1;
  float w2[H];
  float b2;
  float w3[A];
  float w4;
  float b3[A];
  float b4;

  XA_DEV void load(const float* __restrict__ theta, int lane) {
    const ParamOffsets o = param_offsets(OBS, A);
#pragma unroll
    for (int k = 0; k < OBS; ++k) w1[k] = theta[o.w1 + k * H + lane];
    b1 = theta[o.b1 + lane];
#pragma unroll
    for (int k = 0; k < H; ++k) w2[k] = theta[o.w2 + k * H + lane];
    b2 = theta[o.b2 + lane];
#pragma unroll
    for (int a = 0; a < A; ++a) {
      w3[a] = theta[o.w3 + lane * A + a];
      b3[a] = theta[o.b3 + a];
    }
    w4 = theta[o.w4 + lane];
    b4 = theta[o.b4];
  }

  // x: wave-uniform observation. sh: this wave's 64-float LDS row.
  // layer 1 and the h1 broadcast through this wave's LDS row (16 x ds_read_b128)
  XA_DEV void layer1(const float (&x)[OBS], float* sh, int lane, float4 (&hv)[H / 4]) const {
    float z1 = 0.0f;
#pragma unroll
    for (int k = 0; k < OBS; ++k) z1 = fmaf(x[k], w1[k], z1);
    const float h1 = xa_tanhf(z1 + b1);
    sh[lane] = h1;
    wave_sync();
#pragma unroll
    for (int k = 0; k < H / 4; ++k) hv[k] = reinterpret_cast<const float4*>(sh)[k];
    wave_sync();  // the row is rewritten by the next forward
  }

  // 8 interleaved 8-long fma chains, chain r over k = r (mod 8), run as 4 packed
  // (v_pk_fma_f32) chains fed straight from the ds_read_b128 registers
  XA_DEV float layer2(const float4 (&hv)[H / 4]) const {
    xa_f2 c01 = {0.0f, 0.0f}, c23 = c01, c45 = c01, c67 = c01;
#pragma unroll
    for (int m = 0; m < H / 8; ++m) {
      const float4 q0 = hv[2 * m], q1 = hv[2 * m + 1];
      c01 = xa_fma2(xa_f2{q0.x, q0.y}, xa_f2{w2[8 * m + 0], w2[8 * m + 1]}, c01);
      c23 = xa_fma2(xa_f2{q0.z, q0.w}, xa_f2{w2[8 * m + 2], w2[8 * m + 3]}, c23);
      c45 = xa_fma2(xa_f2{q1.x, q1.y}, xa_f2{w2[8 * m + 4], w2[8 * m + 5]}, c45);
      c67 = xa_fma2(xa_f2{q1.z, q1.w}, xa_f2{w2[8 * m + 6], w2[8 * m + 7]}, c67);
    }
    return xa_tanhf((((c01.x + c01.y) + (c23.x + c23.y)) + ((c45.x + c45.y) + (c67.x + c67.y))) +
                    b2);
  }

  XA_DEV void heads(float h2, float (&logits)[A], float& value) const {
#pragma unroll
    for (int a = 0; a < A; ++a) logits[a] = xa_wave_sum(h2 * w3[a]) + b3[a];
    value = xa_wave_sum(h2 * w4) + b4;
  }

  // x: wave-uniform observation. sh: this wave's 64-float LDS row.
  XA_DEV void forward(const float (&x)[OBS], float* sh, int lane, float (&logits)[A],
                      float& value) const {
    float4 hv[H / 4];
    layer1(x, sh, lane, hv);
    heads(layer2(hv), logits, value);
  }
};

// Heads HF .. A of the chunk pass (HF = 0: logits and value; HF = A: the value only) for
// the step whose h2 row this lane reads: head a = sum_j h2_j W34[j][a] with the products
// rounded and summed as pairs, quads, octets, 16-unit rows, then (S2 + S3) + (S0 + S1) --
// the tree xa_wave_sum's butterfly builds in lane 63, so every head equals its in-step
// value bit for bit. wt: the wave's [H][AHP] table of (W3[j][0 .. A), w4[j], pad).
template <int A, int HF, int UNROLL = 1>
XA_DEV void chunk_heads(const float* __restrict__ hrow, const float* __restrict__ wt,
                        float (&z)[A + 1]) {
  constexpr int AH = A + 1, AHP = (AH + 3) & ~3;
  float s_prev[AH], p01[AH];
  // one 16-unit row per iteration, not unrolled in the step loop (the row's 16 h2 values and
  // table rows are all that is live on top of its state); UNROLL 4 where registers allow
#pragma unroll UNROLL
  for (int r = 0; r < 4; ++r) {
    float O[AH][2];
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      float Q[AH][2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int j0 = 16 * r + 8 * o + 4 * q;
        const float4 h4 = *reinterpret_cast<const float4*>(hrow + j0);
        const float hj[4] = {h4.x, h4.y, h4.z, h4.w};
        float v[AH][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float wr[AHP];
#pragma unroll
          for (int a4 = 0; a4 < AHP; a4 += 4) {
            const float4 t = *reinterpret_cast<const float4*>(wt + (j0 + u) * AHP + a4);
            wr[a4] = t.x; wr[a4 + 1] = t.y; wr[a4 + 2] = t.z; wr[a4 + 3] = t.w;
          }
#pragma unroll
          for (int a = HF; a < AH; ++a) v[a][u] = hj[u] * wr[a];
        }
#pragma unroll
        for (int a = HF; a < AH; ++a) Q[a][q] = (v[a][0] + v[a][1]) + (v[a][2] + v[a][3]);
      }
#pragma unroll
      for (int a = HF; a < AH; ++a) O[a][o] = Q[a][0] + Q[a][1];
    }
#pragma unroll
    for (int a = HF; a < AH; ++a) {
      const float S = O[a][0] + O[a][1];  // row r's sum
      if (r & 1) {
        const float pr = s_prev[a] + S;
        if (r == 1) p01[a] = pr;
        else z[a] = pr + p01[a];  // (S2 + S3) + (S0 + S1)
      } else {
        s_prev[a] = S;
      }
    }
  }
}

// Categorical over logits (TFP Categorical(logits=...), a2c/agent.py:59-94):
// log_prob(a) = (l_a - m) - log(sum_k e^{l_k - m}); entropy = -sum p_k log p_k.
template <int A>
struct CatOut {
  int action;
  float logp, entropy;
};

// max, shifted exponentials and their sum: the part both the sample and the
// log-prob / entropy need (the same operations in both, so a sample drawn on the
// step's critical path and a log-prob computed later agree bit for bit)
template <int A>
XA_DEV float cat_exp(const float (&l)[A], float (&e)[A], float& s) {
  float m = l[0];
#pragma unroll
  for (int a = 1; a < A; ++a) m = fmaxf(m, l[a]);
  s = 0.0f;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    e[a] = xa_expf(l[a] - m);
    s = s + e[a];
  }
  return m;
}

// inverse-CDF sample: the first a with u * s < e_0 + ... + e_a (A - 1 if none)
template <int A>
XA_DEV int cat_pick(const float (&e)[A], float s, float u) {
  const float target = u * s;
  int act = A - 1;
  float c = 0.0f;
  bool found = false;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    c = c + e[a];
    if (!found && target < c) {
      act = a;
      found = true;
    }
  }
  return act;
}

template <int A>
XA_DEV int cat_sample(const float (&l)[A], float u) {
  float e[A], s;
  cat_exp<A>(l, e, s);
  return cat_pick<A>(e, s, u);
}

template <int A>
XA_DEV CatOut<A> categorical(const float (&l)[A], float u, int given_action) {
  float e[A], s;
  const float m = cat_exp<A>(l, e, s);
  const float ls = xa_logf(s);
  const int act = given_action < 0 ? cat_pick<A>(e, s, u) : given_action;
  float ent = 0.0f, logp = 0.0f;
  const float inv_s = 1.0f / s;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float lp = (l[a] - m) - ls;
    const float p = e[a] * inv_s;
    ent = ent - p * lp;
    if (a == act) logp = lp;
  }
  return CatOut<A>{act, logp, ent};
}

// sin and cos of a pole angle: |x| <= 0.5 rad (always, below the 0.2095-rad termination
// threshold plus one Euler step) by their Taylor series to x^15 / x^16 in Horner form on the
// f64 FMA unit (truncation < 2.3e-17, within an ulp of libm, like any two libms), larger
// angles by the library functions. The library sin / cos carry a branch-free Payne-Hanek
// reduction (~250 f64 instructions) that dominated the per-step dependency chain of the
// dynamics rollout.
XA_DEV void pole_sincos(double x, double& sn, double& cs) {
  if (fabs(x) > 0.5) {
    sn = sin(x);
    cs = cos(x);
    return;
  }
  const double x2 = x * x;
  double ps = 1.0 / 1307674368000.0;               // 1 / 15!
  ps = fma(ps, -x2, 1.0 / 6227020800.0);           // 1 / 13!
  ps = fma(ps, -x2, 1.0 / 39916800.0);             // 1 / 11!
  ps = fma(ps, -x2, 1.0 / 362880.0);               // 1 / 9!
  ps = fma(ps, -x2, 1.0 / 5040.0);                 // 1 / 7!
  ps = fma(ps, -x2, 1.0 / 120.0);                  // 1 / 5!
  ps = fma(ps, -x2, 1.0 / 6.0);                    // 1 / 3!
  sn = fma(-x * x2, ps, x);
  double pc = 1.0 / 20922789888000.0;              // 1 / 16!
  pc = fma(pc, -x2, 1.0 / 87178291200.0);          // 1 / 14!
  pc = fma(pc, -x2, 1.0 / 479001600.0);            // 1 / 12!
  pc = fma(pc, -x2, 1.0 / 3628800.0);              // 1 / 10!
  pc = fma(pc, -x2, 1.0 / 40320.0);                // 1 / 8!
  pc = fma(pc, -x2, 1.0 / 720.0);                  // 1 / 6!
  pc = fma(pc, -x2, 1.0 / 24.0);                   // 1 / 4!
  pc = fma(pc, -x2, 0.5);                          // 1 / 2!
  cs = fma(-x2, pc, 1.0);
}

// gym CartPole-v1 (classic_control/cartpole.py), Euler integration in f64.
XA_DEV bool cartpole_step(double (&s)[4], int action) {
  const double gravity = 9.8, masspole = 0.1, total_mass = 1.1, length = 0.5;
  const double polemass_length = 0.05, force_mag = 10.0, tau = 0.02;
  const double force = action == 1 ? force_mag : -force_mag;
  double sintheta, costheta;
  pole_sincos(s[2], sintheta, costheta);
  const double temp = (force + polemass_length * s[3] * s[3] * sintheta) / total_mass;
  const double thetaacc = (gravity * sintheta - costheta * temp) /
                          (length * (4.0 / 3.0 - masspole * costheta * costheta / total_mass));
  const double xacc = temp - polemass_length * thetaacc * costheta / total_mass;
  s[0] = s[0] + tau * s[1];
  s[1] = s[1] + tau * xacc;
  s[2] = s[2] + tau * s[3];
  s[3] = s[3] + tau * thetaacc;
  const double theta_thr = 12.0 * 2.0 * 3.141592653589793 / 360.0;
  return s[0] < -2.4 || s[0] > 2.4 || s[2] < -theta_thr || s[2] > theta_thr;
}

// The sampling uniforms of 64 consecutive steps, lane j holding step t0 + j, fetched a
// chunk ahead and read back per step with readlane (no memory access on the step chain).
struct StepChunk {
  float u_given, u_philox;  // picked per step: a select here would wait on the load
};

XA_DEV void load_chunk(const XaRolloutArgs& p, int env, int lane, int cur0, int t0, uint64_t ctr,
                       StepChunk& c) {
  const int T = p.n_steps;
  const int tj = t0 + lane;
  // loads are unconditional (indices clamped) so every path issues the same number
  // of them and the waits the compiler places stay exact
  const float* up = p.uniforms ? p.uniforms + (size_t)env * T : p.theta;
  c.u_given = up[p.uniforms ? min(tj, T - 1) : 0];
  const xa_u4 r = xa_philox((uint32_t)env, (uint32_t)tj, (uint32_t)ctr, (uint32_t)(ctr >> 32),
                            (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
  c.u_philox = xa_u01(r.x);
}

XA_DEV float xa_readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// the CartPole-dynamics env (the next input depends on the sampled action)
template <int OBS, int A>
__global__ __launch_bounds__(64 * kRollWaves) void mlp_rollout_kernel(XaRolloutArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int AH = A + 1, AHP = (AH + 3) & ~3;
  constexpr int HF = A;  // first head of the chunk pass: the value
  __shared__ __attribute__((aligned(16))) float hbuf[kRollWaves][kChunk * kHS];
  __shared__ __attribute__((aligned(16))) float wtab[kRollWaves][H * AHP];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int env = blockIdx.x * kRollWaves + wid;
  if (env >= p.n_envs) return;  // wave-uniform (no block barriers below)
  const int T = p.n_steps;
  float* sh = smem + wid * H;
  const bool fused = p.ret_out != nullptr && p.return_kind != XA_RETURNS_NONE;
  // [rew | val | done] per wave when fused
  float* hist = smem + kRollWaves * H + wid * 3 * T;
  float* const hb = hbuf[wid];  // h2 of the chunk's steps, row j = step t0 + j

  XA_STAMP_DECL
  LaneMlp<OBS, A> net;
  net.load(p.theta, lane);
  {  // the chunk pass's head weights, lane j writes row j
    float* wr = wtab[wid] + lane * AHP;
#pragma unroll
    for (int a = 0; a < AHP; ++a) wr[a] = a < A ? net.w3[a] : a == A ? net.w4 : 0.0f;
  }

  const uint64_t ctr = p.rng_counter ? *p.rng_counter : 0ull;

  float x[OBS];  // policy input (wave-uniform)
  float st[OBS]; // post-reset env state
#pragma unroll
  for (int k = 0; k < OBS; ++k) st[k] = x[k] = p.env_state[(size_t)env * OBS + k];
  double cp[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) cp[k] = p.env_state64[(size_t)env * 4 + k];
  const int cur0 = p.env_cursor[env];
  int cur = cur0;
  float ep_ret = p.ep_return[env];
  float d_last = p.env_done[env];
  if (lane == 0) p.done_out[(size_t)env * (T + 1)] = d_last;

  // per-step scalars park in lane (t & 63) and leave as one coalesced store per
  // output after each 64-step chunk (no stores inside the step loop). What the next
  // step does not read -- the value, log-prob and entropy -- is computed once per chunk
  // with lane j on step t0 + j (the same operations as in-step, so bit for bit the same).
  float b_obs[OBS] = {};
  int b_act = 0;
  float b_l[A] = {};
  float b_val = 0.0f, b_rew = 0.0f, b_done = 0.0f, b_epret = 0.0f;

  auto run_chunk = [&](const StepChunk& c, int t0) {
    const int n = min(64, T - t0);
    for (int j = 0; j < n; ++j) {
      XA_STAMP(0);
      float logits[A];
      {
        float4 hv[H / 4];
        net.layer1(x, sh, lane, hv);
        XA_STAMP(1);
        const float h2 = net.layer2(hv);
        XA_STAMP(2);
        hb[j * kHS + lane] = h2;  // the chunk pass's value head
#pragma unroll
        for (int a = 0; a < A; ++a) logits[a] = xa_wave_sum(h2 * net.w3[a]) + net.b3[a];
      }
      XA_STAMP(3);
      const bool mine = lane == j;
      float r, d;
      {
        const float u = p.uniforms ? xa_readlane(c.u_given, j) : xa_readlane(c.u_philox, j);
        const int act = cat_sample<A>(logits, u);
        XA_STAMP(4);
        bool done = cartpole_step(cp, act);
        cur = cur + 1;
        if (cur >= p.max_episode_steps) done = true;  // gym TimeLimit
        r = 1.0f;
        d = done ? 1.0f : 0.0f;
        if (mine) {
#pragma unroll
          for (int k = 0; k < OBS; ++k) b_obs[k] = x[k];
          b_act = act;
          b_rew = r;
          b_done = d;
        }
#pragma unroll
        for (int k = 0; k < OBS; ++k) x[k] = (float)cp[k < 4 ? k : 3];  // pre-reset obs
        if (done) {
          // reset: np_random.uniform(-0.05, 0.05, size=(4,))
          const xa_u4 rr = xa_philox((uint32_t)env, (uint32_t)(t0 + j), (uint32_t)ctr,
                                     (uint32_t)(ctr >> 32) ^ 0x5eed5eedu, (uint32_t)p.seed,
                                     (uint32_t)(p.seed >> 32));
          const uint32_t rv[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            cp[k] = -0.05 + 0.1 * ((double)rv[k] * 2.3283064365386963e-10);
          cur = 0;
        }
      }
      if (mine) {
#pragma unroll
        for (int a = 0; a < A; ++a) b_l[a] = logits[a];
      }
      ep_ret = ep_ret + r;
      if (mine) b_epret = ep_ret;
      if (d != 0.0f) ep_ret = 0.0f;
      d_last = d;
      XA_STAMP(6);
    }
    // chunk pass: lane j finishes step t0 + j
    wave_sync();  // the chunk's h2 rows are in LDS
    {
      float z[AH];
      chunk_heads<A, HF>(hb + lane * kHS, wtab[wid], z);
      b_val = z[A] + net.b4;
    }
    wave_sync();  // the next chunk rewrites the rows
    const float u = p.uniforms ? c.u_given : c.u_philox;
    const CatOut<A> cat = categorical<A>(b_l, u, b_act);
    float o_obs[OBS];
#pragma unroll
    for (int k = 0; k < OBS; ++k) {
      o_obs[k] = b_obs[k];
      st[k] = (float)cp[k < 4 ? k : 3];  // post-reset state
    }
    XA_STAMP(7);
    if (lane < n) {
      const size_t o = (size_t)env * T + t0 + lane;
#pragma unroll
      for (int k = 0; k < OBS; ++k) p.obs_out[o * OBS + k] = o_obs[k];
      p.act_out[o] = cat.action;
      p.logp_out[o] = cat.logp;
      p.val_out[o] = b_val;
      if (p.ent_out) p.ent_out[o] = cat.entropy;
      p.rew_out[o] = b_rew;
      p.done_out[(size_t)env * (T + 1) + 1 + t0 + lane] = b_done;
      if (p.epret_out) p.epret_out[o] = b_epret;
      if (fused) {
        hist[t0 + lane] = b_rew;
        hist[T + t0 + lane] = b_val;
        hist[2 * T + t0 + lane] = b_done;
      }
    }
  };

  // two chunk buffers: the next chunk's loads are in flight while this one runs
  StepChunk ca, cb;
  load_chunk(p, env, lane, cur0, 0, ctr, ca);
  for (int t0 = 0; t0 < T; t0 += 128) {
    load_chunk(p, env, lane, cur0, t0 + 64, ctr, cb);
    run_chunk(ca, t0);
    if (t0 + 64 >= T) break;
    load_chunk(p, env, lane, cur0, t0 + 128, ctr, ca);
    run_chunk(cb, t0 + 64);
  }

  XA_STAMP(5);
  // bootstrap V(get_states()) on the post-reset state (ppo/agent.py:72)
  float logits[A], v_next;
  net.forward(st, sh, lane, logits, v_next);
  if (lane < OBS) p.env_state[(size_t)env * OBS + lane] = st[lane];
  if (lane < 4) p.env_state64[(size_t)env * 4 + lane] = cp[lane];
  if (lane == 0) {
    p.env_cursor[env] = cur;
    p.ep_return[env] = ep_ret;
    p.env_done[env] = d_last;
    p.next_val[env] = v_next;
  }
  wave_sync();  // every lane's chunk of the history is in LDS
  if (fused && lane == 0) {
    const float* hr = hist;
    const float* hv = hist + T;
    const float* hd = hist + 2 * T;
    float* out = p.ret_out + (size_t)env * T;
    if (p.return_kind == XA_RETURNS_GAE) {
      float carry = 0.0f, vn = v_next;
      for (int t = T - 1; t >= 0; --t) {
        const float nnt = 1.0f - hd[t];
        const float vt = hv[t];
        const float delta = (hr[t] + (p.gamma * vn) * nnt) - vt;
        carry = delta + ((p.gamma_lam * nnt) * carry);
        out[t] = carry + vt;
        vn = vt;
      }
    } else {
      float carry = v_next;
      for (int t = T - 1; t >= 0; --t) {
        const float nnt = 1.0f - hd[t];
        carry = hr[t] + (p.gamma * carry) * nnt;
        out[t] = carry;
      }
    }
  }
}

// Batched forward: one wave per sample (a2c/agent.py:65-94).
template <int OBS, int A>
__global__ __launch_bounds__(256) void mlp_forward_kernel(const float* __restrict__ theta,
                                                          const float* __restrict__ obs, int B,
                                                          const int* __restrict__ actions_in,
                                                          const float* __restrict__ uniforms,
                                                          int* actions_out, float* logp,
                                                          float* value, float* entropy,
                                                          float* logits_out) {
  __shared__ __attribute__((aligned(16))) float smem[kWaves * H];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  LaneMlp<OBS, A> net;
  net.load(theta, lane);
  for (int b = blockIdx.x * kWaves + wid; b < B; b += gridDim.x * kWaves) {
    float x[OBS];
#pragma unroll
    for (int k = 0; k < OBS; ++k) x[k] = obs[(size_t)b * OBS + k];
    float l[A], v;
    net.forward(x, smem + wid * H, lane, l, v);
    const int given = actions_in ? actions_in[b] : -1;
    const float u = (given < 0 && uniforms) ? uniforms[b] : 0.0f;
    const CatOut<A> c = categorical<A>(l, u, given);
    if (lane == 0) {
      if (actions_out) actions_out[b] = c.action;
      if (logp) logp[b] = c.logp;
      if (value) value[b] = v;
      if (entropy) entropy[b] = c.entropy;
    }
    if (logits_out && lane < A) {
#pragma unroll
      for (int a = 0; a < A; ++a)
        if (lane == a) logits_out[(size_t)b * A + a] = l[a];
    }
  }
}

// ---- replay env: every step's policy input is known before the rollout starts ----------
// The record stream ignores the actions, so step t's input is fixed in advance: the env
// state for t = 0 and the record obs of step t - 1 after that; the bootstrap
// V(get_states()) of ppo/agent.py:72 takes the post-reset record state of step T - 1. All
// T forwards are therefore independent rows of one batched forward: 16-row tiles, one per
// tile wave, W2 on v_mfma_f32_16x16x4f32 (an exact k-ordered fmaf chain), one accumulator
// per interleaved chain r (k = r (mod 8)), so each h2 unit is the same 8 chains and the same
// sum tree as the step loop's packed chains, bit for bit. Lane l of a tile holds row
// m = l & 15 and chain slot j = l >> 4 (k = r + 32 h + 8 j for MFMA half h); layer 1 is
// computed straight into that operand layout. Then lane per row: heads (chunk_heads'
// butterfly tree), sample, log-prob, entropy, stores. Beside the tiles, one wave runs the
// bootstrap forward (lane per unit, as the step loop) and one the episode-return scan
// (records only); the fused returns follow the last pass. The two step-order chains run on
// one lane from LDS with the per-step terms precomputed lane-parallel (same operations,
// same order as xo_gae / xo_nstep and the step loop).
constexpr int kRW = 8;                // waves per env: 16-row tiles per pass
constexpr int kRRows = 16 * kRW;      // rows per pass (T = 128: one pass)
// the chunk pass takes waves 0 and 1; in the last pass waves 2 and 3 run the bootstrap
// forward and the episode-return chain after their tiles, before the tile barrier
constexpr int kBootW = 2, kScanW = 3;
// the fused returns after the last pass: a wave with no global stores of its own in flight
// (a loop head waits for every outstanding vector-memory op of its wave)
constexpr int kRetW = 4;

typedef float rf32x4 __attribute__((ext_vector_type(4)));
#define XA_STR_(x) #x
#define XA_UNROLL(n) _Pragma(XA_STR_(unroll n))
#ifndef XA_RNT_UNROLL
#define XA_RNT_UNROLL 1  // output-column tiles of W2 in flight per tile wave
#endif
#ifndef XA_RHEADS_UNROLL
#define XA_RHEADS_UNROLL 4
#endif

#ifdef XA_STAMPS
// (diagnostic) lane 0 of block 0's wave: cycles since the wave start into slot
#define XA_WSTAMP(slot)                                                              \
  do {                                                                               \
    if (blockIdx.x == 0 && lane == 0) {                                              \
      unsigned long long t_;                                                         \
      __builtin_amdgcn_sched_barrier(0);                                             \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
      __builtin_amdgcn_sched_barrier(0);                                             \
      xa_stamp_acc[slot] += t_ - xa_w0_;                                             \
    }                                                                                \
  } while (0)
#else
#define XA_WSTAMP(slot) \
  do {                  \
  } while (0)
#endif

// xa_tanhf on two values with packed f32 ops: every lane of every op rounds exactly as the
// scalar sequence does
XA_DEV xa_f2 xa_tanhf2(xa_f2 x) {
  const float c = 7.90531110763549805f;
  const xa_f2 xc = {fminf(fmaxf(x.x, -c), c), fminf(fmaxf(x.y, -c), c)};
  const xa_f2 x2 = xc * xc;
  auto k2 = [](float v) { return xa_f2{v, v}; };
  xa_f2 p = xa_fma2(x2, k2(-2.76076847742355e-16f), k2(2.00018790482477e-13f));
  p = xa_fma2(x2, p, k2(-8.60467152213735e-11f));
  p = xa_fma2(x2, p, k2(5.12229709037114e-08f));
  p = xa_fma2(x2, p, k2(1.48572235717979e-05f));
  p = xa_fma2(x2, p, k2(6.37261928875436e-04f));
  p = xa_fma2(x2, p, k2(4.89352455891786e-03f));
  p = xc * p;
  xa_f2 q = xa_fma2(x2, k2(1.19825839466702e-06f), k2(1.18534705686654e-04f));
  q = xa_fma2(x2, q, k2(2.26843463243900e-03f));
  q = xa_fma2(x2, q, k2(4.89352518554385e-03f));
  xa_f2 r = {__int_as_float(0x7EF311C3 - __float_as_int(q.x)),
             __int_as_float(0x7EF311C3 - __float_as_int(q.y))};
  r = xa_fma2(r, xa_fma2(-q, r, k2(1.0f)), r);
  r = xa_fma2(r, xa_fma2(-q, r, k2(1.0f)), r);
  const xa_f2 t = p * r;
  return xa_fma2(r, xa_fma2(-q, t, p), t);
}

// record index of step t (the cursor wraps at t_rec)
XA_DEV size_t replay_rec(const XaRolloutArgs& p, int env, int cur0, int t) {
  return (size_t)env * p.t_rec + (size_t)(((uint32_t)cur0 + (uint32_t)t) % (uint32_t)p.t_rec);
}

// policy input of step t (0 <= t < T); t = T: the bootstrap input
template <int OBS>
XA_DEV const float* replay_input(const XaRolloutArgs& p, int env, int cur0, int t, int T) {
  if (t == 0) return p.env_state + (size_t)env * OBS;
  const size_t base = replay_rec(p, env, cur0, t - 1) * OBS;
  return (t >= T ? p.rep_state : p.rep_obs) + base;
}

// a chunk-pass row's inputs, fetched a pass ahead
template <int OBS>
struct ReplayRow {
  float r, d, u, x[OBS];
  XA_DEV void load(const XaRolloutArgs& p, int env, int cur0, int t, int T, uint64_t ctr) {
    const int tc = min(t, T - 1);
    const size_t rb = replay_rec(p, env, cur0, tc);
    r = p.rep_rew[rb];
    d = p.rep_done[rb];
    if (p.uniforms) {
      u = p.uniforms[(size_t)env * T + tc];
    } else {
      const xa_u4 rr = xa_philox((uint32_t)env, (uint32_t)tc, (uint32_t)ctr, (uint32_t)(ctr >> 32),
                                 (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
      u = xa_u01(rr.x);
    }
    const float* xin = replay_input<OBS>(p, env, cur0, tc, T);
#pragma unroll
    for (int k = 0; k < OBS; ++k) x[k] = xin[k];
  }
};

// The step-order chains: lane q holds step b0 + q of a 64-step block; lane 0 walks the
// block with v_readlane (constant lane indices on a whole block), so a step is two dependent
// VALU ops on lane 0's register and the per-step operands come from SGPRs; the results go
// to LDS row o (o[q] = the value after step q), read back lane-parallel.
// episode returns (a2c/agent.py:119-126): ep += r_q, o_q = ep, ep = +0 after a done (km_q =
// d_q != 0 ? 0 : ~0, so the reset is one AND)
XA_DEV void epret_block(float r, int km, int n, float* __restrict__ o, float& ep) {
  if (n == 64) {
#pragma unroll
    for (int q0 = 0; q0 < 64; q0 += 8) {
      float r8[8];
      int k8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // 8 steps' operands read ahead of their chain
        r8[e] = xa_readlane(r, q0 + e);
        k8[e] = __builtin_amdgcn_readlane(km, q0 + e);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sm = ep + r8[e];
        o[q0 + e] = sm;
        ep = __int_as_float(__float_as_int(sm) & k8[e]);
      }
    }
  } else {
    for (int q = 0; q < n; ++q) {
      const float sm = ep + xa_readlane(r, q);
      o[q] = sm;
      ep = __int_as_float(__float_as_int(sm) & __builtin_amdgcn_readlane(km, q));
    }
  }
}

// returns backwards over a block (xo_gae / xo_nstep): GAE carry = a_q + c_q carry with
// a = delta, c = gamma lambda (1 - d); n-step carry = a_q + (gamma carry) c_q with a = r,
// c = 1 - d. o[q] = the carry after step q.
template <bool GAE>
XA_DEV float returns_op(float aq, float cq, float gamma, float carry) {
  return GAE ? aq + (cq * carry) : aq + (gamma * carry) * cq;
}

template <bool GAE>
XA_DEV void returns_block(float a, float c, int n, float gamma, float* __restrict__ o,
                          float& carry) {
  if (n == 64) {
#pragma unroll
    for (int q0 = 63; q0 >= 0; q0 -= 8) {
      float a8[8], c8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // 8 steps' operands read ahead of their chain
        a8[e] = xa_readlane(a, q0 - e);
        c8[e] = xa_readlane(c, q0 - e);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        carry = returns_op<GAE>(a8[e], c8[e], gamma, carry);
        o[q0 - e] = carry;
      }
    }
  } else {
    for (int q = n - 1; q >= 0; --q) {
      carry = returns_op<GAE>(xa_readlane(a, q), xa_readlane(c, q), gamma, carry);
      o[q] = carry;
    }
  }
}

// returns_block's full-block form with the per-step terms staged in LDS rows sa / sc (written
// lane-parallel): lane 0 reads them 4 steps per 16-B broadcast read, two groups ahead of the
// chain, so a step is its two dependent VALU ops with no v_readlane beside them; the carries
// leave 4 per 16-B store. Same operations, same order as returns_block.
template <bool GAE>
XA_DEV void returns_block64_lds(const float* __restrict__ sa, const float* __restrict__ sc,
                                float gamma, float* __restrict__ o, float& carry) {
  const float4* a4 = reinterpret_cast<const float4*>(sa);
  const float4* c4 = reinterpret_cast<const float4*>(sc);
  float4 a_n = a4[15], c_n = c4[15], a_nn = a4[14], c_nn = c4[14];
#pragma unroll
  for (int g = 15; g >= 0; --g) {
    const float4 a = a_n, c = c_n;
    a_n = a_nn;
    c_n = c_nn;
    if (g >= 2) {
      a_nn = a4[g - 2];
      c_nn = c4[g - 2];
    }
    float4 r;
    carry = returns_op<GAE>(a.w, c.w, gamma, carry);
    r.w = carry;
    carry = returns_op<GAE>(a.z, c.z, gamma, carry);
    r.z = carry;
    carry = returns_op<GAE>(a.y, c.y, gamma, carry);
    r.y = carry;
    carry = returns_op<GAE>(a.x, c.x, gamma, carry);
    r.x = carry;
    reinterpret_cast<float4*>(o)[g] = r;
  }
}

template <int OBS, int A>
__global__ __launch_bounds__(64 * kRW) void replay_rollout_kernel(XaRolloutArgs p) {
  constexpr int AH = A + 1, AHP = (AH + 3) & ~3;
  constexpr int W1S = (OBS + 1 + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float hb[kRRows * kHS];  // h2 rows of one pass
  __shared__ __attribute__((aligned(16))) float wtab[H * AHP];     // (W3[j][.], w4[j], pad)
  // weights in the tile's operand order: layer-1 unit k = r + 32 h + 8 js of operand
  // q = 2 r + h as [q][js][W1[0..OBS) b1 pad] (the 16 lanes of one js read the same row),
  // the W2 fragments as [nt][q][lane] (B[slot js][col 16 nt + mr])
  __shared__ __attribute__((aligned(16))) float sw1[16 * 4 * W1S];
  __shared__ __attribute__((aligned(16))) float sw2[4 * 16 * 64];
  __shared__ __attribute__((aligned(16))) float sx[64], sy[64];  // bootstrap h1 / h2 rows
  __shared__ __attribute__((aligned(16))) float sep[64], sret[64];  // chain result rows
  __shared__ __attribute__((aligned(16))) float sra[64], src[64];    // the returns' step terms
  __shared__ float s_vnext;
  extern __shared__ __attribute__((aligned(16))) float hist[];  // fused: (rew, val, done, .)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int env = blockIdx.x;
  const int T = p.n_steps;
  const int mr = lane & 15, js = lane >> 4;
  const bool fused = p.ret_out != nullptr && p.return_kind != XA_RETURNS_NONE;
  const ParamOffsets o = param_offsets(OBS, A);
  const float* __restrict__ th = p.theta;
  XA_STAMP_DECL
  XA_STAMP(15);
#ifdef XA_STAMPS
  // (diagnostic) every wave's arrival at the first tile barrier, from its own start
  unsigned long long xa_w0_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(xa_w0_)::"memory");
#endif

  // ---- prologue: every load the first pass needs is issued before the barrier
  const int cur0 = p.env_cursor[env];
  const uint64_t ctr = p.rng_counter ? *p.rng_counter : 0ull;
  for (int e = threadIdx.x; e < 4 * 16 * 64; e += 64 * kRW) {
    const int l = e & 63, q = (e >> 6) & 15, nt = e >> 10;
    const int k = (q >> 1) + 32 * (q & 1) + 8 * (l >> 4);
    sw2[e] = th[o.w2 + k * H + 16 * nt + (l & 15)];
  }
  for (int e = threadIdx.x; e < 16 * 4 * W1S; e += 64 * kRW) {
    const int i = e % W1S, jq = e / W1S, q = jq >> 2;
    const int k = (q >> 1) + 32 * (q & 1) + 8 * (jq & 3);
    sw1[e] = i < OBS ? th[o.w1 + i * H + k] : i == OBS ? th[o.b1 + k] : 0.0f;
  }
  if (w == kBootW) {
    float* wr = wtab + lane * AHP;
#pragma unroll
    for (int a = 0; a < AHP; ++a)
      wr[a] = a < A ? th[o.w3 + lane * A + a] : a == A ? th[o.w4 + lane] : 0.0f;
  }
  if (threadIdx.x == 0) p.done_out[(size_t)env * (T + 1)] = p.env_done[env];
  float b2[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) b2[nt] = th[o.b2 + 16 * nt + mr];
  float xt[OBS];  // this lane's tile row input, a pass ahead
  {
    const float* xin = replay_input<OBS>(p, env, cur0, min(16 * w + mr, T - 1), T);
#pragma unroll
    for (int i = 0; i < OBS; ++i) xt[i] = xin[i];
  }
  ReplayRow<OBS> row;  // chunk-pass waves: this lane's row, a pass ahead
  if (w < kRRows / 64) row.load(p, env, cur0, 64 * w + lane, T, ctr);
  // bootstrap wave: s_T and this unit's layer-1 / layer-2 constants; return wave: the
  // records of the first 128 steps and the carried return
  float bx[OBS], bw1[OBS], bb1 = 0.0f, bb2 = 0.0f;
  float sr[2] = {0.0f, 0.0f}, sd[2] = {-1.0f, -1.0f}, ep0 = 0.0f;
  if (w == kBootW) {
    const float* st = replay_input<OBS>(p, env, cur0, T, T);
#pragma unroll
    for (int i = 0; i < OBS; ++i) {
      bx[i] = st[i];
      bw1[i] = th[o.w1 + i * H + lane];
    }
    bb1 = th[o.b1 + lane];
    bb2 = th[o.b2 + lane];
  } else if (w == kScanW) {
    ep0 = p.ep_return[env];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int t = 64 * b + lane;
      const size_t rb = replay_rec(p, env, cur0, min(t, T - 1));
      sr[b] = p.rep_rew[rb];
      sd[b] = t < T ? p.rep_done[rb] : -1.0f;  // -1: past the last step
    }
  }
  __syncthreads();  // weights staged; every read of the env's carried state is done
  XA_STAMP(8);

  if (w == kBootW) {  // the env's carried state: every read of it is behind the barrier
#pragma unroll
    for (int i = 0; i < OBS; ++i)
      if (lane == i) p.env_state[(size_t)env * OBS + i] = bx[i];
    if (lane == 0) p.env_cursor[env] = (int)(((uint32_t)cur0 + (uint32_t)T) % (uint32_t)p.t_rec);
  }

  // episode returns in step order (a2c/agent.py:119-126), from the records alone, one 64-step
  // block at a time with the next block's records in flight; the return wave runs the first
  // half of the blocks after its last tile (beside the other waves' tiles) and the rest
  // beside the last chunk pass
  float sc_ep = ep0, sc_dl = 0.0f;
  int sc_b0 = 0;
  auto scan_blocks = [&](int until_block) {
    for (; sc_b0 < T && sc_b0 < 64 * until_block; sc_b0 += 64) {
      const int b0 = sc_b0;
      const float r = sr[0], d = sd[0];
      sr[0] = sr[1];
      sd[0] = sd[1];
      if (b0 + 128 < T) {
        const int t = b0 + 128 + lane;
        const size_t rb = replay_rec(p, env, cur0, min(t, T - 1));
        sr[1] = p.rep_rew[rb];
        sd[1] = t < T ? p.rep_done[rb] : -1.0f;
      }
      const int nv = min(64, T - b0);
      sc_dl = xa_readlane(d, nv - 1);
      // every lane's operands: the asm pins them here, in all lanes (the compiler would
      // otherwise sink them into the lane-0 branch, and the readlanes read other lanes)
      int km = d != 0.0f ? 0 : -1;
      float rv = r;
      asm volatile("" : "+v"(km), "+v"(rv));
      if (lane == 0) epret_block(rv, km, nv, sep, sc_ep);
      wave_sync();
      if (p.epret_out && b0 + lane < T) p.epret_out[(size_t)env * T + b0 + lane] = sep[lane];
      wave_sync();  // the next block rewrites the row
    }
    if (sc_b0 >= T && lane == 0) {
      p.ep_return[env] = sc_ep;
      p.env_done[env] = sc_dl;
    }
  };

  for (int c0 = 0; c0 < T; c0 += kRRows) {
    const int nr = min(kRRows, T - c0);
    if (16 * w < nr) {  // tile w of the pass: rows c0 + 16 w + m
      float h1[16];
#pragma unroll
      for (int q = 0; q < 16; q += 2) {
        float zz[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float* wr = sw1 + ((q + e) * 4 + js) * W1S;
          float wv[W1S];
#pragma unroll
          for (int i4 = 0; i4 < W1S; i4 += 4) {
            const float4 t4 = *reinterpret_cast<const float4*>(wr + i4);
            wv[i4] = t4.x; wv[i4 + 1] = t4.y; wv[i4 + 2] = t4.z; wv[i4 + 3] = t4.w;
          }
          float z = 0.0f;
#pragma unroll
          for (int i = 0; i < OBS; ++i) z = fmaf(xt[i], wv[i], z);
          zz[e] = z + wv[OBS];
        }
        const xa_f2 h = xa_tanhf2(xa_f2{zz[0], zz[1]});
        h1[q] = h.x;
        h1[q + 1] = h.y;
      }
      if (c0 + kRRows < T) {  // the next pass's tile row
        const float* xin =
            replay_input<OBS>(p, env, cur0, min(c0 + kRRows + 16 * w + mr, T - 1), T);
#pragma unroll
        for (int i = 0; i < OBS; ++i) xt[i] = xin[i];
      }
      XA_UNROLL(XA_RNT_UNROLL)
      for (int nt = 0; nt < 4; ++nt) {
        float wb[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) wb[q] = sw2[(nt * 16 + q) * 64 + lane];
        rf32x4 acc[8];
#pragma unroll
        for (int r = 0; r < 8; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(h1[2 * r], wb[2 * r],
                                                        rf32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 8; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(h1[2 * r + 1], wb[2 * r + 1], acc[r], 0, 0,
                                                        0);
        float bn = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) bn = nt == u ? b2[u] : bn;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          float s[2];
#pragma unroll
          for (int e = 0; e < 2; ++e)
            s[e] = (((acc[0][i + e] + acc[1][i + e]) + (acc[2][i + e] + acc[3][i + e])) +
                    ((acc[4][i + e] + acc[5][i + e]) + (acc[6][i + e] + acc[7][i + e]))) + bn;
          const xa_f2 h = xa_tanhf2(xa_f2{s[0], s[1]});
          hb[(16 * w + 4 * js + i) * kHS + 16 * nt + mr] = h.x;
          hb[(16 * w + 4 * js + i + 1) * kHS + 16 * nt + mr] = h.y;
        }
      }
    }
    // last pass: waves 2 and 3 (done with their tiles, while the second wave of each SIMD
    // still runs its) compute the bootstrap value and the episode returns
    if (c0 + kRRows >= T) {
      if (w == kBootW) {
        XA_WSTAMP(54);
        // bootstrap V(s_T): the step loop's lane-per-unit forward (layer1 / layer2 order), the
        // value head by chunk_heads on the h2 row
        float z1 = 0.0f;
#pragma unroll
        for (int i = 0; i < OBS; ++i) z1 = fmaf(bx[i], bw1[i], z1);
        sx[lane] = xa_tanhf(z1 + bb1);
        wave_sync();
        const int nt = lane >> 4, ml = lane & 15;
        float c[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < H; ++k) {  // W2[k][lane] from the fragment table
          const int q = 2 * (k & 7) + (k >> 5), l = 16 * ((k >> 3) & 3) + ml;
          c[k & 7] = fmaf(sx[k], sw2[(nt * 16 + q) * 64 + l], c[k & 7]);
        }
        sy[lane] = xa_tanhf((((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]))) +
                               bb2);
        wave_sync();
        if (lane == 0) {
          float z[AH];
          chunk_heads<A, A, 2>(sy, wtab, z);
          const float vn = z[A] + th[o.b4];
          p.next_val[env] = vn;
          s_vnext = vn;
        }
        XA_WSTAMP(55);
      } else if (w == kScanW) {
        scan_blocks(((T + 63) / 64 + 1) / 2);  // the first half of the 64-step blocks
      }
    }
    XA_STAMP(9);  // tiles (+ wave 0 has nothing else before the barrier)
#ifdef XA_STAMPS
    if (c0 == 0 && blockIdx.x == 0 && lane == 0) {
      unsigned long long t_;
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      xa_stamp_acc[32 + w] += t_ - xa_w0_;
    }
#endif
    __syncthreads();  // the pass's h2 rows are in LDS
    XA_STAMP(10);
    const int rl = 64 * w + lane, t = c0 + rl;
    if (w < kRRows / 64 && rl < nr) {
      float z[AH];
      chunk_heads<A, 0, XA_RHEADS_UNROLL>(hb + rl * kHS, wtab, z);
      const size_t it = (size_t)env * T + t;
      float l[A];
#pragma unroll
      for (int a = 0; a < A; ++a) l[a] = z[a] + th[o.b3 + a];
      const float val = z[A] + th[o.b4];
      const CatOut<A> cat = categorical<A>(l, row.u, -1);
#pragma unroll
      for (int k = 0; k < OBS; ++k) p.obs_out[it * OBS + k] = row.x[k];
      p.act_out[it] = cat.action;
      p.logp_out[it] = cat.logp;
      p.val_out[it] = val;
      if (p.ent_out) p.ent_out[it] = cat.entropy;
      p.rew_out[it] = row.r;
      p.done_out[(size_t)env * (T + 1) + 1 + t] = row.d;
      if (fused) *reinterpret_cast<float4*>(hist + 4 * t) = float4{row.r, val, row.d, 0.0f};
      if (c0 + kRRows < T) row.load(p, env, cur0, t + kRRows, T, ctr);
    } else if (w == kScanW && c0 + kRRows >= T) {
      scan_blocks((T + 63) / 64);  // the rest of the blocks
    }
    XA_STAMP(11);  // chunk pass
    __syncthreads();  // the next pass rewrites hb; the last pass's values are in LDS
    XA_STAMP(12);
  }

  if (w == kRetW) {
    XA_WSTAMP(56);
    if (fused) {
      // returns (xo_gae / xo_nstep order), backwards one 64-step block at a time: the terms
      // that do not depend on the carry lane-parallel, the carry chain on lane 0
      const bool gae = p.return_kind == XA_RETURNS_GAE;
      float carry = gae ? 0.0f : s_vnext;
      XA_WSTAMP(57);
      for (int b0 = (T - 1) & ~63; b0 >= 0; b0 -= 64) {
        const int t = b0 + lane, tc = min(t, T - 1), nb = min(64, T - b0);
        const float4 hv = *reinterpret_cast<const float4*>(hist + 4 * tc);
        const float nnt = 1.0f - hv.z;
        if (gae) {
          const float vn = tc + 1 < T ? hist[4 * (tc + 1) + 1] : s_vnext;
          float delta = (hv.x + (p.gamma * vn) * nnt) - hv.y;
          float coef = p.gamma_lam * nnt;
          asm volatile("" : "+v"(delta), "+v"(coef));  // in all lanes (see the episode returns)
          if (nb == 64) {
            sra[lane] = delta;
            src[lane] = coef;
            wave_sync();
            if (lane == 0) returns_block64_lds<true>(sra, src, p.gamma, sret, carry);
          } else if (lane == 0) {
            returns_block<true>(delta, coef, nb, p.gamma, sret, carry);
          }
        } else {
          float rr = hv.x, nn = nnt;
          asm volatile("" : "+v"(rr), "+v"(nn));
          if (nb == 64) {
            sra[lane] = rr;
            src[lane] = nn;
            wave_sync();
            if (lane == 0) returns_block64_lds<false>(sra, src, p.gamma, sret, carry);
          } else if (lane == 0) {
            returns_block<false>(rr, nn, nb, p.gamma, sret, carry);
          }
        }
        wave_sync();
        if (t < T) p.ret_out[(size_t)env * T + t] = gae ? sret[lane] + hv.y : sret[lane];
        wave_sync();  // the next block rewrites the row
      }
      XA_WSTAMP(58);
      XA_WSTAMP(59);
    }
  }
  XA_STAMP(14);  // state + returns
}

template <int OBS, int A>
int launch_rollout(const XaRolloutArgs* p, hipStream_t s) {
  const bool fused = p->ret_out != nullptr && p->return_kind != XA_RETURNS_NONE;
  if (p->env_kind == XA_ENV_REPLAY) {
    const size_t lds = fused ? (size_t)4 * p->n_steps * sizeof(float) : 0;
    hipLaunchKernelGGL((replay_rollout_kernel<OBS, A>), dim3(p->n_envs), dim3(64 * kRW), lds, s,
                       *p);
    XA_CHECK_LAUNCH("xa_mlp_rollout");
    return 0;
  }
  const size_t lds = (size_t)kRollWaves * H * sizeof(float) +
                     (fused ? (size_t)kRollWaves * 3 * p->n_steps * sizeof(float) : 0);
  dim3 grid((p->n_envs + kRollWaves - 1) / kRollWaves);
  if constexpr (OBS == 4 && A == 2)
    hipLaunchKernelGGL((mlp_rollout_kernel<OBS, A>), grid, dim3(64 * kRollWaves), lds, s, *p);
  XA_CHECK_LAUNCH("xa_mlp_rollout");
  return 0;
}

template <int OBS, int A>
int launch_forward(const float* theta, const float* obs, int B, const int* ain, const float* u,
                   int* aout, float* logp, float* value, float* ent, float* logits,
                   hipStream_t s) {
  const int blocks = min((B + kWaves - 1) / kWaves, 2048);
  hipLaunchKernelGGL((mlp_forward_kernel<OBS, A>), dim3(blocks), dim3(256), 0, s, theta, obs, B,
                     ain, u, aout, logp, value, ent, logits);
  XA_CHECK_LAUNCH("xa_mlp_forward");
  return 0;
}

#define XA_DISPATCH_OBS_A(OBSV, AV, CALL)                                  \
  if (obs_dim == OBSV && n_actions == AV) return CALL<OBSV, AV>

}  // namespace

extern "C" int xa_mlp_rollout(const XaRolloutArgs* p, void* stream) {
  XA_CHECK_ARG(p != nullptr, "xa_mlp_rollout: null args");
  XA_CHECK_ARG(p->n_envs > 0 && p->n_steps > 0, "xa_mlp_rollout: n_envs, n_steps must be > 0");
  XA_CHECK_ARG(p->theta && p->env_state && p->env_done && p->env_cursor && p->ep_return,
               "xa_mlp_rollout: null env/param pointer");
  XA_CHECK_ARG(p->obs_out && p->act_out && p->logp_out && p->val_out && p->rew_out &&
                   p->done_out && p->next_val,
               "xa_mlp_rollout: null output pointer");
  if (p->env_kind == XA_ENV_REPLAY) {
    XA_CHECK_ARG(p->rep_obs && p->rep_state && p->rep_rew && p->rep_done && p->t_rec > 0,
                 "xa_mlp_rollout: replay env needs rep_obs/rep_state/rep_rew/rep_done/t_rec");
  } else if (p->env_kind == XA_ENV_CARTPOLE) {
    XA_CHECK_ARG(p->env_state64 && p->obs_dim == 4 && p->n_actions == 2 &&
                     p->max_episode_steps > 0,
                 "xa_mlp_rollout: cartpole env needs env_state64, obs_dim 4, 2 actions");
  } else {
    XA_CHECK_ARG(false, "xa_mlp_rollout: unknown env_kind %d", p->env_kind);
  }
  XA_CHECK_ARG(p->ret_out == nullptr || p->return_kind == XA_RETURNS_NONE ||
                   p->n_steps <= kFusedMaxT,
               "xa_mlp_rollout: fused returns need n_steps <= %d (use xa_gae)", kFusedMaxT);
  XA_CHECK_ARG(p->uniforms || p->rng_counter, "xa_mlp_rollout: need uniforms or rng_counter");
  const int obs_dim = p->obs_dim, n_actions = p->n_actions;
  hipStream_t s = (hipStream_t)stream;
  XA_DISPATCH_OBS_A(4, 2, launch_rollout)(p, s);
  XA_DISPATCH_OBS_A(6, 3, launch_rollout)(p, s);
  XA_DISPATCH_OBS_A(8, 4, launch_rollout)(p, s);
  XA_DISPATCH_OBS_A(2, 3, launch_rollout)(p, s);
  xa_set_error("xa_mlp_rollout: unsupported (obs_dim, n_actions) = (%d, %d)", obs_dim, n_actions);
  return -3;
}

extern "C" int xa_mlp_forward(const float* theta, const float* obs, int batch, int obs_dim,
                              int n_actions, const int* actions_in, const float* uniforms,
                              int* actions_out, float* logp, float* value, float* entropy,
                              float* logits, void* stream) {
  XA_CHECK_ARG(theta && obs && batch > 0, "xa_mlp_forward: bad arguments");
  XA_CHECK_ARG(actions_in || uniforms || !actions_out,
               "xa_mlp_forward: sampling needs uniforms");
  hipStream_t s = (hipStream_t)stream;
  XA_DISPATCH_OBS_A(4, 2, launch_forward)(theta, obs, batch, actions_in, uniforms, actions_out,
                                          logp, value, entropy, logits, s);
  XA_DISPATCH_OBS_A(6, 3, launch_forward)(theta, obs, batch, actions_in, uniforms, actions_out,
                                          logp, value, entropy, logits, s);
  XA_DISPATCH_OBS_A(8, 4, launch_forward)(theta, obs, batch, actions_in, uniforms, actions_out,
                                          logp, value, entropy, logits, s);
  XA_DISPATCH_OBS_A(2, 3, launch_forward)(theta, obs, batch, actions_in, uniforms, actions_out,
                                          logp, value, entropy, logits, s);
  xa_set_error("xa_mlp_forward: unsupported (obs_dim, n_actions) = (%d, %d)", obs_dim, n_actions);
  return -3;
}

XA_DIAG_READER(xa_diag_read_stamps_rollout)
